"""The Grid scene's shadow queries on a shadow tree with a Grid cell certificate (round 6).

A triangle scene on the Grid renders its two-pass frames with the wavefront replay; since round 6 its
shadow queries walk a 4-ary tree collapsed from a BVH of the same objects (child boxes widened by
2^-16 of the scene's largest coordinate, drt_upload_grid_shadow_bvh), a hit at t < |L| counts only
when the ray's point at t lies well inside a cell the object is listed in (grid_certificate), and
the queries without a certificate go to the Grid walk (grid_fallback, Grid::Traverse(Ray&),
grid.cpp:309-358).  The answers, hence the frames, are the Grid walk's: every frame here is compared
bit for bit with the same frame on the walk alone (DRT_GRID_SHADOW_TREE=0, grid_stream), and with
every certificate refused (DRT_GRID_TREE_NOCERT=1: each tree hit re-walked on the Grid).  The
whole-frame Grid headline against the oracle (test_gpu_parity.py FULL_SIZE) runs this path too.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def drt():
    import distributionraytracer_amd as d

    return d


@pytest.fixture(scope="module")
def renderer(drt):
    r = drt.Renderer(0)
    yield r
    r.close()


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def grid_scene(drt, first, n_tris, res=(40, 36), spp=16, seed=None, scale=None):
    import bench

    s = drt.Scene()
    c = bench.CAMERA
    s.set_camera(c["eye"], c["at"], c["up"], c["fovy"], c["hither"], res[0], res[1], 0.0, 1.0)
    s.set_background((0.078, 0.361, 0.753))
    s.set_accel("grid")
    s.set_spp(spp)
    quad = ((4, 3, 2), (1, 1, 1), (4, 2, 2), (3, 3, 2), 16)
    if first == "quad":
        s.add_light_quad(*quad)
        s.add_light_point((-3, 1, 5), (1, 1, 1))
    elif first == "point":
        s.add_light_point((-3, 1, 5), (1, 1, 1))
        s.add_light_quad(*quad)
    s.add_material((1, 0.9, 0.7), 0.5, (1, 1, 1), 0.5, 30.0827, 0, 1)
    tris = bench.synthetic_triangles(n_tris) if seed is None else bench.synthetic_triangles(n_tris, seed)
    if scale is not None:
        tris = (np.asarray(tris, np.float32) * np.float32(scale[0]) + np.float32(scale[1])).astype(np.float32)
    s.add_triangles(tris)
    s.build()
    return s


CASES = [
    # (spp, first light, light_spp, max_depth, roughness)
    (16, "quad", 1, 4, 0.0),     # AA, quad light first
    (9, "point", 4, 2, 0.0),     # AA, point first, 4 area samples per quad light
    (0, "quad", 1, 3, 0.0),      # Whitted quad-light frame
    (0, "point", 1, 3, 0.0),     # Whitted point-light frame
    (9, "quad", 1, 3, 0.2),      # in-order glossy frame (MODE_SKEL + wavefront replay)
    (16, "quad", 1, 8, 0.0),     # deep mirror chains
]


@pytest.mark.parametrize("nocert", [False, True])
@pytest.mark.parametrize("spp,first,light_spp,md,rough", CASES)
def test_grid_tree_frame_equals_grid_walk(drt, renderer, monkeypatch, spp, first, light_spp, md, rough, nocert):
    if nocert:
        monkeypatch.setenv("DRT_GRID_TREE_NOCERT", "1")  # read by the upload
    if spp == 0 and first == "point":
        monkeypatch.setenv("DRT_WHITTED_TWO_PASS", "2")
    s = grid_scene(drt, first, 20_000, spp=spp)
    renderer.upload(s)
    kw = {"max_depth": md, "light_spp": light_spp, "roughness": rough}
    plan = renderer.plan(renderer.frame_params(seed=6, **kw))
    assert plan["passes"] == 2 and plan["wavefront"]
    tree = renderer.render(seed=6, **kw)
    monkeypatch.setenv("DRT_GRID_SHADOW_TREE", "0")
    walk = renderer.render(seed=6, **kw)
    np.testing.assert_array_equal(bits(tree), bits(walk))
    # a stats frame on the tree (DRT_GRID_SHADOW_TREE=2): the same frame, samples and shadow queries as
    # the walk's stats frame; the tree took (nearly) every query
    wst_img = renderer.render(seed=6, stats=True, **kw)
    wst = renderer.stats()
    monkeypatch.setenv("DRT_GRID_SHADOW_TREE", "2")
    tst_img = renderer.render(seed=6, stats=True, **kw)
    tst = renderer.stats()
    np.testing.assert_array_equal(bits(tst_img), bits(walk))
    np.testing.assert_array_equal(bits(wst_img), bits(walk))
    assert tst["samples"] == wst["samples"] and tst["shadow_rays"] == wst["shadow_rays"] > 0
    assert tst["wide_shadow_rays"] > 0.95 * tst["shadow_rays"], (tst["wide_shadow_rays"], tst["shadow_rays"])


def test_grid_tree_far_from_origin_and_lightless(drt, renderer, monkeypatch):
    """Scenes whose coordinates are large against their extent (the certificate's margin grows with
    them, K in grid_certificate) and a scene without lights (no query at all)."""
    s = grid_scene(drt, "quad", 8_000, spp=9, seed=3, scale=(3.0, 250.0))
    renderer.upload(s)
    img = renderer.render(seed=2, max_depth=3)
    monkeypatch.setenv("DRT_GRID_SHADOW_TREE", "0")
    np.testing.assert_array_equal(bits(img), bits(renderer.render(seed=2, max_depth=3)))
    monkeypatch.delenv("DRT_GRID_SHADOW_TREE")
    s = grid_scene(drt, "none", 8_000, spp=9)
    renderer.upload(s)
    img = renderer.render(seed=2, max_depth=3)
    monkeypatch.setenv("DRT_GRID_SHADOW_TREE", "0")
    np.testing.assert_array_equal(bits(img), bits(renderer.render(seed=2, max_depth=3)))


def test_grid_tree_headline_scene_equals_grid_walk(drt, renderer, monkeypatch):
    """The 1M-triangle headline scene on the Grid at 512 x 512 x 16 spp: the frame on the tree equals
    the frame on the walk alone bit for bit (the 64-spp frame is checked against the oracle whole in
    test_gpu_parity.py::test_full_size_config_matches_oracle[headline_grid_tri1M_512_64spp])."""
    import types

    import bench

    args = types.SimpleNamespace(scene="synthetic", res=512, spp=16)
    ext = {"aperture": 0.0, "focal": 1.0, "accel": "grid", "ks": 0.5}
    a = bench.make_scene(drt, args, bench.synthetic_triangles(1_000_000, 1), ext)
    a.build()
    renderer.upload(a)
    monkeypatch.setenv("DRT_AA_TWO_PASS", "2")
    tree = renderer.render(seed=7)
    monkeypatch.setenv("DRT_GRID_SHADOW_TREE", "0")
    walk = renderer.render(seed=7)
    np.testing.assert_array_equal(bits(tree), bits(walk))
