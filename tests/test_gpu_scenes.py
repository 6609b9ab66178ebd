"""GPU parity on the reference's shipped scenes (P3D_Scenes/*.p3f, from the data fixture
tests/golden/shipped_scenes.npz) and on BASELINE config C1.

Each scene is loaded by the product's P3F loader and by the oracle's from the same text, with
the same (downsampled) skybox faces, rendered on the HIP path and by the oracle with the same
keyed-RNG seed, and compared per channel within TOL; traversal counts must be identical.
Resolutions are the shipped ones (the oracle finishes each in seconds) except where a case
overrides them.
"""
import numpy as np
import pytest

from tests import shipped
from tests.test_gpu_parity import TOL, assert_default_frame_work, assert_same_work, bits, compare_images

pytestmark = pytest.mark.gpu

# name: (P3F overrides, render kwargs)
SCENE_CASES = {
    # BASELINE.json configs[0] (C1): balls_low, accel none, 256x256, 1 spp — whole frame
    "C1_balls_low_none_256_1spp": ("balls_low", dict(res=(256, 256), spp=1), {}),
    "balls_low_shipped_none_16spp": ("balls_low", {}, {}),
    "balls_low_grid_16spp": ("balls_low", dict(accel="grid"), {}),
    "balls_low_bvh_16spp_C2": ("balls_low", dict(accel="bvh"), {}),
    "dof_none_aperture12": ("dof", {}, {}),
    "dof_bvh_aperture12": ("dof", dict(accel="bvh"), {}),
    "motion_none_spp32_n5": ("motion", {}, {}),
    "teste_none_16spp": ("teste", {}, {}),
    "teste_grid_16spp": ("teste", dict(accel="grid"), {}),
    "balls_box_grid_whitted_sky": ("balls_box", {}, {}),
    "balls_high_grid_whitted_sky": ("balls_high", {}, {}),
    "balls_high_bvh_whitted_sky": ("balls_high", dict(accel="bvh"), {}),
    "blueDiamond_grid_glass_sky": ("blueDiamond", {}, {}),
    "dragon_grid_whitted_sky": ("dragon", {}, {}),
    "assignment1_grid_whitted_sky": ("assignment1", {}, {}),
    "dragon_assignment1_bvh_whitted_sky": ("dragon_assignment1", {}, {}),
    # round 5: AA frames of scenes with glass (trans 1) run as MODE_TCHAIN + MODE_TREPLAY two-pass frames
    # in this suite (DRT_AA_TWO_PASS=2, tests/conftest.py): dragon_assignment1 on the BVH (the tree replay's
    # shadow queries on the shadow tree), assignment1 on the Grid (TREE_CASES below checks the plan);
    # blueDiamond's 178 objects keep the one-pass glass frame (DRT_AA_TWO_PASS_MIN_PRIMS)
    "dragon_assignment1_bvh_aa16_glass": ("dragon_assignment1", dict(res=(256, 256), spp=16), {}),
    "blueDiamond_bvh_aa4_glass": ("blueDiamond", dict(accel="bvh", res=(160, 120), spp=4), {}),
    "assignment1_grid_aa4_glass": ("assignment1", dict(res=(128, 128), spp=4), {}),
    # balls_high has no glass: its AA frame is a mixed-primitive two-pass frame with the wavefront replay
    "balls_high_bvh_aa16_mixed": ("balls_high", dict(accel="bvh", res=(192, 192), spp=16), {}),
}
TREE_CASES = ("dragon_assignment1_bvh_aa16_glass", "assignment1_grid_aa4_glass")


@pytest.fixture(scope="module")
def drt():
    import distributionraytracer_amd as d

    return d


@pytest.fixture(scope="module")
def renderer(drt):
    r = drt.Renderer(0)
    yield r
    r.close()


def load_both(drt, O, tmp_path, name, **over):
    p = shipped.write(tmp_path, name, **over)
    faces = shipped.skybox_faces(name)
    return drt.Scene.load_p3f(p, skybox_faces=faces), O.Scene.load_p3f(p, skybox_faces=faces)


@pytest.mark.parametrize("case", sorted(SCENE_CASES))
def test_shipped_scene_matches_oracle(drt, oracle_mod, renderer, tmp_path, case):
    name, over, kw = SCENE_CASES[case]
    a, b = load_both(drt, oracle_mod, tmp_path, name, **over)
    renderer.upload(a)
    img = renderer.render(seed=2718, stats=True, **kw)
    st = renderer.stats()
    ref, rst = b.render(seed=2718, **kw)
    exact = compare_images(img, ref, TOL)
    assert exact > 0.5, f"only {exact:.3f} of the channels are bit-identical"
    assert_default_frame_work(a.info().accel, st, rst)
    assert st["samples"] == rst["samples"]
    # the reference's traversal order: the same frame bit for bit, the oracle's traversal work
    img_r = renderer.render(seed=2718, stats=True, reference_order=True, **kw)
    np.testing.assert_array_equal(bits(img_r), bits(img))
    assert_same_work(a.info().accel, renderer.stats(), rst)
    if shipped.env(name):  # the sky, not bclr, fills the misses
        assert a.info().skybox_loaded


@pytest.mark.parametrize("case", TREE_CASES + ("balls_high_bvh_aa16_mixed", "blueDiamond_bvh_aa4_glass"))
def test_shipped_aa_frame_plans(drt, renderer, tmp_path, case):
    """The glass cases above take the tree two-pass frame (two passes, no wavefront: the closest hits
    of a refracting scene form a tree, MODE_TCHAIN + MODE_TREPLAY); balls_high's takes the wavefront;
    blueDiamond (178 objects) one pass."""
    name, over, kw = SCENE_CASES[case]
    p = shipped.write(tmp_path, name, **over)
    renderer.upload(drt.Scene.load_p3f(p, skybox_faces=shipped.skybox_faces(name)))
    plan = renderer.plan(renderer.frame_params(seed=2718, **kw))
    assert plan["passes"] == (1 if case.startswith("blueDiamond") else 2)
    assert plan["wavefront"] == (1 if case == "balls_high_bvh_aa16_mixed" else 0)


def test_dragon_assignment1_traversal_count_matches_reference_run(drt, renderer, tmp_path):
    """the reference renders dragon_assignment1 (Whitted, BVH, 512x512) with
    1 436 437 BVH::Traverse calls (closest + shadow).  RNG-independent: it pins the BVH, the
    primitive intersection and rayTracing's branching end to end — here on the HIP path."""
    p = shipped.write(tmp_path, "dragon_assignment1")
    s = drt.Scene.load_p3f(p, skybox_faces=shipped.skybox_faces("dragon_assignment1"))
    renderer.upload(s)
    img = renderer.render(seed=1, stats=True)
    st = renderer.stats()
    assert img.shape == (512, 512, 3)
    assert st["closest_rays"] + st["shadow_rays"] == 1436437
    # Whitted: one sample per pixel (light 0 is punctual)
    assert st["samples"] == 512 * 512
