"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference goldens.

Bars (north_star): identical traversal decisions (closest-hit object, t and normal bit-equal,
shadow occlusion equal, identical ray / node / primitive counts), and images within 1e-5 per
channel of the oracle on identical keyed-RNG seeds.  The only non-bitwise arithmetic is
powf / expf / double pow (ocml vs glibc, <= 1 ulp), hence the image tolerance.
"""
import numpy as np
import pytest

from tests import scenegen as sg
from distributionraytracer_amd.sharding import TileLayout

pytestmark = pytest.mark.gpu

TOL = 1e-5  # per-channel float tolerance (BASELINE.json north_star)


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


def load_both(drt, O, tmp_path, text, name="s.p3f"):
    p = sg.write(tmp_path, name, text)
    return drt.Scene.load_p3f(p), O.Scene.load_p3f(p)


def compare_images(img, ref, tol=TOL):
    assert img.shape == ref.shape
    assert np.isfinite(img).all() == np.isfinite(ref).all()
    d = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    d[~np.isfinite(d)] = 0
    exact = float((img == ref).mean())
    assert d.max() <= tol, f"max |diff| {d.max():.3g} > {tol} (exact fraction {exact:.4f})"
    return exact


def assert_same_work(accel, st, rst):
    """Identical branching => identical traversal work: rays on every accelerator; on the BVH
    inner-node visits, leaf visits and primitive tests (bvh.cpp:245-312); on the Grid the cells
    examined (leaf) and the objects tested in them (grid.cpp:262-273)."""
    if accel == 0:
        return
    assert st["closest_rays"] == rst["closest_calls"] and st["shadow_rays"] == rst["shadow_calls"]
    keys = ("closest_leaf", "shadow_leaf", "closest_prims", "shadow_prims")
    if accel == 2:
        keys += ("closest_inner", "shadow_inner")
    for k in keys:
        assert st[k] == rst[k], (k, st[k], rst[k])


def assert_same_work_frame(renderer, img, rst, seed, **kw):
    """Re-render a frame with the kernel's stats build in the reference's traversal order
    (DRT_FRAME_REFERENCE_ORDER: one pass, every shadow query on the reference's binary tree): the
    same frame bit for bit as `img` (the default frame: AA and in-order BVH frames in two passes,
    their replay pass's shadow queries on the 4-ary shadow tree), and the oracle's traversal work
    (assert_same_work)."""
    img_s = renderer.render(seed=seed, stats=True, reference_order=True, **kw)
    np.testing.assert_array_equal(bits(img_s), bits(img))
    assert_same_work(renderer.scene.info().accel, renderer.stats(), rst)


def assert_default_frame_work(accel, st, rst):
    """A default frame: every ray counted and the closest-hit work equal to the oracle's; shadow
    queries may have walked the 4-ary shadow tree (counted in the wide_* fields)."""
    if accel == 0:
        return
    assert st["closest_rays"] == rst["closest_calls"] and st["shadow_rays"] == rst["shadow_calls"]
    for k in ("closest_leaf", "closest_prims") + (("closest_inner",) if accel == 2 else ()):
        assert st[k] == rst[k], (k, st[k], rst[k])
    if st["wide_shadow_rays"] == 0:
        assert_same_work(accel, st, rst)


GOLD_CASES = ["tiny", "mixed", "tris2k"]


@pytest.mark.parametrize("case", GOLD_CASES)
def test_bvh_traverse_matches_reference_golden(drt, renderer, tmp_path, case):
    from tests.test_oracle_pinning import GOLD

    g = np.load(GOLD / f"ref_{case}.npz")
    p = tmp_path / "s.p3f"
    p.write_bytes(g["scene_text"].tobytes())
    s = drt.Scene.load_p3f(p)
    s.set_accel("bvh")
    renderer.upload(s)
    t, n, obj = renderer.trace_closest(g["rays"])
    np.testing.assert_array_equal(obj, g["bvh_obj"])
    np.testing.assert_array_equal(bits(t), bits(g["bvh_t"]))
    np.testing.assert_array_equal(bits(n), bits(g["bvh_n"]))
    np.testing.assert_array_equal(renderer.trace_shadow(g["shadow_rays"]), g["bvh_occ"])  # 4-ary shadow tree
    renderer.set_trace_stats(True, reference_order=True)
    try:
        np.testing.assert_array_equal(renderer.trace_shadow(g["shadow_rays"]), g["bvh_occ"])  # the reference's tree
        st = renderer.trace_stats()
        assert st["wide_shadow_rays"] == 0 and st["shadow_rays"] == len(g["shadow_rays"])
    finally:
        renderer.set_trace_stats(False)


@pytest.mark.parametrize("case", ["mixed", "tris2k"])
def test_grid_traverse_matches_reference_golden(drt, renderer, tmp_path, case):
    from tests.test_oracle_pinning import GOLD

    g = np.load(GOLD / f"ref_{case}.npz")
    p = tmp_path / "s.p3f"
    p.write_bytes(g["scene_text"].tobytes())
    s = drt.Scene.load_p3f(p)
    s.set_accel("grid")
    renderer.upload(s)
    t, n, obj = renderer.trace_closest(g["grid_rays"])
    np.testing.assert_array_equal(obj, g["grid_obj"])
    np.testing.assert_array_equal(bits(t), bits(g["grid_t"]))
    np.testing.assert_array_equal(bits(n), bits(g["grid_n"]))
    np.testing.assert_array_equal(renderer.trace_shadow(g["grid_rays"]), g["grid_occ"])


def test_none_traverse_matches_oracle(drt, oracle_mod, renderer, tmp_path):
    a, b = load_both(drt, oracle_mod, tmp_path, sg.mixed_scene_text(n_tris=200, accel="none"))
    renderer.upload(a)
    rays = sg.random_rays(3000, seed=9)
    t, n, obj = renderer.trace_closest(rays)
    rt, rn, ro = b.trace_closest(rays)
    np.testing.assert_array_equal(obj, ro)
    np.testing.assert_array_equal(bits(t), bits(rt))
    np.testing.assert_array_equal(bits(n), bits(rn))
    np.testing.assert_array_equal(renderer.trace_shadow(rays), b.trace_shadow(rays))


RENDER_CASES = {
    # name: (scene text, render kwargs)
    "aa_bvh_glass_quad": (lambda: sg.mixed_scene_text(res=(40, 32), spp=4, accel="bvh"), {}),
    "aa_grid_glass_quad": (lambda: sg.mixed_scene_text(res=(40, 32), spp=4, accel="grid"), {}),
    "aa_none_glass_quad": (lambda: sg.mixed_scene_text(res=(40, 32), spp=4, accel="none", n_tris=40), {}),
    "aa_nonsquare_spp": (lambda: sg.mixed_scene_text(res=(24, 24), spp=5, accel="bvh"), {}),
    "whitted_quad_bvh": (lambda: sg.mixed_scene_text(res=(40, 32), spp=0, accel="bvh"), {}),
    "whitted_point_grid": (lambda: sg.mixed_scene_text(res=(40, 32), spp=0, accel="grid", quad=False), {}),
    "dof_bvh": (lambda: sg.mixed_scene_text(res=(32, 24), spp=4, accel="bvh", aperture=8.0, focal=1.5), {}),
    "dof_none": (lambda: sg.mixed_scene_text(res=(32, 24), spp=4, accel="none", n_tris=30, aperture=8.0,
                                             focal=1.5), {}),
    "glossy_ext": (lambda: sg.mixed_scene_text(res=(24, 24), spp=4, accel="bvh"), {"roughness": 0.1}),
    "depth8_ext": (lambda: sg.mixed_scene_text(res=(24, 24), spp=4, accel="bvh"), {"max_depth": 8}),
    "tris_soup_bvh": (lambda: sg.synthetic_scene_text(20000, res=(48, 48), spp=4), {}),
    "edge_image_not_multiple_of_tile": (lambda: sg.mixed_scene_text(res=(37, 19), spp=1, accel="bvh"), {}),
    # light_spp extension: 4 / 3 shadow samples per quad light
    "soft4_bvh": (lambda: sg.mixed_scene_text(res=(32, 24), spp=4, accel="bvh"), {"light_spp": 4}),
    "soft3_grid": (lambda: sg.mixed_scene_text(res=(32, 24), spp=4, accel="grid"), {"light_spp": 3}),
    "soft4_none": (lambda: sg.mixed_scene_text(res=(24, 16), spp=4, accel="none", n_tris=30), {"light_spp": 4}),
    "soft4_whitted": (lambda: sg.mixed_scene_text(res=(32, 24), spp=0, accel="bvh"), {"light_spp": 4}),
    "soft4_dof": (lambda: sg.mixed_scene_text(res=(24, 16), spp=4, accel="bvh", aperture=8.0, focal=1.5),
                  {"light_spp": 4}),
    "c3_tris_soft4": (lambda: sg.synthetic_scene_text(20000, res=(40, 40), spp=4), {"light_spp": 4}),
    # in-order (keyed-stream) modes on the persistent BVH kernel: Whitted with glossy reflection
    "whitted_glossy_quad_bvh": (lambda: sg.mixed_scene_text(res=(24, 16), spp=0, accel="bvh"), {"roughness": 0.2}),
    "whitted_glossy_point_bvh": (lambda: sg.mixed_scene_text(res=(24, 16), spp=0, accel="bvh", quad=False),
                                 {"roughness": 0.2}),
    "dof_glossy_depth8_bvh": (lambda: sg.mixed_scene_text(res=(24, 16), spp=9, accel="bvh", aperture=8.0,
                                                          focal=1.5), {"roughness": 0.1, "max_depth": 8}),
    # oversized BVH leaves (>= 31 objects: count-31 descriptors, count in the first record)
    "big_leaf_bvh": (lambda: sg.mixed_scene_text(res=(32, 24), spp=4, accel="bvh", cluster=40), {}),
    # the per-pixel shuffle prepass at its byte limit (spp 256), and past it (the kernel's own walk)
    "aa_spp256_bvh": (lambda: sg.mixed_scene_text(res=(8, 6), spp=256, accel="bvh", n_tris=60), {}),
    "aa_spp289_bvh": (lambda: sg.mixed_scene_text(res=(6, 5), spp=289, accel="bvh", n_tris=60), {}),
    "dof_spp256_bvh": (lambda: sg.mixed_scene_text(res=(6, 5), spp=256, accel="bvh", n_tris=60, aperture=8.0,
                                                   focal=1.5), {}),
    "big_leaf_dof_bvh": (lambda: sg.mixed_scene_text(res=(24, 16), spp=4, accel="bvh", cluster=40, aperture=8.0,
                                                     focal=1.5), {}),
}


def test_big_leaf_traverse_matches_oracle(drt, oracle_mod, renderer, tmp_path):
    a, b = load_both(drt, oracle_mod, tmp_path, sg.mixed_scene_text(accel="bvh", cluster=40))
    renderer.upload(a)
    rays = sg.random_rays(4000, seed=21)
    rays[: len(rays) // 2, :3] = (-0.5, -0.5, 0.3)  # half start inside the concentric spheres
    t, n, obj = renderer.trace_closest(rays)
    rt, rn, ro = b.trace_closest(rays)
    np.testing.assert_array_equal(obj, ro)
    np.testing.assert_array_equal(bits(t), bits(rt))
    np.testing.assert_array_equal(bits(n), bits(rn))
    np.testing.assert_array_equal(renderer.trace_shadow(rays), b.trace_shadow(rays))


@pytest.mark.parametrize("case", sorted(RENDER_CASES))
def test_render_matches_oracle(drt, oracle_mod, renderer, tmp_path, case):
    mk, kw = RENDER_CASES[case]
    a, b = load_both(drt, oracle_mod, tmp_path, mk())
    renderer.upload(a)
    seed = 12345
    img = renderer.render(seed=seed, stats=True, **kw)
    st = renderer.stats()
    ref, rst = b.render(seed=seed, **kw)
    compare_images(img, ref)
    assert_default_frame_work(a.info().accel, st, rst)
    assert st["samples"] == rst["samples"]
    # the reference's traversal order: the same frame bit for bit, identical traversal work
    img_r = renderer.render(seed=seed, stats=True, reference_order=True, **kw)
    np.testing.assert_array_equal(bits(img_r), bits(img))
    assert_same_work(a.info().accel, renderer.stats(), rst)


@pytest.mark.parametrize("accel,aperture,roughness", [("bvh", 0.0, 0.0), ("bvh", 8.0, 0.2), ("grid", 0.0, 0.0),
                                                     ("none", 8.0, 0.0)])
def test_progressive_matches_oracle(drt, oracle_mod, renderer, tmp_path, accel, aperture, roughness):
    """Zone A (main.cpp:536-599): three progressive frames, each lerped into the running buffer."""
    a, b = load_both(drt, oracle_mod, tmp_path,
                     sg.mixed_scene_text(res=(24, 16), spp=4, accel=accel, aperture=aperture, focal=1.5, n_tris=60))
    renderer.upload(a)
    acc_g = np.zeros((16, 24, 3), np.float32)
    acc_o = np.zeros((16, 24, 3), np.float32)
    for n in (1, 2, 3):
        renderer.render(seed=40 + n, roughness=roughness, progressive_frame=n, accum=acc_g, stats=True)
        st = renderer.stats()
        _, rst = b.render(seed=40 + n, roughness=roughness, progressive_frame=n, accum=acc_o)
        compare_images(acc_g, acc_o)
        assert st["samples"] == rst["samples"] == 24 * 16
        assert_same_work(a.info().accel, st, rst)
    before = acc_g.copy()
    renderer.render(seed=9, progressive_frame=10000, accum=acc_g)  # MAX_SAMPLES: untouched
    np.testing.assert_array_equal(acc_g, before)


@pytest.mark.parametrize("accel,aperture", [("bvh", 8.0), ("grid", 0.0)])
def test_camera_orbit_without_reupload(drt, oracle_mod, renderer, tmp_path, accel, aperture):
    """The interactive renderer moves the camera every frame (SetEye, main.cpp:530-533) and
    renders zone A (main.cpp:536-599).  drt_set_camera replaces the camera alone — the primitives
    and the accelerator stay resident — and an orbit of progressive frames equals the same orbit
    rendered with a fresh full upload per frame, bit for bit, and the oracle's orbit within TOL.
    A zone-B frame after the orbit equals a fresh upload's too."""
    a, b = load_both(drt, oracle_mod, tmp_path, sg.mixed_scene_text(res=(32, 24), spp=4, accel=accel, n_tris=60,
                                                                     aperture=aperture, focal=1.5))
    renderer.upload(a)
    fresh = drt.Renderer(0)
    e0 = np.array(a.camera_frame().eye, np.float64)
    acc_g, acc_f, acc_o = (np.zeros((24, 32, 3), np.float32) for _ in range(3))
    for n in range(1, 5):
        ang = 0.15 * n
        eye = np.array([e0[0] * np.cos(ang) - e0[1] * np.sin(ang), e0[0] * np.sin(ang) + e0[1] * np.cos(ang),
                        e0[2] + 0.05 * n])
        a.set_eye(eye)
        b.set_eye(eye)
        renderer.set_camera(a)
        renderer.render(seed=60 + n, progressive_frame=n, accum=acc_g)
        fresh.upload(a)
        fresh.render(seed=60 + n, progressive_frame=n, accum=acc_f)
        b.render(seed=60 + n, progressive_frame=n, accum=acc_o)
        np.testing.assert_array_equal(bits(acc_g), bits(acc_f), err_msg=f"frame {n}")
        compare_images(acc_g, acc_o)
    np.testing.assert_array_equal(bits(renderer.render(seed=9)), bits(fresh.render(seed=9)))
    ref, _ = b.render(seed=9)
    compare_images(renderer.render(seed=9), ref)
    fresh.close()


def test_set_camera_refuses_a_new_resolution(drt, renderer, tmp_path):
    """Camera::SetEye keeps the resolution (camera.h:63-72) and the caller's frame buffers are sized
    by the resident one: drt_set_camera (and drt_group_set_camera, validated on every device before
    any changes) refuses a camera of another resolution and leaves the resident camera in place."""
    a = drt.Scene.load_p3f(sg.write(tmp_path, "a.p3f", sg.mixed_scene_text(res=(32, 24), spp=1, n_tris=40)))
    big = drt.Scene.load_p3f(sg.write(tmp_path, "b.p3f", sg.mixed_scene_text(res=(64, 48), spp=1, n_tris=40)))
    renderer.upload(a)
    before = renderer.render(seed=3)
    with pytest.raises(RuntimeError, match="DRT_E_INVALID"):
        renderer.set_camera(big)
    np.testing.assert_array_equal(bits(renderer.render(seed=3)), bits(before))
    g = drt.RendererGroup([0])
    g.upload(a)
    with pytest.raises(RuntimeError, match="DRT_E_INVALID"):
        g.set_camera(big)
    np.testing.assert_array_equal(bits(g.render(seed=3)), bits(before))
    g.close()


def test_set_camera_host_overhead_at_1M_triangles(drt, renderer):
    """Per-frame host cost of the interactive camera at the headline size: drt_set_camera (the
    camera alone) against a full upload (1M primitive records packed and copied, BVH re-uploaded),
    and the frame after it equals a fresh upload's."""
    import time

    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(1_000_000), 128, 1)
    s.build()
    renderer.upload(s)
    t0 = time.perf_counter()
    renderer.upload(s)
    full_ms = (time.perf_counter() - t0) * 1e3
    e = np.array(s.camera_frame().eye)
    cam_ms = []
    for k in range(20):
        s.set_eye(e + 0.01 * (k + 1))
        t0 = time.perf_counter()
        renderer.set_camera(s)
        cam_ms.append((time.perf_counter() - t0) * 1e3)
    moved = renderer.render(seed=2)
    renderer.upload(s)
    np.testing.assert_array_equal(bits(moved), bits(renderer.render(seed=2)))
    print(f"\n[camera] full upload {full_ms:.1f} ms, set_camera median {np.median(cam_ms) * 1e3:.1f} us")
    assert np.median(cam_ms) < 1.0 and full_ms > 10 * np.median(cam_ms)


def test_sharded_frame_equals_whole_frame(drt, renderer, tmp_path):
    """Interleaved 16x16 tile shards rendered separately and reassembled == one-shot frame."""
    import torch

    p = sg.write(tmp_path, "s.p3f", sg.mixed_scene_text(res=(70, 45), spp=4, accel="bvh"))
    s = drt.Scene.load_p3f(p)
    renderer.upload(s)
    whole = renderer.render(seed=7)
    for n_shards in (2, 3, 8):
        p0 = renderer.frame_params(seed=7, shard=0, n_shards=n_shards)
        layout = TileLayout(70, 45, 16, n_shards)
        tiles, floats = renderer.shard_layout(p0)
        assert (tiles, floats) == (len(layout.tiles_of(0)), layout.floats_per_shard)
        bufs = torch.zeros((n_shards, floats), dtype=torch.float32, device="cuda")
        for r in range(n_shards):
            renderer.render_device(renderer.frame_params(seed=7, shard=r, n_shards=n_shards), bufs[r].data_ptr())
        frame = torch.zeros(whole.shape, dtype=torch.float32, device="cuda")
        renderer.unshard_device(p0, bufs.data_ptr(), frame.data_ptr())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(frame.cpu().numpy().view(np.uint32), whole.view(np.uint32))
        # the device shard buffers follow the host layout of distributionraytracer_amd.sharding
        host = bufs.cpu().numpy()
        for r in range(n_shards):
            np.testing.assert_array_equal(host[r].view(np.uint32), layout.pack_host(whole, r).view(np.uint32))


def test_reference_scene_balls_low_bvh(drt, oracle_mod, renderer, tmp_path):
    """SURVEY §8d config 2 geometry (balls_low with accel bvh, 16 spp) at reduced resolution."""
    text = sg.balls_low_text(res=(96, 96), spp=16, accel="bvh")
    a, b = load_both(drt, oracle_mod, tmp_path, text)
    renderer.upload(a)
    img = renderer.render(seed=99)
    ref, rst = b.render(seed=99)
    compare_images(img, ref)
    assert_same_work_frame(renderer, img, rst, 99)


def test_full_size_frame_properties(drt, renderer, tmp_path):
    """At a production size: deterministic re-render, finite, colours clamped to [0, 1]."""
    p = sg.write(tmp_path, "s.p3f", sg.synthetic_scene_text(100_000, res=(256, 256), spp=16))
    s = drt.Scene.load_p3f(p)
    renderer.upload(s)
    a = renderer.render(seed=3)
    b = renderer.render(seed=3)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.isfinite(a).all() and a.min() >= 0.0 and a.max() <= 1.0
    c = renderer.render(seed=4)
    assert (a != c).any()


def test_trace_device_streaming_matches_reference_golden(drt, renderer, tmp_path):
    """drt_trace_device (device buffers, streaming traversal kernel, several 256-query wave
    chunks and a ragged tail) returns the reference's BVH::Traverse results bit for bit."""
    import torch
    from tests.test_oracle_pinning import GOLD

    g = np.load(GOLD / "ref_tris2k.npz")
    p = tmp_path / "s.p3f"
    p.write_bytes(g["scene_text"].tobytes())
    s = drt.Scene.load_p3f(p)
    s.set_accel("bvh")
    renderer.upload(s)
    rays = torch.from_numpy(np.ascontiguousarray(g["rays"], np.float32)).cuda()
    n = rays.shape[0]
    t = torch.empty(n, dtype=torch.float32, device="cuda")
    nrm = torch.empty((n, 3), dtype=torch.float32, device="cuda")
    obj = torch.empty(n, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    renderer.set_trace_stats(True)
    renderer.trace_device(False, rays.data_ptr(), n, t.data_ptr(), nrm.data_ptr(), obj.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    st = renderer.trace_stats()
    renderer.set_trace_stats(False)
    np.testing.assert_array_equal(obj.cpu().numpy(), g["bvh_obj"])
    np.testing.assert_array_equal(bits(t.cpu().numpy()), bits(g["bvh_t"]))
    np.testing.assert_array_equal(bits(nrm.cpu().numpy()), bits(g["bvh_n"]))
    assert st["closest_rays"] == n and st["closest_inner"] > 0 and st["kernel_ms"] > 0
    srays = torch.from_numpy(np.ascontiguousarray(g["shadow_rays"], np.float32)).cuda()
    occ = torch.empty(srays.shape[0], dtype=torch.uint8, device="cuda")
    renderer.trace_device(True, srays.data_ptr(), srays.shape[0], d_occluded=occ.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(occ.cpu().numpy(), g["bvh_occ"])
    # queries issued back to back on two other streams share the context's query records and
    # claim counter: the second waits for the first on the device, both stay exact
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    t2 = torch.empty_like(t)
    obj2 = torch.full_like(obj, -7)
    occ2 = torch.empty_like(occ)
    big = rays.repeat(8, 1)  # a larger query first: the next one must not regrow under it
    tb = torch.empty(big.shape[0], dtype=torch.float32, device="cuda")
    nb = torch.empty((big.shape[0], 3), dtype=torch.float32, device="cuda")
    ob = torch.empty(big.shape[0], dtype=torch.int32, device="cuda")
    renderer.trace_device(False, big.data_ptr(), big.shape[0], tb.data_ptr(), nb.data_ptr(), ob.data_ptr(),
                          stream=s1.cuda_stream)
    renderer.trace_device(True, srays.data_ptr(), srays.shape[0], d_occluded=occ2.data_ptr(), stream=s2.cuda_stream)
    renderer.trace_device(False, rays.data_ptr(), n, t2.data_ptr(), nrm.data_ptr(), obj2.data_ptr(),
                          stream=s1.cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ob.cpu().numpy(), np.tile(g["bvh_obj"], 8))
    np.testing.assert_array_equal(occ2.cpu().numpy(), g["bvh_occ"])
    np.testing.assert_array_equal(obj2.cpu().numpy(), g["bvh_obj"])
    np.testing.assert_array_equal(bits(t2.cpu().numpy()), bits(g["bvh_t"]))


def test_streaming_traverse_many_chunks_matches_oracle(drt, oracle_mod, renderer, tmp_path):
    """60k queries (hundreds of wave chunks) on a 20k-triangle soup: closest and shadow results
    equal the oracle's BVH::Traverse restatement."""
    a, b = load_both(drt, oracle_mod, tmp_path, sg.synthetic_scene_text(20000, res=(8, 8), spp=1))
    renderer.upload(a)
    rays = sg.random_rays(60001, seed=33, origin_box=2.0)
    t, n, obj = renderer.trace_closest(rays)
    rt, rn, ro = b.trace_closest(rays)
    np.testing.assert_array_equal(obj, ro)
    np.testing.assert_array_equal(bits(t), bits(rt))
    np.testing.assert_array_equal(bits(n), bits(rn))
    np.testing.assert_array_equal(renderer.trace_shadow(rays), b.trace_shadow(rays))


# BASELINE.json configs at their full sizes: the GPU renders the whole frame and the oracle (on
# every host core) the WHOLE frame too, except C4, whose 813 M rays take the oracle minutes: there
# it renders 128 rows spread over the same frame — top (sky), middle (objects, glass, mirrors),
# bottom (floor) and both edge rows (its cost is per row; the keyed RNG makes rows independent).
def spread_rows(res, n):
    return sorted(set(np.linspace(0, res - 1, n).round().astype(int).tolist()))


FULL_SIZE = {
    # name: (scene, render kwargs, oracle rows (None = the whole frame))
    "C2_balls_low_bvh_512_16spp": (dict(scene="balls_low", res=512, spp=16), {}, None),
    "C3_tri100k_512_64spp_soft4": (dict(tris=100_000, res=512, spp=64), {"light_spp": 4}, None),
    "headline_tri1M_512_64spp": (dict(tris=1_000_000, res=512, spp=64), {}, None),
    "C4_tri1M_1024_64spp_dof_glossy_depth8": (dict(tris=1_000_000, res=1024, spp=64, aperture=8.0, focal=1.0),
                                              {"roughness": 0.1, "max_depth": 8}, spread_rows(1024, 128)),
    # the headline scene on the uniform grid (f4): 307 x 307 x 85 cells, 93 % empty, so both caps
    # of the Grid stepper (empty-cell walk, object pairs per call) are exercised on every row
    "headline_grid_tri1M_512_64spp": (dict(tris=1_000_000, res=512, spp=64, accel="grid"), {}, None),
}


@pytest.mark.parametrize("case", sorted(FULL_SIZE))
def test_full_size_config_matches_oracle(drt, oracle_mod, renderer, case):
    import types

    import bench

    sk, kw, rows = FULL_SIZE[case]
    args = types.SimpleNamespace(scene=sk.get("scene", "synthetic"), res=sk["res"], spp=sk["spp"])
    ext = {"aperture": sk.get("aperture", 0.0), "focal": sk.get("focal", 1.0), "accel": sk.get("accel", "bvh"), "ks": 0.5}
    tris = bench.synthetic_triangles(sk["tris"], 1) if "tris" in sk else None
    a = bench.make_scene(drt, args, tris, ext)
    a.build()
    renderer.upload(a)
    img = renderer.render(seed=7, **kw)
    b = bench.make_scene(oracle_mod, args, tris, ext)
    b.build()
    thr = oracle_mod.host_threads()
    if rows is None:
        ref, rst = b.render(seed=7, threads=thr, **kw)
        compare_images(img, ref)
        # and the whole frame's traversal work equals the oracle's (the stats build of the kernel)
        assert_same_work_frame(renderer, img, rst, 7, **kw)
        return
    for y in rows:
        ref, _ = b.render(seed=7, rows=(y, y + 1), threads=thr, **kw)
        compare_images(img[y:y + 1], ref[y:y + 1])
    # rows outside the checked set: rendered, finite, clamped
    assert np.isfinite(img).all() and img.min() >= 0.0 and img.max() <= 1.0
    # the checked rows cover sky, objects and floor: not all one colour
    assert len({tuple(np.round(img[y].mean(axis=0), 3)) for y in rows}) > len(rows) // 2


@pytest.mark.parametrize("accel,spp", [("bvh", 4), ("grid", 0), ("none", 4)])
def test_skybox_render_matches_oracle(drt, oracle_mod, renderer, tmp_path, accel, spp):
    """Misses and mirror bounces that leave the scene read the cube map (scene.cpp:380-458):
    six random bottom-up RGB8 faces of different sizes fed to both sides."""
    rng = np.random.default_rng(17)
    faces = [rng.integers(0, 256, size=(12 + 4 * i, 12 + 4 * i, 3), dtype=np.uint8) for i in range(6)]
    text = sg.mixed_scene_text(res=(40, 32), spp=spp, accel=accel, n_tris=60, env="sky")
    p = sg.write(tmp_path, "sky.p3f", text)
    a = drt.Scene.load_p3f(p, skybox_faces=faces)
    b = oracle_mod.Scene.load_p3f(p, skybox_faces=faces)
    renderer.upload(a)
    img = renderer.render(seed=5)
    ref, rst = b.render(seed=5)
    compare_images(img, ref)
    assert_same_work_frame(renderer, img, rst, 5)
    bg = np.array([0.078, 0.361, 0.753], np.float32)
    assert (np.abs(img - bg).max(axis=-1) > 1e-3).mean() > 0.9  # the sky, not bclr, fills the misses


EDGE_CASES = {
    # no objects: every ray misses (root / grid box inverted, NONE scans nothing)
    "empty_bvh": lambda: "\n".join(sg.header(res=(24, 16), spp=4, accel="bvh") + ["light punctual -3 1 5 1 1 1"]) + "\n",
    "empty_grid": lambda: "\n".join(sg.header(res=(24, 16), spp=0, accel="grid") + ["light punctual -3 1 5 1 1 1"]) + "\n",
    "empty_none": lambda: "\n".join(sg.header(res=(24, 16), spp=4, accel="none")) + "\n",
}


@pytest.mark.parametrize("case", sorted(EDGE_CASES))
def test_edge_scene_matches_oracle(drt, oracle_mod, renderer, tmp_path, case):
    a, b = load_both(drt, oracle_mod, tmp_path, EDGE_CASES[case]())
    renderer.upload(a)
    img = renderer.render(seed=3)
    ref, rst = b.render(seed=3)
    compare_images(img, ref)
    assert_same_work_frame(renderer, img, rst, 3)
    np.testing.assert_allclose(img, np.broadcast_to(np.float32([0.078, 0.361, 0.753]), img.shape), atol=1e-6)


def test_no_lights_and_deepest_recursion_match_oracle(drt, oracle_mod, renderer, tmp_path):
    """No lights: secondary rays get lightPos (0,0,0) (Q2) and only reflections/refractions add
    colour; MAX_DEPTH 15 is the deepest call chain the frame stack holds (kMaxFrames - 1)."""
    lines = sg.mixed_scene_text(res=(32, 24), spp=4, accel="bvh", n_tris=80).split("\n")
    text = "\n".join(l for l in lines if not l.startswith("light")) + "\n"
    a, b = load_both(drt, oracle_mod, tmp_path, text)
    renderer.upload(a)
    for kw in ({}, {"max_depth": 15}):
        img = renderer.render(seed=8, **kw)
        ref, rst = b.render(seed=8, **kw)
        compare_images(img, ref)
        assert_same_work_frame(renderer, img, rst, 8, **kw)


@pytest.mark.parametrize("pipe,aux", [(2, "0"), (2, "1"), (4, "1")])
def test_pipelined_slots_match_sequential_frame(drt, renderer, tmp_path, monkeypatch, pipe, aux):
    """Frames in flight (scratch slots 0 .. pipe-1, one stream each, bench.py --frames-in-flight)
    give the frames lone renders give, bit for bit, with and without the auxiliary shuffle /
    reduce streams (DRT_AUX_STREAMS; every frame has its own seed, so a permutation or sample
    buffer reused too early would show); a slot outside DRT_FRAME_SLOTS is refused."""
    import torch

    p = sg.write(tmp_path, "s.p3f", sg.synthetic_scene_text(20000, res=(64, 48), spp=16))
    s = drt.Scene.load_p3f(p)
    renderer.upload(s)
    n = 3 * pipe
    lone = [renderer.render(seed=21 + i) for i in range(n)]
    monkeypatch.setenv("DRT_AUX_STREAMS", aux)
    streams = [torch.cuda.Stream() for _ in range(pipe)]
    outs = [torch.zeros((48, 64, 3), dtype=torch.float32, device="cuda") for _ in range(n)]
    for i in range(n):
        j = i % pipe
        renderer.render_device(renderer.frame_params(seed=21 + i, slot=j), outs[i].data_ptr(), streams[j].cuda_stream)
    torch.cuda.synchronize()
    for i in range(n):
        np.testing.assert_array_equal(outs[i].cpu().numpy().view(np.uint32), lone[i].view(np.uint32))
    with pytest.raises(RuntimeError, match="slot"):
        renderer.render_device(renderer.frame_params(seed=21, slot=4), outs[0].data_ptr(), streams[0].cuda_stream)


@pytest.mark.parametrize("aperture", [0.0, 8.0])
def test_shuffle_prepass_matches_in_kernel_walk(drt, renderer, tmp_path, aperture, monkeypatch):
    """The per-pixel Fisher-Yates prepass (shuffle_kernel) and the kernel's own backward walk over
    the swaps (DRT_PERM=0) give the same frame, bit for bit (AA and in-order DoF frames)."""
    p = sg.write(tmp_path, "s.p3f", sg.mixed_scene_text(res=(40, 24), spp=16, accel="bvh", n_tris=80,
                                                        aperture=aperture, focal=1.5))
    renderer.upload(drt.Scene.load_p3f(p))
    with_perm = renderer.render(seed=5)
    monkeypatch.setenv("DRT_PERM", "0")
    walk = renderer.render(seed=5)
    np.testing.assert_array_equal(with_perm.view(np.uint32), walk.view(np.uint32))



def test_failed_upload_leaves_no_scene(drt, renderer, tmp_path):
    """drt_upload_scene validates the whole descriptor before it commits anything: after a
    rejected upload (bad primitive type, malformed skybox face, bad light type) the context has
    no scene, so a render returns DRT_E_STATE instead of reading the old buffers."""
    import ctypes as C

    from distributionraytracer_amd import _lib

    L = _lib.load()
    p = sg.write(tmp_path, "s.p3f", sg.mixed_scene_text(res=(24, 16), spp=1, accel="bvh", n_tris=20))
    good = drt.Scene.load_p3f(p)
    cam = good.camera_frame()
    cam.res_x, cam.res_y = 640, 480  # a bigger frame than the scene that is resident
    mat = (_lib.DrtMaterial * 1)()
    prim = (_lib.DrtPrim * 1)()
    light = (_lib.DrtLight * 1)()
    prim[0].type, prim[0].material, prim[0].r = 1, 0, 0.5
    variants = {"bad prim type": lambda d: setattr(prim[0], "type", 7),
                "bad light type": lambda d: setattr(light[0], "type", 5),
                "skybox face missing": lambda d: setattr(d, "has_skybox", 1)}
    for what, spoil in variants.items():
        renderer.upload(good)
        renderer.render(seed=1)
        prim[0].type, light[0].type = 1, 0
        d = _lib.DrtSceneDesc()
        d.camera = cam
        d.materials, d.n_materials = mat, 1
        d.prims, d.n_prims = prim, 1
        d.lights, d.n_lights = light, 1
        d.accel, d.spp = 2, 1
        spoil(d)
        rc = L.drt_upload_scene(renderer.h, C.byref(d))
        assert rc == -1, (what, rc)
        out = np.zeros((480, 640, 3), np.float32)
        params = renderer.frame_params(seed=1)
        assert L.drt_render(renderer.h, C.byref(params), out.ctypes.data_as(_lib._f)) == -5, what
        assert not out.any()
    renderer.upload(good)  # a good upload restores the context


def test_frame_plan_routes_huge_frames_to_64bit_kernel(drt, renderer, tmp_path):
    """8192^2 x 64 spp AA is exactly 2^32 work items: the persistent kernel's 32-bit claim
    counters would wrap, so the plan hands the frame to the 64-bit path_kernel."""
    text = sg.mixed_scene_text(res=(8192, 8192), spp=64, accel="bvh", n_tris=20)
    renderer.upload(drt.Scene.load_p3f(sg.write(tmp_path, "big.p3f", text)))
    plan = renderer.plan(renderer.frame_params(seed=1))
    assert plan["work_items"] == 2 ** 32 and plan["sample_slots"] == 2 ** 32 and plan["mode"] == 0
    assert not plan["persistent"]
    small = sg.mixed_scene_text(res=(512, 512), spp=64, accel="bvh", n_tris=20)
    renderer.upload(drt.Scene.load_p3f(sg.write(tmp_path, "small.p3f", small)))
    plan = renderer.plan(renderer.frame_params(seed=1))
    assert plan["work_items"] == 512 * 512 * 64 and plan["persistent"]
    plan = renderer.plan(renderer.frame_params(seed=1, roughness=0.1))  # in-order keyed stream
    assert plan["mode"] == 1 and plan["work_items"] == 512 * 512 and plan["sample_slots"] == 512 * 512 * 64


@pytest.mark.parametrize("walk,pairs", [(1, 1), (2, 3), (64, 1 << 20)])
def test_grid_stepper_caps_do_not_change_the_frame(drt, renderer, monkeypatch, walk, pairs):
    """The Grid stepper's per-call caps (DRT_GRID_WALK empty cells, DRT_GRID_PAIRS object pairs;
    grid_step) only reschedule a lane's cells and objects across loop iterations: the frame and the
    ray / sample counts are identical to the default caps' on the 1M-triangle grid scene."""
    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(1_000_000), 128, 4, accel="grid")
    s.build()
    renderer.upload(s)
    ref = renderer.render(seed=11, stats=True)
    rst = renderer.stats()
    monkeypatch.setenv("DRT_GRID_WALK", str(walk))
    monkeypatch.setenv("DRT_GRID_PAIRS", str(pairs))
    img = renderer.render(seed=11, stats=True)
    st = renderer.stats()
    np.testing.assert_array_equal(bits(img), bits(ref))
    for k in ("closest_rays", "shadow_rays", "closest_leaf", "shadow_leaf", "closest_prims", "shadow_prims", "samples",
            "wide_shadow_rays", "wide_inner", "wide_leaf", "wide_prims", "wide_verify"):
        assert st[k] == rst[k], k


@pytest.mark.parametrize("layout", ["0", "2"])
def test_node_record_layout_does_not_change_the_frame(drt, renderer, monkeypatch, layout):
    """Where drt_upload_bvh puts each inner node record in memory (DRT_NODE_LAYOUT: 1, the default,
    pairs a record with its larger child's in one 128-B line; 0 keeps the reference's node order;
    2 pairs siblings) changes only addresses: on the 1M-triangle scene, AA and glossy in-order frames
    and every ray, node, leaf and primitive count equal the default layout's bit for bit."""
    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(1_000_000), 96, 4)
    s.build()
    keys = ("closest_rays", "shadow_rays", "closest_inner", "shadow_inner", "closest_leaf", "shadow_leaf",
            "closest_prims", "shadow_prims", "samples",
            "wide_shadow_rays", "wide_inner", "wide_leaf", "wide_prims", "wide_verify")
    out = {}
    for lay in ("1", layout):
        monkeypatch.setenv("DRT_NODE_LAYOUT", lay)
        renderer.upload(s)
        out[lay] = [(bits(renderer.render(seed=3, stats=True, **kw)), renderer.stats())
                    for kw in ({}, {"roughness": 0.1, "max_depth": 6})]
    for (img, st), (ref, rst) in zip(out[layout], out["1"]):
        np.testing.assert_array_equal(img, ref)
        for k in keys:
            assert st[k] == rst[k], k


@pytest.mark.parametrize("accel", ["bvh", "grid"])
def test_seq_tail_handover_does_not_change_the_frame(drt, renderer, tmp_path, monkeypatch, accel):
    """MODE_SEQ frames (DoF + glossy: a lane runs a pixel's samples in order) hand pixels between
    waves at sample boundaries once every pixel is claimed (FrameArgs::seq_cont).  A handed-over
    pixel goes on from the same sample and keyed-stream position, so the frame and every ray /
    traversal count equal the frame with the hand-over off (DRT_SEQ_DONATE=0), bit for bit, with
    or without a bound on the pixels waiting (DRT_SEQ_BACKLOG), on the BVH and the Grid kernel,
    and with frames in flight on several scratch slots.  The 1M-triangle scene makes the samples
    long enough for waves to hand pixels over mid-pixel: the frame's push / pop counters show
    pixels were handed over, and every one was taken up again.  Auto mode (the default) leaves a
    frame alone without the hand-over and turns it on under a frame in flight on another stream."""
    import torch

    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(1_000_000), 192, 16, aperture=8.0, focal=1.0, accel=accel)
    s.build()
    renderer.upload(s)
    kw = {"roughness": 0.1, "max_depth": 8}
    monkeypatch.setenv("DRT_SEQ_TWO_PASS", "0")  # the one-pass in-order frame (the two-pass one has no tail)
    monkeypatch.setenv("DRT_SEQ_DONATE", "0")
    ref = renderer.render(seed=13, stats=True, **kw)
    rst = renderer.stats()
    assert rst["seq_handover"] == 0 and rst["seq_pushed"] == 0
    monkeypatch.setenv("DRT_SEQ_DONATE", "1")
    for backlog in ("0", "64"):
        monkeypatch.setenv("DRT_SEQ_BACKLOG", backlog)
        img = renderer.render(seed=13, stats=True, **kw)
        st = renderer.stats()
        np.testing.assert_array_equal(bits(img), bits(ref), err_msg=f"backlog {backlog}")
        for k in ("closest_rays", "shadow_rays", "closest_inner", "shadow_inner", "closest_leaf", "shadow_leaf",
                  "closest_prims", "shadow_prims", "samples",
            "wide_shadow_rays", "wide_inner", "wide_leaf", "wide_prims", "wide_verify"):
            assert st[k] == rst[k], (backlog, k)
        # the hand-over happened: pixels were pushed, and every push was popped by a kept wave
        assert st["seq_handover"] == 1
        assert st["seq_pushed"] > 0 and st["seq_popped"] == st["seq_pushed"], st
    monkeypatch.delenv("DRT_SEQ_BACKLOG")
    # auto: a lone blocking frame keeps the plain path
    monkeypatch.delenv("DRT_SEQ_DONATE")
    img = renderer.render(seed=13, stats=True, **kw)
    assert renderer.stats()["seq_handover"] == 0
    np.testing.assert_array_equal(bits(img), bits(ref))
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.zeros((192, 192, 3), dtype=torch.float32, device="cuda") for _ in range(4)]
    for i in range(4):
        renderer.render_device(renderer.frame_params(seed=13, slot=i % 2, **kw), outs[i].data_ptr(),
                               streams[i % 2].cuda_stream)
    # the last frame was issued while the one before it (other slot, other stream) was in flight
    assert renderer.stats()["seq_handover"] == 1
    torch.cuda.synchronize()
    for o in outs:
        np.testing.assert_array_equal(bits(o.cpu().numpy()), bits(ref))


def test_slot_reused_from_another_stream_waits_for_its_last_frame(drt, renderer, tmp_path, monkeypatch):
    """A scratch slot's samples / permutation / counters belong to its last frame until that frame
    ends: a frame on the same slot from another stream waits for it on the device (and an aux
    shuffle waits for the slot's last path kernel whether or not that frame used the auxiliary
    streams — ADVICE r2).  Frames alternate streams on ONE slot, and the auxiliary streams switch
    on mid-run (auto mode after a long frame); every frame equals its lone render bit for bit."""
    import torch

    p = sg.write(tmp_path, "s.p3f", sg.synthetic_scene_text(20000, res=(64, 48), spp=16))
    renderer.upload(drt.Scene.load_p3f(p))
    n = 8
    lone = [renderer.render(seed=31 + i) for i in range(n)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.zeros((48, 64, 3), dtype=torch.float32, device="cuda") for _ in range(n)]
    for i in range(n):
        monkeypatch.setenv("DRT_AUX_STREAMS", "0" if i < n // 2 else "1")
        renderer.render_device(renderer.frame_params(seed=31 + i, slot=0), outs[i].data_ptr(),
                               streams[i % 3].cuda_stream)
    torch.cuda.synchronize()
    for i in range(n):
        np.testing.assert_array_equal(outs[i].cpu().numpy().view(np.uint32), lone[i].view(np.uint32), err_msg=str(i))


@pytest.mark.parametrize("accel,kw", [("bvh", {}), ("bvh", {"light_spp": 4}), ("bvh", {"max_depth": 8}),
                                      ("grid", {}), ("grid", {"light_spp": 4, "max_depth": 8})])
def test_aa_two_pass_frame_equals_one_pass(drt, renderer, monkeypatch, accel, kw):
    """AA frames of refraction-free BVH and Grid scenes run in two passes (round 4; drt_capi.hip
    plan, FrameMode MODE_CHAIN / MODE_REPLAY): the samples' closest-hit chains, then every sample's
    shading with its closest hits read back, whose shadow queries walk the 4-ary shadow tree (BVH) or
    the Grid.  The frame equals the one-pass AA frame (DRT_AA_TWO_PASS=0 / DRT_AA_TWO_PASS_GRID=0)
    and the reference-order frame bit for bit, with the same rays and closest-hit work; the
    reference-order frame is one pass with the reference's shadow work (on the Grid every count is
    the same in all three frames)."""
    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(50_000), 64, 16, accel=accel)
    s.build()
    renderer.upload(s)
    assert renderer.plan(renderer.frame_params(seed=6, **kw))["passes"] == 2
    assert renderer.plan(renderer.frame_params(seed=6, reference_order=True, **kw))["passes"] == 1
    img = renderer.render(seed=6, stats=True, **kw)
    st = renderer.stats()
    if accel == "bvh":
        assert st["wide_shadow_rays"] > 0.99 * st["shadow_rays"]
    else:
        assert st["wide_shadow_rays"] == 0
    monkeypatch.setenv("DRT_AA_TWO_PASS_GRID" if accel == "grid" else "DRT_AA_TWO_PASS", "0")
    assert renderer.plan(renderer.frame_params(seed=6, **kw))["passes"] == 1
    one = renderer.render(seed=6, stats=True, **kw)
    st1 = renderer.stats()
    ref = renderer.render(seed=6, stats=True, reference_order=True, **kw)
    rst = renderer.stats()
    np.testing.assert_array_equal(bits(img), bits(one))
    np.testing.assert_array_equal(bits(img), bits(ref))
    keys = ["closest_rays", "shadow_rays", "closest_inner", "closest_leaf", "closest_prims", "samples"]
    if accel == "grid":
        keys += ["shadow_inner", "shadow_leaf", "shadow_prims"]
    for k in keys:
        assert st[k] == st1[k] == rst[k], k
    for k in ("shadow_inner", "shadow_leaf", "shadow_prims"):
        assert st1[k] == rst[k], k


@pytest.mark.parametrize("accel", ["bvh", "grid"])
def test_aa_two_pass_size_rule(drt, monkeypatch, accel):
    """Small AA frames keep one pass (the second pass's tail costs ~0.5 ms per frame rendered alone):
    by default (DRT_AA_TWO_PASS=1) a frame is planned in two passes when the whole frame has >= 2^23
    samples or the scene >= 2^19 objects.  The plan depends on the params and the scene only — the
    same params plan the same way before and after frames complete — and both plans render the same
    frame."""
    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(20_000), 64, 16, accel=accel)
    s.build()
    monkeypatch.setenv("DRT_AA_TWO_PASS", "1")
    r = drt.Renderer(0)
    try:
        r.upload(s)
        assert r.plan(r.frame_params(seed=3))["passes"] == 1  # 64 x 64 x 16 samples, 20 002 objects
        one = r.render(seed=3)
        assert r.plan(r.frame_params(seed=3))["passes"] == 1  # no timing history
        monkeypatch.setenv("DRT_AA_TWO_PASS_MIN_SAMPLES", str(64 * 64 * 16))
        assert r.plan(r.frame_params(seed=3))["passes"] == 2
        monkeypatch.delenv("DRT_AA_TWO_PASS_MIN_SAMPLES")
        monkeypatch.setenv("DRT_AA_TWO_PASS_BIG_SCENE", "20002")
        assert r.plan(r.frame_params(seed=3))["passes"] == 2
        two = r.render(seed=3)
        monkeypatch.delenv("DRT_AA_TWO_PASS_BIG_SCENE")
        monkeypatch.setenv("DRT_AA_TWO_PASS", "2")
        assert r.plan(r.frame_params(seed=3))["passes"] == 2
        np.testing.assert_array_equal(bits(one), bits(two))
    finally:
        r.close()


@pytest.mark.parametrize("accel,spp,kw", [("bvh", 16, {"roughness": 0.1, "max_depth": 8}), ("grid", 9, {"roughness": 0.2}),
                                          ("bvh", 0, {"roughness": 0.2})])
def test_two_pass_in_order_frame_equals_one_pass(drt, renderer, tmp_path, monkeypatch, accel, spp, kw):
    """In-order keyed-stream frames (DoF / glossy) of scenes without refraction run in two passes
    (drt_capi.hip plan, FrameMode MODE_SKEL / MODE_REPLAY): the pixels' closest-hit chains with the
    samples in order, then every sample on its own from its recorded stream position with its
    closest hits read back.  The frame and every ray / node / primitive count equal the one-pass
    frame's (DRT_SEQ_TWO_PASS=0) bit for bit — AA with DoF, depth 8 and glossy bounces on the BVH,
    the Grid, and the Whitted light-sample loop (spp 0) with glossy reflection — and a scene with a
    refracting material keeps the one-pass frame."""
    import bench

    if spp:
        s = drt.Scene()
        bench.populate(s, bench.synthetic_triangles(50_000), 64, spp, aperture=8.0 if accel == "bvh" else 0.0,
                       focal=1.0, accel=accel)
        s.build()
    else:  # the Whitted case on a mixed scene made refraction-free (every material's T set to 0)
        import re
        text = sg.mixed_scene_text(res=(32, 24), spp=0, accel=accel, n_tris=80)
        text = "\n".join(re.sub(r"^(mat\s+(?:\S+\s+){9})\S+", r"\g<1>0", l) for l in text.split("\n"))
        s = drt.Scene.load_p3f(sg.write(tmp_path, "s.p3f", text))
    renderer.upload(s)
    assert renderer.plan(renderer.frame_params(seed=5, **kw))["passes"] == 2
    img = renderer.render(seed=5, **kw)  # the replay pass's shadow queries on the shadow tree (BVH)
    img_r = renderer.render(seed=5, stats=True, reference_order=True, **kw)
    st = renderer.stats()
    monkeypatch.setenv("DRT_SEQ_TWO_PASS", "0")
    assert renderer.plan(renderer.frame_params(seed=5, **kw))["passes"] == 1
    ref = renderer.render(seed=5, stats=True, reference_order=True, **kw)
    rst = renderer.stats()
    np.testing.assert_array_equal(bits(img), bits(ref))
    np.testing.assert_array_equal(bits(img_r), bits(ref))
    for k in ("closest_rays", "shadow_rays", "closest_inner", "shadow_inner", "closest_leaf", "shadow_leaf",
              "closest_prims", "shadow_prims", "samples",
            "wide_shadow_rays", "wide_inner", "wide_leaf", "wide_prims", "wide_verify"):
        assert st[k] == rst[k], k
    monkeypatch.delenv("DRT_SEQ_TWO_PASS")
    glass = sg.mixed_scene_text(res=(24, 16), spp=4, accel="bvh", n_tris=40, aperture=8.0, focal=1.5)
    renderer.upload(drt.Scene.load_p3f(sg.write(tmp_path, "glass.p3f", glass)))
    assert renderer.plan(renderer.frame_params(seed=5, roughness=0.1))["passes"] == 1


@pytest.mark.parametrize("accel,first", [("bvh", "quad"), ("grid", "quad"), ("bvh", "point"), ("grid", "point")])
def test_whitted_two_pass_frame_equals_one_pass(drt, renderer, monkeypatch, accel, first):
    """Whitted frames (spp 0, main.cpp:674-703) of refraction-free scenes run in two passes (round 5):
    the closest-chain pass traces ONE chain per pixel, because the grid_res light samples of a pixel
    share its pixel-centre primary ray and every mirror bounce (main.cpp:683-696), and the replay pass
    runs every (pixel, light sample) with that pixel's hits read back.  The frame equals the one-pass
    frame (DRT_WHITTED_TWO_PASS=0) and the reference-order frame bit for bit, with the same samples
    and shadow rays; a quad-light frame traverses grid_res times fewer closest-hit queries."""
    import bench

    s = drt.Scene()
    c = bench.CAMERA
    s.set_camera(c["eye"], c["at"], c["up"], c["fovy"], c["hither"], 48, 48, 0.0, 1.0)
    s.set_background((0.078, 0.361, 0.753))
    s.set_accel(accel)
    s.set_spp(0)
    quad = ((4, 3, 2), (1, 1, 1), (4, 2, 2), (3, 3, 2), 16)
    if first == "quad":
        s.add_light_quad(*quad)
        s.add_light_point((-3, 1, 5), (1, 1, 1))
    else:
        s.add_light_point((-3, 1, 5), (1, 1, 1))
        s.add_light_quad(*quad)
    s.add_material((1, 0.9, 0.7), 0.5, (1, 1, 1), 0.5, 30.0827, 0, 1)
    s.add_triangles(bench.synthetic_triangles(20_000))
    s.build()
    renderer.upload(s)
    kw = {"max_depth": 6}
    assert renderer.plan(renderer.frame_params(seed=4, **kw))["passes"] == 2
    img = renderer.render(seed=4, stats=True, **kw)
    st = renderer.stats()
    monkeypatch.setenv("DRT_WHITTED_TWO_PASS", "0")
    assert renderer.plan(renderer.frame_params(seed=4, **kw))["passes"] == 1
    one = renderer.render(seed=4, stats=True, **kw)
    st1 = renderer.stats()
    ref = renderer.render(seed=4, stats=True, reference_order=True, **kw)
    rst = renderer.stats()
    np.testing.assert_array_equal(bits(img), bits(one))
    np.testing.assert_array_equal(bits(img), bits(ref))
    div = 16 if first == "quad" else 1
    assert st["samples"] == st1["samples"] == rst["samples"] == 48 * 48 * div
    assert st["shadow_rays"] == st1["shadow_rays"] == rst["shadow_rays"]
    for k in ("closest_rays", "closest_inner", "closest_leaf", "closest_prims"):
        assert st1[k] == rst[k], k
        assert st[k] * div == st1[k], k
    if accel == "grid":
        for k in ("shadow_inner", "shadow_leaf", "shadow_prims"):
            assert st[k] == st1[k] == rst[k], k
    else:
        assert st["wide_shadow_rays"] > 0.99 * st["shadow_rays"]
    # the default rule: a quad-light Whitted frame takes two passes at any size, a point-light one by
    # the AA frames' size rule (this 48 x 48 frame of 20 002 objects keeps one pass)
    monkeypatch.delenv("DRT_WHITTED_TWO_PASS")
    monkeypatch.setenv("DRT_AA_TWO_PASS", "1")
    assert renderer.plan(renderer.frame_params(seed=4, **kw))["passes"] == (2 if first == "quad" else 1)



@pytest.mark.parametrize("accel,spp,first,light_spp,md,rough,chunk", [
    ("bvh", 16, "quad", 1, 4, 0, 0), ("bvh", 16, "point", 4, 6, 0, 0), ("bvh", 9, "quad", 1, 1, 0, 0),
    ("bvh", 0, "quad", 1, 5, 0, 0), ("bvh", 0, "point", 1, 3, 0, 0), ("grid", 16, "quad", 1, 4, 0, 0),
    ("grid", 9, "point", 4, 2, 0, 0), ("grid", 0, "quad", 1, 3, 0, 0),
    # in-order frames (glossy: MODE_SKEL + MODE_REPLAY's keyed-stream draws), and pass 2 in chunks
    ("bvh", 16, "quad", 1, 8, 0.1, 0), ("bvh", 0, "point", 1, 4, 0.2, 0), ("grid", 9, "quad", 1, 3, 0.2, 0),
    ("bvh", 16, "quad", 4, 4, 0, 5000), ("bvh", 9, "point", 1, 6, 0.1, 7777), ("grid", 16, "quad", 1, 3, 0, 9000),
    # XCD bands of the query array (DRT_WAVEFRONT_BANDS=8; chunk -1: bands alone)
    ("bvh", 16, "point", 1, 4, 0, -1), ("grid", 9, "quad", 1, 3, 0.2, -1),
    # a scene without lights: no shadow query at all, the frame is the mirrored background
    ("bvh", 16, "none", 1, 4, 0, 0), ("grid", 4, "none", 1, 2, 0, 0),
    # round 6: the marker layout instead of the compact queries (chunk -2: DRT_WAVEFRONT_COMPACT=0; the Grid
    # then runs MODE_QSTREAM instead of grid_stream)
    ("bvh", 16, "quad", 1, 4, 0, -2), ("grid", 16, "quad", 1, 4, 0, -2), ("grid", 0, "point", 1, 3, 0.2, -2)])
def test_wavefront_replay_equals_persistent_replay(drt, renderer, monkeypatch, accel, spp, first, light_spp, md, rough,
                                                   chunk):
    """Pass 2 of an AA / Whitted two-pass BVH frame as a wavefront (round 5; drt_kernels.hpp WfArgs):
    wf_gen writes every shadow query of every recorded level, trace_stream answers them on the shadow
    tree, wf_combine adds the unshadowed light terms in the light loop's order and unwinds the mirror
    chain.  The frame equals the persistent MODE_AREPLAY pass's (DRT_WAVEFRONT=0) and the
    reference-order frame bit for bit, with the same shadow rays and shadow-tree work — AA with a quad
    light first or last and 4 area samples per light, the depth cut at max_depth 1..8, Whitted frames,
    in-order (glossy) frames whose lens and reflectDir draws wf_gen takes from the recorded stream
    positions, pass 2 in chunks of sample slots (DRT_WAVEFRONT_CHUNK_SLOTS, a partial last chunk), and the
    query array in 8 XCD bands (DRT_WAVEFRONT_BANDS, a padded last band).
    On the Grid the queries run on its stepper (round 6: grid_stream over the compact queries; MODE_QSTREAM
    over the marker layout with DRT_WAVEFRONT_COMPACT=0), with the same cell work."""
    if chunk == -2:
        monkeypatch.setenv("DRT_WAVEFRONT_COMPACT", "0")
        chunk = 0
    if chunk > 0:
        monkeypatch.setenv("DRT_WAVEFRONT_CHUNK_SLOTS", str(chunk))
    # (BVH frames default to 8 XCD bands, Grid frames to 1): chunked frames run with 8, so the last band
    # of a chunk is padded, and the other cases with the default
    if chunk:
        monkeypatch.setenv("DRT_WAVEFRONT_BANDS", "8")
    import bench

    s = drt.Scene()
    c = bench.CAMERA
    s.set_camera(c["eye"], c["at"], c["up"], c["fovy"], c["hither"], 40, 36, 0.0, 1.0)
    s.set_background((0.078, 0.361, 0.753))
    s.set_accel(accel)
    s.set_spp(spp)
    quad = ((4, 3, 2), (1, 1, 1), (4, 2, 2), (3, 3, 2), 16)
    if first == "quad":
        s.add_light_quad(*quad)
        s.add_light_point((-3, 1, 5), (1, 1, 1))
    elif first == "point":
        s.add_light_point((-3, 1, 5), (1, 1, 1))
        s.add_light_quad(*quad)
    s.add_material((1, 0.9, 0.7), 0.5, (1, 1, 1), 0.5, 30.0827, 0, 1)
    s.add_triangles(bench.synthetic_triangles(20_000))
    s.build()
    renderer.upload(s)
    kw = {"max_depth": md, "light_spp": light_spp, "roughness": rough}
    plan = renderer.plan(renderer.frame_params(seed=6, **kw))
    assert plan["passes"] == 2 and plan["wavefront"]
    wf = renderer.render(seed=6, stats=True, **kw)
    st = renderer.stats()
    monkeypatch.setenv("DRT_WAVEFRONT", "0")
    assert not renderer.plan(renderer.frame_params(seed=6, **kw))["wavefront"]
    pers = renderer.render(seed=6, stats=True, **kw)
    st1 = renderer.stats()
    ref = renderer.render(seed=6, stats=True, reference_order=True, **kw)
    rst = renderer.stats()
    np.testing.assert_array_equal(bits(wf), bits(pers))
    np.testing.assert_array_equal(bits(wf), bits(ref))
    assert st["samples"] == st1["samples"] == rst["samples"]
    assert st["shadow_rays"] == st1["shadow_rays"] == rst["shadow_rays"]
    assert (st["shadow_rays"] > 0) == (first != "none")
    for k in ("closest_rays", "closest_inner", "closest_leaf", "closest_prims", "shadow_inner", "shadow_leaf",
              "shadow_prims"):
        assert st[k] == st1[k], k


@pytest.mark.parametrize("accel,spp", [("bvh", 4), ("grid", 4), ("bvh", 0), ("grid", 0)])
def test_refraction_two_pass_frame_equals_one_pass(drt, oracle_mod, renderer, tmp_path, monkeypatch, accel, spp):
    """AA and Whitted frames of scenes WITH a refracting material (glass spheres, trans 1) run in two
    passes (round 5; FrameMode MODE_TCHAIN / MODE_TREPLAY): a sample's closest hits form a binary tree
    (refraction child first, then reflection, main.cpp:465-512); pass 1 records the whole tree in
    rayTracing()'s query order without shadow rays, pass 2 runs rayTracing() with the hits read back in
    that order.  The frame equals the one-pass frame (DRT_TREE_TWO_PASS=0), the reference-order frame
    and the oracle; samples and shadow rays are equal, closest-hit work equal (AA) or grid_res times
    smaller (the Whitted light samples of a pixel share its tree)."""
    text = sg.mixed_scene_text(res=(40, 32), spp=spp, accel=accel, n_tris=1500)
    s, o = load_both(drt, oracle_mod, tmp_path, text)
    s.build()
    renderer.upload(s)
    kw = {"max_depth": 5}
    assert renderer.plan(renderer.frame_params(seed=9, **kw))["passes"] == 2
    img = renderer.render(seed=9, stats=True, **kw)
    st = renderer.stats()
    monkeypatch.setenv("DRT_TREE_TWO_PASS", "0")
    assert renderer.plan(renderer.frame_params(seed=9, **kw))["passes"] == 1
    one = renderer.render(seed=9, stats=True, **kw)
    st1 = renderer.stats()
    ref = renderer.render(seed=9, stats=True, reference_order=True, **kw)
    rst = renderer.stats()
    np.testing.assert_array_equal(bits(img), bits(one))
    np.testing.assert_array_equal(bits(img), bits(ref))
    oimg, ost = o.render(seed=9, **kw)
    compare_images(img, oimg)
    div = 4 if spp == 0 else 1  # mixed_scene_text's quad light 0 has gridRes 4
    assert st["samples"] == st1["samples"] == rst["samples"]
    assert st["shadow_rays"] == st1["shadow_rays"] == rst["shadow_rays"]
    for k in ("closest_rays", "closest_inner", "closest_leaf", "closest_prims"):
        assert st1[k] == rst[k], k
        assert st[k] * div == st1[k], k
    assert st1["closest_rays"] == ost["closest_calls"] and st1["shadow_rays"] == ost["shadow_calls"]


def test_frame_pass_times_split_the_path_time(drt, monkeypatch):
    """drt_frame_pass_times (round 5; bench.py roofline.passes): a two-pass frame's closest-chain and
    replay launches, timed on the frame's stream, add up to its path-kernel time; a one-pass frame
    reports its kernel as pass 1 and ~0 for pass 2."""
    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(20_000), 96, 16)
    s.build()
    r = drt.Renderer(0)
    try:
        r.upload(s)
        monkeypatch.setenv("DRT_AA_TWO_PASS", "2")
        for _ in range(3):
            r.render(seed=5)
        monkeypatch.setenv("DRT_AA_TWO_PASS", "0")
        for _ in range(3):
            r.render(seed=5)
        path_ms, _ = r.frame_times(6)
        p1, p2 = r.frame_pass_times(6)
        assert len(p1) == len(p2) == 6
        # (a one-pass frame's pass-2 span is two events recorded back to back: a few microseconds)
        assert (p1 > 0).all() and (p2[:3] > 0.05).all() and (p2[3:] < 0.05).all()
        np.testing.assert_allclose(p1 + p2, path_ms, rtol=1e-3, atol=2e-3)
    finally:
        r.close()


def test_frame_wave_times_cover_the_persistent_launch(drt, monkeypatch):
    """drt_frame_wave_times (round 6, tools/launch_tail.py): a stats frame's persistent launches stamp each
    resident wave's start and end; every wave ends after it starts, and the spans lie inside the frame."""
    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(20_000), 96, 16, aperture=4.0, focal=1.0)
    s.build()
    r = drt.Renderer(0)
    try:
        r.upload(s)
        monkeypatch.setenv("DRT_AA_TWO_PASS", "2")
        r.render(seed=5, stats=True, max_depth=3)
        assert r.plan(r.frame_params(seed=5, max_depth=3))["passes"] == 2
        w = r.wave_times(0)
        assert len(w) > 64 and (w[:, 1] >= w[:, 0]).all()
        span_us = w[:, 1].max() - w[:, 0].min()
        path_ms, _ = r.frame_times(1)
        assert 0 < span_us <= path_ms[-1] * 1e3 * 1.05 + 20
        r.render(seed=5)  # a frame without stats does not stamp
        with pytest.raises(RuntimeError):
            r.wave_times(0)
    finally:
        r.close()
