"""Several GPUs behind the C ABI (drt_group_*, include/drt.h).

A group deals 16x16 tiles over its devices, renders each device's shard on its own stream,
all-gathers the shard buffers with RCCL (ncclCommInitAll clique, librccl loaded at run time) and
reassembles the frame on device 0.  Every group size takes that path — a one-device group's
all-gather is a local copy — so on a one-GPU box these tests run the RCCL collective path with
N = 1; the frame must equal a single context's frame bit for bit.  Larger N (one rank per
device) uses the same code with more communicator ranks and is not run here (one GPU per box).
"""
import numpy as np
import pytest

from tests import scenegen as sg
from tests import shipped

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def drt():
    import distributionraytracer_amd as d

    return d


def n_devices():
    import torch

    return torch.cuda.device_count()


@pytest.mark.parametrize("accel,spp,kw", [("bvh", 4, {}), ("grid", 0, {}), ("none", 4, {}), ("bvh", 4, {"roughness": 0.2}),
                                          ("bvh", 9, {"light_spp": 4})])
def test_group_frame_equals_single_context_frame(drt, tmp_path, accel, spp, kw):
    p = sg.write(tmp_path, "s.p3f", sg.mixed_scene_text(res=(70, 45), spp=spp, accel=accel, n_tris=80))
    scene = drt.Scene.load_p3f(p)
    r = drt.Renderer(0)
    r.upload(scene)
    whole = r.render(seed=19, **kw)
    r.close()
    g = drt.RendererGroup(range(n_devices()))
    g.upload(scene)
    frame = g.render(seed=19, **kw)
    again = g.render(seed=19, **kw)  # buffers reused
    g.close()
    np.testing.assert_array_equal(frame.view(np.uint32), whole.view(np.uint32))
    np.testing.assert_array_equal(again.view(np.uint32), whole.view(np.uint32))


def test_group_render_device_and_shipped_scene(drt, tmp_path):
    import torch

    name = "dragon_assignment1"
    scene = drt.Scene.load_p3f(shipped.write(tmp_path, name, res=(200, 150)), skybox_faces=shipped.skybox_faces(name))
    r = drt.Renderer(0)
    r.upload(scene)
    whole = r.render(seed=3)
    r.close()
    g = drt.RendererGroup(range(n_devices()))
    g.upload(scene)
    d = torch.zeros((150, 200, 3), dtype=torch.float32, device="cuda:0")
    s = torch.cuda.Stream()
    g.render_device(d.data_ptr(), seed=3, stream=s.cuda_stream)
    g.synchronize()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy().view(np.uint32), whole.view(np.uint32))
    g.close()


def test_group_progressive_and_errors(drt, tmp_path):
    p = sg.write(tmp_path, "s.p3f", sg.mixed_scene_text(res=(24, 16), spp=4, accel="bvh", n_tris=40))
    scene = drt.Scene.load_p3f(p)
    r = drt.Renderer(0)
    r.upload(scene)
    g = drt.RendererGroup(range(n_devices()))
    g.upload(scene)
    acc_r = np.zeros((16, 24, 3), np.float32)
    acc_g = np.zeros((16, 24, 3), np.float32)
    for n in (1, 2, 3):
        r.render(seed=n, progressive_frame=n, accum=acc_r)
        if n_devices() == 1:
            g.render(seed=n, progressive_frame=n, accum=acc_g)
    if n_devices() == 1:
        np.testing.assert_array_equal(acc_g.view(np.uint32), acc_r.view(np.uint32))
    with pytest.raises(RuntimeError):
        drt.RendererGroup([0, 0])  # one rank per device
    r.close()
    g.close()


def test_cpp_caller_renders_group_frame(drt, tmp_path):
    """A C++ host renders a tile-sharded frame through drt_group_* without torch
    (tests/cpp/scene_caller.cpp `group` mode: drt::upload_scene / drt::render_scene on a group)."""
    from tests.test_cpp_api import CALLER, run

    p = sg.write(tmp_path, "s.p3f", sg.mixed_scene_text(res=(40, 32), spp=4, accel="bvh", n_tris=60))
    run(CALLER, "group", p, 11, n_devices(), tmp_path / "f.out")
    img = np.fromfile(tmp_path / "f.out", np.float32).reshape(32, 40, 3)
    r = drt.Renderer(0)
    r.upload(drt.Scene.load_p3f(p))
    mine = r.render(seed=11)
    r.close()
    np.testing.assert_array_equal(img.view(np.uint32), mine.view(np.uint32))


def test_c5_workload_sharded_and_grouped_equal_whole_frame(drt):
    """BASELINE config C5 on one GPU: the C4 workload (1M triangles + floor, 1024^2, 64 spp, DoF
    aperture 8 focal 1, depth 8, roughness 0.1) split as the 8-GPU run splits it — eight
    interleaved 16x16-tile shards, each rendered into its own shard-compact buffer, reassembled by
    drt_unshard_device — and through a RendererGroup over every device of the box (shard ->
    RCCL all-gather -> unshard).  Both equal the whole frame bit for bit (the loop being split is
    main.cpp:603-721; the whole frame is checked against the oracle by
    test_full_size_config_matches_oracle[C4...])."""
    import torch

    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(1_000_000), 1024, 64, aperture=8.0, focal=1.0)
    s.build()
    kw = dict(roughness=0.1, max_depth=8)
    r = drt.Renderer(0)
    r.upload(s)
    whole = r.render(seed=7, **kw)
    p0 = r.frame_params(seed=7, shard=0, n_shards=8, **kw)
    tiles, floats = r.shard_layout(p0)
    assert tiles * 8 >= (1024 // 16) ** 2
    bufs = torch.zeros((8, floats), dtype=torch.float32, device="cuda")
    for k in range(8):
        r.render_device(r.frame_params(seed=7, shard=k, n_shards=8, **kw), bufs[k].data_ptr())
    frame = torch.zeros((1024, 1024, 3), dtype=torch.float32, device="cuda")
    r.unshard_device(p0, bufs.data_ptr(), frame.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(frame.cpu().numpy().view(np.uint32), whole.view(np.uint32))
    r.close()
    del bufs, frame
    g = drt.RendererGroup(range(n_devices()))
    g.upload(s)
    gf = g.render(seed=7, **kw)
    g.close()
    np.testing.assert_array_equal(gf.view(np.uint32), whole.view(np.uint32))
