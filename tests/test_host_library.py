"""CPU tests of the product's host side (libdrt.so without touching a GPU).

* the library loads and exports every symbol include/*.h declares;
* the host P3F loader, camera frame and the BVH / Grid builds are identical to the oracle and
  to the reference-generated golden vectors (bit for bit: tree shape, boxes, object order,
  grid CSR) — these are what the GPU kernels consume;
* calls that need a device fail loudly (no silent CPU fallback).
"""
import re
from pathlib import Path

import numpy as np
import pytest

import distributionraytracer_amd as drt
from distributionraytracer_amd import _lib
from tests import scenegen as sg
from tests.conftest import SCENES, needs_reference

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"


@pytest.fixture(scope="module", autouse=True)
def built():
    if not _lib.LIB_PATH.exists():
        _lib.build()


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def declared_symbols():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = h.read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(drt_[a-z0-9_]+)\s*\(", text, re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    names = declared_symbols()
    assert len(names) >= 35
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) <= set(_lib.SIGNATURES), sorted(set(names) - set(_lib.SIGNATURES))
    assert L.drt_abi_version() == 3


def test_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="gfx950|NODEVICE|drt_create"):
        drt.Renderer(0)


def _both(O, tmp_path, text):
    p = sg.write(tmp_path, "s.p3f", text)
    return drt.Scene.load_p3f(p), O.Scene.load_p3f(p)


CASES = ["tiny", "mixed", "tris2k"]


@pytest.mark.parametrize("case", CASES)
def test_bvh_build_matches_reference_golden(tmp_path, case):
    g = np.load(GOLD / f"ref_{case}.npz")
    p = tmp_path / "s.p3f"
    p.write_bytes(g["scene_text"].tobytes())
    s = drt.Scene.load_p3f(p)
    s.set_accel("bvh")
    s.build()
    b = s.bvh_export()
    for k in ("leaf", "index", "nobjs", "order"):
        np.testing.assert_array_equal(b[k], g["bvh_" + k], err_msg=k)
    np.testing.assert_array_equal(bits(b["boxes"]), bits(g["bvh_boxes"]))


@pytest.mark.parametrize("case", ["mixed", "tris2k"])
def test_grid_build_matches_reference_golden(tmp_path, case):
    g = np.load(GOLD / f"ref_{case}.npz")
    p = tmp_path / "s.p3f"
    p.write_bytes(g["scene_text"].tobytes())
    s = drt.Scene.load_p3f(p)
    s.set_accel("grid")
    s.build()
    gr = s.grid_export()
    assert gr["dims"] == tuple(g["grid_dims"])
    np.testing.assert_array_equal(bits(gr["bmin"]), bits(g["grid_bmin"]))
    np.testing.assert_array_equal(gr["cell_start"], g["grid_cell_start"])
    np.testing.assert_array_equal(gr["cell_objs"], g["grid_cell_objs"])


def test_parallel_bvh_build_matches_oracle_large(oracle_mod, tmp_path):
    """100k triangles: the threaded host build splices subtrees back into the reference's
    node numbering; it must equal the oracle's serial restatement exactly."""
    O = oracle_mod
    a, b = _both(O, tmp_path, sg.synthetic_scene_text(100_000, res=(8, 8), spp=1))
    a.build()
    b.build()
    x, y = a.bvh_export(), b.bvh_export()
    for k in ("leaf", "index", "nobjs", "order"):
        np.testing.assert_array_equal(x[k], y[k], err_msg=k)
    np.testing.assert_array_equal(bits(x["boxes"]), bits(y["boxes"]))


def test_p3f_parse_of_100k_triangles_is_fast_and_matches_oracle(oracle_mod, tmp_path):
    """f1 (scene.cpp:565-594): Scene::load_p3f of a 100k-triangle mesh file (the §8d scene written
    by scenegen.write_synthetic_p3f, '%.9g' floats) parses well inside a second here (the reference
    takes ~3.7 s to load + build it), to the oracle's scene: the same counts and camera,
    and the same BVH as the oracle built from that file and as the scene built from the in-memory
    triangles."""
    import time

    import bench

    p = sg.write_synthetic_p3f(tmp_path / "t100k.p3f", 100_000, res=(8, 8), spp=1)
    drt._lib.load()
    t0 = time.perf_counter()
    a = drt.Scene.load_p3f(p)
    parse_s = time.perf_counter() - t0
    b = oracle_mod.Scene.load_p3f(p)
    c = drt.Scene()
    bench.populate(c, bench.synthetic_triangles(100_000), 8, 1)
    ia, ib = a.info(), b.info()
    for k in ("res_x", "res_y", "spp", "accel", "n_objects", "n_lights", "n_materials"):
        assert getattr(ia, k) == getattr(ib, k) == getattr(c.info(), k), k
    for s in (a, b, c):
        s.build()
    x, y, z = a.bvh_export(), b.bvh_export(), c.bvh_export()
    for k in ("leaf", "index", "nobjs", "order"):
        np.testing.assert_array_equal(x[k], y[k], err_msg=k)
        np.testing.assert_array_equal(x[k], z[k], err_msg=k)
    np.testing.assert_array_equal(bits(x["boxes"]), bits(y["boxes"]))
    np.testing.assert_array_equal(bits(x["boxes"]), bits(z["boxes"]))
    # the parse time is reported, not asserted (a loaded host would fail a correct build); bench.py's
    # `load` field times the 1M-triangle file on the GPU box
    print(f"P3F parse of 100k triangles: {parse_s:.2f} s")


def test_survey_synthetic_scene_bvh_has_the_reference_run_node_count():
    """Reference pin: the reference's BVH over the survey's 100k-triangle
    soup + floor has 118 983 nodes.  The soup is the survey's generator as reconstructed by
    tools/generator_search.py (scenegen.survey_triangles); the product's build must give that count."""
    s = drt.Scene()
    s.set_accel("bvh")
    s.add_material((1, 0.9, 0.7), 0.5, (1, 1, 1), 0.5, 30.0827, 0, 1)
    s.add_triangles(np.concatenate([sg.survey_triangles(100_000), sg.FLOOR]))
    s.build()
    assert s.info().bvh_nodes == 118_983


def test_cluster_scene_has_oversized_leaf_matching_oracle(oracle_mod, tmp_path):
    """The `cluster` scene of the GPU big-leaf cases really yields a leaf of >= 31 objects
    (the count-31 descriptor path), in the same tree as the oracle's build."""
    a, b = _both(oracle_mod, tmp_path, sg.mixed_scene_text(accel="bvh", cluster=40))
    a.build()
    b.build()
    x, y = a.bvh_export(), b.bvh_export()
    for k in ("leaf", "index", "nobjs", "order"):
        np.testing.assert_array_equal(x[k], y[k], err_msg=k)
    assert (np.asarray(x["nobjs"])[np.asarray(x["leaf"]).astype(bool)] >= 31).any()


def test_camera_frame_matches_reference_golden():
    g = np.load(GOLD / "ref_misc.npz")
    for ci, c in enumerate(g["cam_params"]):
        s = drt.Scene()
        s.set_camera(c[0:3], c[3:6], c[6:9], c[9], c[10], int(c[11]), int(c[12]), c[13], c[14])
        f = s.camera_frame()
        mine = np.array([f.plane_dist, f.aperture, f.w, f.h, *f.u, *f.v, *f.n], np.float32)
        np.testing.assert_array_equal(bits(mine), bits(g["cam_frames"][ci]))


def test_set_eye_matches_oracle_camera(oracle_mod):
    """Camera::SetEye (camera.h:63-72), the interactive camera motion (main.cpp:530-533): the host
    camera and the oracle recompute the frame (u, v, n) and the plane distance bit for bit; the view
    window (w, h) and the aperture keep their construction values, as in the reference."""
    g = np.load(GOLD / "ref_misc.npz")
    for ci, c in enumerate(g["cam_params"]):
        a, b = drt.Scene(), oracle_mod.Scene.new()
        for s in (a, b):
            s.set_camera(c[0:3], c[3:6], c[6:9], c[9], c[10], int(c[11]), int(c[12]), c[13], c[14])
        f0 = a.camera_frame()
        for k in range(5):  # an orbit about the z axis through `at`, plus a change of height
            ang = 0.7 * (k + 1)
            e = np.array(c[0:3], np.float64) - np.array(c[3:6], np.float64)
            eye = np.array(c[3:6], np.float64) + np.array([e[0] * np.cos(ang) - e[1] * np.sin(ang),
                                                           e[0] * np.sin(ang) + e[1] * np.cos(ang), e[2] + 0.1 * k])
            a.set_eye(eye)
            b.set_eye(eye)
            f = a.camera_frame()
            mine = np.array([f.plane_dist, f.aperture, f.w, f.h, *f.u, *f.v, *f.n], np.float32)
            np.testing.assert_array_equal(bits(mine), bits(b.camera_frame()), err_msg=f"camera {ci} eye {k}")
            np.testing.assert_array_equal(np.float32(f.eye), np.float32(eye))
            assert (f.w, f.h, f.aperture) == (f0.w, f0.h, f0.aperture)


@needs_reference
@pytest.mark.parametrize("scene", ["balls_low", "dof", "teste", "motion", "balls_box", "blueDiamond",
                                   "dragon_assignment1"])
def test_p3f_loader_matches_oracle(oracle_mod, scene):
    O = oracle_mod
    a = drt.Scene.load_p3f(SCENES / f"{scene}.p3f", skybox_max_size=8)
    b = O.Scene.load_p3f(SCENES / f"{scene}.p3f", skybox_max_size=8)
    ia, ib = a.info(), b.info()
    for k in ("res_x", "res_y", "spp", "accel", "n_objects", "n_lights", "n_materials", "has_env"):
        assert getattr(ia, k) == getattr(ib, k), k
    assert ia.aperture == ib.aperture
    fa = a.camera_frame()
    mine = np.array([fa.plane_dist, fa.aperture, fa.w, fa.h, *fa.u, *fa.v, *fa.n], np.float32)
    np.testing.assert_array_equal(bits(mine), bits(b.camera_frame()))
    # accelerator built from the parsed scene must match too
    if ia.accel == 2:
        a.build()
        b.build()
        x, y = a.bvh_export(), b.bvh_export()
        np.testing.assert_array_equal(x["order"], y["order"])
        np.testing.assert_array_equal(bits(x["boxes"]), bits(y["boxes"]))


def _u8fromfloat(x):  # maths.h:126-130 in float32
    v = np.float32(x) * np.float32(255.99)
    return np.where(v >= 255.0, 255, np.where(v > 0, v, 0)).astype(np.uint8)


def test_image_rgb8_is_u8fromfloat():
    import distributionraytracer_amd as d

    rng = np.random.default_rng(4)
    f = rng.random((7, 9, 3), dtype=np.float32) * 1.2 - 0.1
    f[0, 0] = [1.0, 0.99609375, 0.0]
    np.testing.assert_array_equal(d.image_rgb8(f), _u8fromfloat(f))


def test_write_png_is_upright_rgb8(tmp_path):
    import distributionraytracer_amd as d
    from PIL import Image

    rng = np.random.default_rng(5)
    f = rng.random((6, 11, 3), dtype=np.float32)
    p = tmp_path / "RT_Output.png"
    d.write_png(p, f)
    img = np.asarray(Image.open(p))
    assert img.shape == (6, 11, 3) and img.dtype == np.uint8
    # lower-left-origin frame: the PNG's top row is the frame's last row (DevIL, main.cpp:251-266)
    np.testing.assert_array_equal(img, _u8fromfloat(f)[::-1])


@pytest.mark.parametrize("scene", ["balls_low", "dof", "motion", "teste", "balls_box", "balls_high", "blueDiamond",
                                   "dragon", "assignment1", "dragon_assignment1"])
def test_shipped_scene_fixture_loads_like_oracle(oracle_mod, tmp_path, scene):
    """Every shipped scene (data fixture, no reference checkout needed): the product's loader
    and the oracle's parse the same objects, lights, camera and accelerator, and the product's
    parallel BVH build gives the oracle's tree."""
    from tests import shipped

    p = shipped.write(tmp_path, scene)
    faces = shipped.skybox_faces(scene)
    a = drt.Scene.load_p3f(p, skybox_faces=faces)
    b = oracle_mod.Scene.load_p3f(p, skybox_faces=faces)
    ia, ib = a.info(), b.info()
    for k in ("res_x", "res_y", "spp", "accel", "n_objects", "n_lights", "n_materials", "has_env"):
        assert getattr(ia, k) == getattr(ib, k), k
    assert ia.skybox_loaded == (faces is not None)
    fa = a.camera_frame()
    mine = np.array([fa.plane_dist, fa.aperture, fa.w, fa.h, *fa.u, *fa.v, *fa.n], np.float32)
    np.testing.assert_array_equal(bits(mine), bits(b.camera_frame()))
    a.set_accel("bvh")
    b.set_accel("bvh")
    a.build()
    b.build()
    x, y = a.bvh_export(), b.bvh_export()
    for k in ("leaf", "index", "nobjs", "order"):
        np.testing.assert_array_equal(x[k], y[k], err_msg=k)
    np.testing.assert_array_equal(bits(x["boxes"]), bits(y["boxes"]))


@pytest.mark.parametrize("case,accel", [("mixed", "bvh"), ("tris2k", "bvh"), ("mixed", "grid"), ("tris2k", "grid")])
def test_scalar_cpu_traverse_matches_reference_golden(tmp_path, case, accel):
    """drt_scene_trace_cpu: the host BVH::Traverse / Grid::Traverse (one ray at a time on the CPU,
    no device) return the reference's results bit for bit."""
    g = np.load(GOLD / f"ref_{case}.npz")
    p = tmp_path / "s.p3f"
    p.write_bytes(g["scene_text"].tobytes())
    s = drt.Scene.load_p3f(p)
    s.set_accel(accel)
    s.build()
    pre = "bvh" if accel == "bvh" else "grid"
    rays = g["rays"] if accel == "bvh" else g["grid_rays"]
    t, n, obj = s.trace_cpu(rays)
    np.testing.assert_array_equal(obj, g[f"{pre}_obj"])
    np.testing.assert_array_equal(bits(t), bits(g[f"{pre}_t"]))
    np.testing.assert_array_equal(bits(n), bits(g[f"{pre}_n"]))
    srays = g["shadow_rays"] if accel == "bvh" else g["grid_rays"]
    np.testing.assert_array_equal(s.trace_cpu(srays, shadow=True), g[f"{pre}_occ"])


def test_group_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="drt_group_create"):
        drt.RendererGroup([0])


def test_grid_vs_bvh_tool_covers_the_shipped_grid_scenes(tmp_path):
    """SURVEY §8 f4 motivates the Grid kernel's perf row by the shipped scenes whose P3F selects
    `accel grid`; tools/grid_vs_bvh.py (profiles/r03_grid_vs_bvh_shipped.jsonl) must time exactly
    those, and each must load with the Grid as its accelerator (scene.h:22, accel 1)."""
    from tests import shipped

    text = (ROOT / "tools" / "grid_vs_bvh.py").read_text()
    scenes = set(re.findall(r'"(\w+)"', re.search(r"SCENES = \(([^)]*)\)", text).group(1)))
    grid_default = {n for n in shipped.names()
                    if re.search(rb"(?m)^accel[ \t]+grid", shipped._npz()[f"{n}/head"].tobytes())}
    assert scenes == grid_default, (scenes, grid_default)
    for n in sorted(grid_default):
        s = drt.Scene.load_p3f(shipped.write(tmp_path, n), skybox_faces=shipped.skybox_faces(n))
        assert s.info().accel == 1, n


@pytest.mark.parametrize("case", ["mixed", "tris2k"])
def test_reference_grid_lists_each_object_in_a_whole_box_of_cells(case):
    """The premise of the Grid shadow tree's cell certificate (round 6, grid_certificate): Grid::Build lists
    an object in EVERY cell of the box [min, max] of its cell coordinates (grid.cpp:78-92), so the min / max
    over the cells that list it (drt_upload_grid's per-object ranges) is that box, and a cell inside it lists
    the object.  Checked on the reference-run grids of the golden fixtures."""
    g = np.load(GOLD / f"ref_{case}.npz")
    nx, ny, nz = (int(d) for d in g["grid_dims"])
    cs, co = g["grid_cell_start"], g["grid_cell_objs"]
    cell = np.repeat(np.arange(nx * ny * nz), np.diff(cs))
    x, y, z = cell % nx, (cell // nx) % ny, cell // (nx * ny)
    n_obj = int(co.max()) + 1
    lo = np.full((n_obj, 3), np.iinfo(np.int64).max)
    hi = np.full((n_obj, 3), -1)
    for a, v in enumerate((x, y, z)):
        np.minimum.at(lo[:, a], co, v)
        np.maximum.at(hi[:, a], co, v)
    count = np.bincount(co, minlength=n_obj)
    listed = count > 0
    assert listed.all()
    np.testing.assert_array_equal(count, np.prod(hi - lo + 1, axis=1))
    # and no object is listed twice in one cell
    assert len(np.unique(cell * n_obj + co)) == len(co)
