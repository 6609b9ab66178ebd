"""ctypes bindings for the CPU ORACLE (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY — importable from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package (distributionraytracer_amd) never imports this module.

The oracle restates rita-mota/DistributionRayTracer's CPU hot path (main.cpp:294-738,
bvh.cpp, grid.cpp, boundingBox.cpp, scene.cpp:10-458, camera.h, maths.h); see
oracle/drt_oracle.h for what is pinned against the reference's own compiled sources and
what is only restated.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"

ACCEL = {"none": 0, "grid": 1, "bvh": 2}
FLT_MAX = np.float32(3.4028234663852886e38)

_f = C.POINTER(C.c_float)
_u8 = C.POINTER(C.c_uint8)
_i32 = C.POINTER(C.c_int32)
_u32 = C.POINTER(C.c_uint32)
_i64 = C.POINTER(C.c_int64)


class OrcInfo(C.Structure):
    _fields_ = [("res_x", C.c_int), ("res_y", C.c_int), ("spp", C.c_uint32), ("accel", C.c_int),
                ("n_objects", C.c_int), ("n_lights", C.c_int), ("n_materials", C.c_int),
                ("has_env", C.c_int), ("skybox_loaded", C.c_int), ("aperture", C.c_float)]


class OrcStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("closest_calls", "shadow_calls", "closest_inner", "closest_leaf",
                                          "shadow_inner", "shadow_leaf", "closest_prims", "shadow_prims",
                                          "samples")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class OrcOptions(C.Structure):
    _fields_ = [("max_depth", C.c_int), ("roughness", C.c_float), ("threads", C.c_int),
                ("row_begin", C.c_int), ("row_end", C.c_int), ("light_spp", C.c_int),
                ("progressive_frame", C.c_int), ("lcg", C.c_int), ("lcg_seed", C.c_uint32)]


def build(force: bool = False) -> None:
    """Compile liboracle.so with g++ (oracle/Makefile)."""
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "drt_oracle.cpp").stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "liboracle.so"], check=True, capture_output=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        vp = C.c_void_p
        L.orc_scene_new.restype = vp
        L.orc_scene_load_p3f.restype = vp
        L.orc_scene_load_p3f.argtypes = [C.c_char_p]
        L.orc_scene_free.argtypes = [vp]
        L.orc_scene_env.restype = C.c_char_p
        L.orc_scene_env.argtypes = [vp]
        L.orc_scene_info.argtypes = [vp, C.POINTER(OrcInfo)]
        L.orc_scene_set_skybox_face.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, _u8]
        L.orc_scene_set_camera.argtypes = [vp, _f, _f, _f, C.c_float, C.c_float, C.c_int, C.c_int, C.c_float, C.c_float]
        L.orc_scene_set_background.argtypes = [vp, _f]
        L.orc_scene_set_accel.argtypes = [vp, C.c_int]
        L.orc_scene_set_spp.argtypes = [vp, C.c_uint32]
        L.orc_scene_add_material.argtypes = [vp, _f, C.c_double, _f, C.c_double, C.c_double, C.c_double, C.c_double]
        L.orc_scene_use_material.argtypes = [vp, C.c_int]
        L.orc_scene_add_sphere.argtypes = [vp, _f, C.c_float]
        L.orc_scene_add_triangle.argtypes = [vp, _f, _f, _f]
        L.orc_scene_add_triangles.argtypes = [vp, _f, C.c_int]
        L.orc_scene_add_plane_pts.argtypes = [vp, _f, _f, _f]
        L.orc_scene_add_plane_nd.argtypes = [vp, _f, C.c_float]
        L.orc_scene_add_box.argtypes = [vp, _f, _f]
        L.orc_scene_add_light_point.argtypes = [vp, _f, _f]
        L.orc_scene_add_light_quad.argtypes = [vp, _f, _f, _f, _f, C.c_uint32]
        L.orc_scene_build.argtypes = [vp]
        L.orc_bvh_num_nodes.argtypes = [vp]
        L.orc_bvh_export.argtypes = [vp, _f, _u32, _u32, _u32, _i32]
        L.orc_grid_export_dims.argtypes = [vp, C.POINTER(C.c_int), _f, _f, _i64]
        L.orc_grid_export.argtypes = [vp, _i64, _i32]
        L.orc_trace_closest.argtypes = [vp, _f, C.c_int, _f, _f, _i32]
        L.orc_trace_shadow.argtypes = [vp, _f, C.c_int, _u8]
        L.orc_object_hit.argtypes = [vp, C.c_int, _f, C.c_int, _f, _f, _u8]
        L.orc_object_bbox.argtypes = [vp, C.c_int, _f]
        L.orc_primary_rays.argtypes = [vp, _f, C.c_int, C.c_int, _f]
        L.orc_skybox_color.argtypes = [vp, _f, C.c_int, _f]
        L.orc_ray_color.argtypes = [vp, _f, _f, C.c_int, C.c_int, C.c_float, C.c_uint32, C.c_uint32, _f]
        L.orc_aabb_hit.argtypes = [_f, _f, C.c_int, _u8, _f, _u8]
        L.orc_camera_frame.argtypes = [vp, _f]
        L.orc_scene_set_eye.argtypes = [vp, _f]
        L.orc_light_points.argtypes = [vp, C.c_int, _f, C.c_int, _f]
        L.orc_vector_ops.argtypes = [_f, _f, C.c_int, _f, _f, _f, _f]
        L.orc_color_ops.argtypes = [_f, C.c_int, _f, _f, _u8]
        L.orc_rnd.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, _f, _u32]
        L.orc_render.argtypes = [vp, C.c_uint32, C.POINTER(OrcOptions), _f, C.POINTER(OrcStats)]
        L.orc_keyed_rand.restype = C.c_uint32
        L.orc_keyed_rand.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_crt_rand.restype = None
        L.orc_crt_rand.argtypes = [C.c_uint32, C.c_int, C.POINTER(C.c_int32)]
        _lib = L
    return _lib


def fp(a):
    return a.ctypes.data_as(_f)


def f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


# ---------------------------------------------------------------------------------------------
# Skybox loading: DevIL with IL_ORIGIN_LOWER_LEFT (scene.cpp:345-346) hands the reference rows
# bottom-up; we decode the JPGs with PIL and flip.  The same bytes feed oracle and product.
# ---------------------------------------------------------------------------------------------
SKY_FACES = ("right", "left", "top", "bottom", "front", "back")  # scene.cpp:333 / CubeMap enum


def load_skybox_dir(path, max_size=None):
    from PIL import Image

    faces = []
    for name in SKY_FACES:
        im = Image.open(os.path.join(path, name + ".jpg")).convert("RGB")
        if max_size is not None and im.width > max_size:
            im = im.resize((max_size, max_size), Image.NEAREST)
        a = np.asarray(im, dtype=np.uint8)[::-1].copy()  # bottom-up
        faces.append(a)
    return faces


class Scene:
    """Oracle scene (owns an orc_scene*)."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("oracle scene creation failed")
        self.h = C.c_void_p(handle)

    def __del__(self):
        try:
            if self.h:
                lib().orc_scene_free(self.h)
                self.h = None
        except Exception:
            pass

    # -- construction --
    @classmethod
    def load_p3f(cls, path, skybox_root=None, skybox_faces=None, skybox_max_size=None):
        s = cls(lib().orc_scene_load_p3f(str(path).encode()))
        env = s.env
        if env:
            if skybox_faces is None:
                root = Path(skybox_root) if skybox_root else Path(path).resolve().parent.parent
                skybox_faces = load_skybox_dir(root / env, skybox_max_size)
            s.set_skybox(skybox_faces)
        return s

    @classmethod
    def new(cls):
        return cls(lib().orc_scene_new())

    @property
    def env(self) -> str:
        return lib().orc_scene_env(self.h).decode()

    def set_skybox(self, faces):
        for i, a in enumerate(faces):
            a = np.ascontiguousarray(a, dtype=np.uint8)
            h, w, bpp = a.shape
            rc = lib().orc_scene_set_skybox_face(self.h, i, w, h, bpp, a.ctypes.data_as(_u8))
            if rc:
                raise ValueError("bad skybox face")

    def info(self) -> OrcInfo:
        i = OrcInfo()
        lib().orc_scene_info(self.h, C.byref(i))
        return i

    def set_camera(self, eye, at, up, fovy, hither, res_x, res_y, aperture=0.0, focal=1.0):
        lib().orc_scene_set_camera(self.h, fp(f32(eye)), fp(f32(at)), fp(f32(up)), fovy, hither, res_x, res_y,
                                   aperture, focal)

    def set_eye(self, eye):
        """Camera::SetEye (camera.h:63-72)."""
        if lib().orc_scene_set_eye(self.h, fp(f32(eye))) != 0:
            raise RuntimeError("set_eye: scene has no camera")

    def set_background(self, rgb):
        lib().orc_scene_set_background(self.h, fp(f32(rgb)))

    def set_accel(self, accel):
        lib().orc_scene_set_accel(self.h, ACCEL[accel] if isinstance(accel, str) else int(accel))

    def set_spp(self, spp):
        lib().orc_scene_set_spp(self.h, int(spp))

    def add_material(self, diff, kd, spec, ks, shine, t, ior):
        return lib().orc_scene_add_material(self.h, fp(f32(diff)), kd, fp(f32(spec)), ks, shine, t, ior)

    def add_sphere(self, c, r):
        return lib().orc_scene_add_sphere(self.h, fp(f32(c)), r)

    def add_triangles(self, verts):
        v = f32(verts).reshape(-1, 9)
        return lib().orc_scene_add_triangles(self.h, fp(v), len(v))

    def add_plane_pts(self, a, b, c):
        return lib().orc_scene_add_plane_pts(self.h, fp(f32(a)), fp(f32(b)), fp(f32(c)))

    def add_plane_nd(self, n, d):
        return lib().orc_scene_add_plane_nd(self.h, fp(f32(n)), d)

    def add_box(self, mn, mx):
        return lib().orc_scene_add_box(self.h, fp(f32(mn)), fp(f32(mx)))

    def add_light_point(self, pos, rgb=(1, 1, 1)):
        return lib().orc_scene_add_light_point(self.h, fp(f32(pos)), fp(f32(rgb)))

    def add_light_quad(self, pos, rgb, v1, v2, grid_res):
        return lib().orc_scene_add_light_quad(self.h, fp(f32(pos)), fp(f32(rgb)), fp(f32(v1)), fp(f32(v2)), grid_res)

    def build(self):
        lib().orc_scene_build(self.h)

    # -- queries --
    def bvh_export(self):
        L = lib()
        n = L.orc_bvh_num_nodes(self.h)
        no = self.info().n_objects
        boxes = np.zeros((n, 6), np.float32)
        leaf = np.zeros(n, np.uint32)
        index = np.zeros(n, np.uint32)
        nobj = np.zeros(n, np.uint32)
        order = np.zeros(no, np.int32)
        L.orc_bvh_export(self.h, fp(boxes), leaf.ctypes.data_as(_u32), index.ctypes.data_as(_u32),
                         nobj.ctypes.data_as(_u32), order.ctypes.data_as(_i32))
        return dict(boxes=boxes, leaf=leaf, index=index, nobjs=nobj, order=order)

    def grid_export(self):
        L = lib()
        dims = (C.c_int * 3)()
        bmin = np.zeros(3, np.float32)
        bmax = np.zeros(3, np.float32)
        nref = C.c_int64()
        L.orc_grid_export_dims(self.h, dims, fp(bmin), fp(bmax), C.byref(nref))
        ncell = dims[0] * dims[1] * dims[2]
        cs = np.zeros(ncell + 1, np.int64)
        co = np.zeros(nref.value, np.int32)
        L.orc_grid_export(self.h, cs.ctypes.data_as(_i64), co.ctypes.data_as(_i32))
        return dict(dims=tuple(dims), bmin=bmin, bmax=bmax, cell_start=cs, cell_objs=co)

    def trace_closest(self, rays):
        rays = f32(rays).reshape(-1, 6)
        n = len(rays)
        t = np.zeros(n, np.float32)
        nrm = np.zeros((n, 3), np.float32)
        obj = np.zeros(n, np.int32)
        lib().orc_trace_closest(self.h, fp(rays), n, fp(t), fp(nrm), obj.ctypes.data_as(_i32))
        return t, nrm, obj

    def trace_shadow(self, rays):
        rays = f32(rays).reshape(-1, 6)
        occ = np.zeros(len(rays), np.uint8)
        lib().orc_trace_shadow(self.h, fp(rays), len(rays), occ.ctypes.data_as(_u8))
        return occ

    def object_hit(self, obj, rays):
        rays = f32(rays).reshape(-1, 6)
        n = len(rays)
        t = np.zeros(n, np.float32)
        nrm = np.zeros((n, 3), np.float32)
        ih = np.zeros(n, np.uint8)
        lib().orc_object_hit(self.h, obj, fp(rays), n, fp(t), fp(nrm), ih.ctypes.data_as(_u8))
        return ih.astype(bool), t, nrm

    def object_bbox(self, obj):
        b = np.zeros(6, np.float32)
        lib().orc_object_bbox(self.h, obj, fp(b))
        return b

    def primary_rays(self, samples, dof=False):
        s = f32(samples).reshape(-1, 4)
        out = np.zeros((len(s), 6), np.float32)
        lib().orc_primary_rays(self.h, fp(s), len(s), int(dof), fp(out))
        return out

    def camera_frame(self):
        f = np.zeros(13, np.float32)
        lib().orc_camera_frame(self.h, fp(f))
        return f

    def light_points(self, light, samples):
        s = f32(samples).reshape(-1, 3)
        out = np.zeros_like(s)
        lib().orc_light_points(self.h, light, fp(s), len(s), fp(out))
        return out

    def skybox_color(self, dirs):
        d = f32(dirs).reshape(-1, 3)
        out = np.zeros_like(d)
        lib().orc_skybox_color(self.h, fp(d), len(d), fp(out))
        return out

    def ray_color(self, rays, light_samples, depth=1, ior=1.0, seed=1, pixel=0):
        r = f32(rays).reshape(-1, 6)
        ls = f32(light_samples).reshape(-1, 3)
        out = np.zeros((len(r), 3), np.float32)
        lib().orc_ray_color(self.h, fp(r), fp(ls), len(r), depth, ior, seed, pixel, fp(out))
        return out

    def render(self, seed=1, max_depth=4, roughness=0.0, threads=0, rows=None, light_spp=1, progressive_frame=0,
               accum=None, lcg_seed=None):
        """progressive_frame n >= 1: zone A frame n, lerped into `accum` (updated in place).
        lcg_seed: draw from the MSVC CRT rand() sequence seeded with it (one thread, pixel order) instead of
        the keyed stream — the RNG of the survey's reference runs."""
        info = self.info()
        opt = OrcOptions(max_depth, roughness, threads, rows[0] if rows else 0, rows[1] if rows else 0, light_spp,
                         progressive_frame, 1 if lcg_seed is not None else 0, lcg_seed or 0)
        if accum is not None:
            assert accum.dtype == np.float32 and accum.shape == (info.res_y, info.res_x, 3) and accum.flags.c_contiguous
            out = accum
        else:
            out = np.zeros((info.res_y, info.res_x, 3), np.float32)
        st = OrcStats()
        rc = lib().orc_render(self.h, seed, C.byref(opt), fp(out), C.byref(st))
        if rc:
            raise RuntimeError(f"orc_render failed ({rc})")
        return out, st.as_dict()


def host_threads():
    """Every host core this process may use: the CPUs of its affinity set, capped by the cgroup
    CPU quota (cpu.max) when one is set.  The CPU baselines and the full-size parity checks run the
    oracle on all of them, whatever OMP_NUM_THREADS says.  (On the GPU boxes nproc is 256 under a
    16-CPU quota; 256 OpenMP threads measured 5.1 Mrays/s there against 6.6-7.0 on 16.)"""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def keyed_rand(seed, pixel, k):
    return lib().orc_keyed_rand(seed, pixel, k)


def aabb_hit(boxes, rays):
    b = f32(boxes).reshape(-1, 6)
    r = f32(rays).reshape(-1, 6)
    n = len(b)
    hit = np.zeros(n, np.uint8)
    t = np.zeros(n, np.float32)
    ins = np.zeros(n, np.uint8)
    lib().orc_aabb_hit(fp(b), fp(r), n, hit.ctypes.data_as(_u8), fp(t), ins.ctypes.data_as(_u8))
    return hit, t, ins


def vector_ops(a, b):
    a = f32(a).reshape(-1, 3)
    b = f32(b).reshape(-1, 3)
    n = len(a)
    nrm = np.zeros((n, 3), np.float32)
    ln = np.zeros(n, np.float32)
    cr = np.zeros((n, 3), np.float32)
    dt = np.zeros(n, np.float32)
    lib().orc_vector_ops(fp(a), fp(b), n, fp(nrm), fp(ln), fp(cr), fp(dt))
    return nrm, ln, cr, dt


def color_ops(c):
    c = f32(c).reshape(-1, 3)
    cl = np.zeros_like(c)
    ex = np.zeros_like(c)
    u8 = np.zeros(c.shape, np.uint8)
    lib().orc_color_ops(fp(c), len(c), fp(cl), fp(ex), u8.ctypes.data_as(_u8))
    return cl, ex, u8


def rnd(seed, pixel, n, sphere, glibc_rand_max=False):
    out = np.zeros((n, 3), np.float32)
    calls = np.zeros(n, np.uint32)
    lib().orc_rnd(seed, pixel, n, int(sphere), int(glibc_rand_max), fp(out), calls.ctypes.data_as(_u32))
    return out, calls


def crt_rand(seed, n):
    """The first n draws of the MSVC CRT rand() after srand(seed) (the oracle's lcg mode)."""
    out = (C.c_int32 * n)()
    lib().orc_crt_rand(seed, n, out)
    return list(out)
