"""ctypes bindings for libdrt.so (include/drt.h + include/drt_host.h).

The shared library is built in-tree by distributionraytracer_amd/csrc/Makefile (hipcc for the
gfx950 kernels, g++ for the host scene library).  There is no fallback: if the library is
missing, load() raises — the product never renders on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "libdrt.so"
CSRC = PKG / "csrc"

DRT_OK = 0
STATUS = {0: "DRT_OK", -1: "DRT_E_INVALID", -2: "DRT_E_HIP", -3: "DRT_E_NODEVICE", -4: "DRT_E_OOM",
          -5: "DRT_E_STATE", -6: "DRT_E_UNSUPPORTED"}
ACCEL = {"none": 0, "grid": 1, "bvh": 2}
FRAME_STATS = 1
FRAME_REFERENCE_ORDER = 4  # shadow queries on the reference's binary tree, in its visit order

_f = C.POINTER(C.c_float)
_u8 = C.POINTER(C.c_uint8)
_i32 = C.POINTER(C.c_int32)
_u32 = C.POINTER(C.c_uint32)
_i64 = C.POINTER(C.c_int64)
_vp = C.c_void_p


class DrtOptions(C.Structure):
    _fields_ = [("device", C.c_int32), ("reserved", C.c_int32 * 7)]


class DrtCamera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3), ("n", C.c_float * 3),
                ("w", C.c_float), ("h", C.c_float), ("plane_dist", C.c_float), ("focal_ratio", C.c_float),
                ("aperture", C.c_float), ("res_x", C.c_int32), ("res_y", C.c_int32)]


class DrtFrameParams(C.Structure):
    _fields_ = [("seed", C.c_uint32), ("max_depth", C.c_int32), ("roughness", C.c_float), ("shard", C.c_int32),
                ("n_shards", C.c_int32), ("tile", C.c_int32), ("flags", C.c_int32), ("light_spp", C.c_int32),
                ("progressive_frame", C.c_int32), ("slot", C.c_int32), ("reserved", C.c_int32 * 2)]


class DrtFrameStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("closest_rays", "shadow_rays", "closest_inner", "closest_leaf",
                                          "shadow_inner", "shadow_leaf", "closest_prims", "shadow_prims",
                                          "samples")] + [("render_ms", C.c_double), ("kernel_ms", C.c_double)] + \
        [(n, C.c_uint64) for n in ("wave_node_iters", "wave_path_iters", "lane_path_iters", "cycles_refill",
                                   "cycles_node", "cycles_shade", "stack_pushes", "stack_spills",
                                   "wave_leaf_iters", "cycles_leaf", "seq_pushed", "seq_popped")] + \
        [("seq_handover", C.c_int32), ("reserved", C.c_int32)] + \
        [(n, C.c_uint64) for n in ("wide_shadow_rays", "wide_inner", "wide_leaf", "wide_prims", "wide_verify",
                                   "wide_grid_walks")]

    def as_dict(self):
        return {n: (float(getattr(self, n)) if n.endswith("_ms") else int(getattr(self, n))) for n, _ in self._fields_
                if n != "reserved"}


class DrtFramePlan(C.Structure):
    _fields_ = [("work_items", C.c_uint64), ("sample_slots", C.c_uint64), ("mode", C.c_int32),
                ("persistent", C.c_int32), ("tiles_in_shard", C.c_int32), ("passes", C.c_int32),
                ("wavefront", C.c_int32), ("reserved", C.c_int32 * 3)]


class DrtLight(C.Structure):
    _fields_ = [("type", C.c_int32), ("pos", C.c_float * 3), ("e1", C.c_float * 3), ("e2", C.c_float * 3),
                ("grid_res", C.c_uint32)]


class DrtMaterial(C.Structure):
    _fields_ = [("diff", C.c_float * 3), ("kd", C.c_float), ("spec", C.c_float * 3), ("ks", C.c_float),
                ("shine", C.c_float), ("refl", C.c_float), ("trans", C.c_float), ("ior", C.c_float)]


class DrtPrim(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("a", C.c_float * 3), ("b", C.c_float * 3),
                ("c", C.c_float * 3), ("r", C.c_float)]


class DrtSceneDesc(C.Structure):
    """drt_scene_desc (include/drt.h): what drt_upload_scene reads."""
    _fields_ = [("camera", DrtCamera), ("materials", C.POINTER(DrtMaterial)), ("n_materials", C.c_int32),
                ("prims", C.POINTER(DrtPrim)), ("n_prims", C.c_int32), ("lights", C.POINTER(DrtLight)),
                ("n_lights", C.c_int32), ("background", C.c_float * 3), ("accel", C.c_int32), ("spp", C.c_uint32),
                ("has_skybox", C.c_int32), ("skybox", C.c_void_p * 6), ("sky_w", C.c_int32 * 6),
                ("sky_h", C.c_int32 * 6), ("sky_bpp", C.c_int32 * 6)]


class DrtSceneInfo(C.Structure):
    _fields_ = [("res_x", C.c_int32), ("res_y", C.c_int32), ("spp", C.c_uint32), ("accel", C.c_int32),
                ("n_objects", C.c_int32), ("n_lights", C.c_int32), ("n_materials", C.c_int32),
                ("has_env", C.c_int32), ("skybox_loaded", C.c_int32), ("aperture", C.c_float),
                ("bvh_nodes", C.c_int32), ("build_ms", C.c_double)]


# Every symbol include/drt.h and include/drt_host.h declare, with its ctypes signature.
SIGNATURES = {
    # drt.h
    "drt_abi_version": (C.c_int, []),
    "drt_create": (C.c_int, [C.POINTER(_vp), C.POINTER(DrtOptions)]),
    "drt_destroy": (None, [_vp]),
    "drt_last_error": (C.c_char_p, [_vp]),
    "drt_upload_scene": (C.c_int, [_vp, C.POINTER(DrtSceneDesc)]),
    "drt_set_camera": (C.c_int, [_vp, C.POINTER(DrtCamera)]),
    "drt_upload_bvh": (C.c_int, [_vp, _vp, C.c_uint32, _u32, C.c_uint32]),
    "drt_upload_grid": (C.c_int, [_vp, _i32, _f, _f, _i64, _i32, C.c_int64]),
    "drt_upload_grid_shadow_bvh": (C.c_int, [_vp, _vp, C.c_uint32, _u32, C.c_uint32]),
    "drt_render": (C.c_int, [_vp, C.POINTER(DrtFrameParams), _f]),
    "drt_shard_layout": (C.c_int, [_vp, C.POINTER(DrtFrameParams), _i64, _i64]),
    "drt_plan_frame": (C.c_int, [_vp, C.POINTER(DrtFrameParams), C.POINTER(DrtFramePlan)]),
    "drt_render_device": (C.c_int, [_vp, C.POINTER(DrtFrameParams), _vp, _vp]),
    "drt_unshard_device": (C.c_int, [_vp, C.POINTER(DrtFrameParams), _vp, _vp, _vp]),
    "drt_trace_closest": (C.c_int, [_vp, _f, C.c_int32, _f, _f, _i32]),
    "drt_trace_shadow": (C.c_int, [_vp, _f, C.c_int32, _u8]),
    "drt_trace_device": (C.c_int, [_vp, C.c_int, _vp, C.c_int32, _vp, _vp, _vp, _vp, _vp]),
    "drt_set_trace_flags": (C.c_int, [_vp, C.c_int]),
    "drt_trace_stats": (C.c_int, [_vp, C.POINTER(DrtFrameStats)]),
    "drt_get_stats": (C.c_int, [_vp, C.POINTER(DrtFrameStats)]),
    "drt_frame_times": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "drt_frame_spans": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_double)]),
    "drt_frame_pass_times": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "drt_frame_wave_times": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_uint64), C.c_int64]),
    "drt_frame_stage_times": (C.c_int, [_vp, C.POINTER(C.c_double)]),
    "drt_frame_resolution": (C.c_int, [_vp, _i32]),
    "drt_group_create": (C.c_int, [C.POINTER(_vp), C.c_int, _i32]),
    "drt_group_destroy": (None, [_vp]),
    "drt_group_last_error": (C.c_char_p, [_vp]),
    "drt_group_size": (C.c_int, [_vp]),
    "drt_group_ctx": (_vp, [_vp, C.c_int]),
    "drt_group_render": (C.c_int, [_vp, C.POINTER(DrtFrameParams), _f]),
    "drt_group_render_device": (C.c_int, [_vp, C.POINTER(DrtFrameParams), _vp, _vp]),
    "drt_group_synchronize": (C.c_int, [_vp]),
    "drt_group_set_camera": (C.c_int, [_vp, C.POINTER(DrtCamera)]),
    # drt_host.h
    "drt_group_scene_upload": (C.c_int, [_vp, _vp]),
    "drt_scene_new": (_vp, []),
    "drt_scene_load_p3f": (_vp, [C.c_char_p]),
    "drt_scene_free": (None, [_vp]),
    "drt_scene_info": (C.c_int, [_vp, C.POINTER(DrtSceneInfo)]),
    "drt_scene_env": (C.c_char_p, [_vp]),
    "drt_scene_set_skybox_face": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.c_int, _u8]),
    "drt_scene_set_camera": (C.c_int, [_vp, _f, _f, _f, C.c_float, C.c_float, C.c_int, C.c_int, C.c_float,
                                       C.c_float]),
    "drt_scene_set_background": (C.c_int, [_vp, _f]),
    "drt_scene_set_accel": (C.c_int, [_vp, C.c_int]),
    "drt_scene_set_spp": (C.c_int, [_vp, C.c_uint32]),
    "drt_scene_add_material": (C.c_int, [_vp, _f, C.c_double, _f, C.c_double, C.c_double, C.c_double, C.c_double]),
    "drt_scene_use_material": (C.c_int, [_vp, C.c_int]),
    "drt_scene_add_sphere": (C.c_int, [_vp, _f, C.c_float]),
    "drt_scene_add_triangles": (C.c_int, [_vp, _f, C.c_int64]),
    "drt_scene_add_plane_pts": (C.c_int, [_vp, _f, _f, _f]),
    "drt_scene_add_plane_nd": (C.c_int, [_vp, _f, C.c_float]),
    "drt_scene_add_box": (C.c_int, [_vp, _f, _f]),
    "drt_scene_add_light_point": (C.c_int, [_vp, _f, _f]),
    "drt_scene_add_light_quad": (C.c_int, [_vp, _f, _f, _f, _f, C.c_uint32]),
    "drt_scene_build": (C.c_int, [_vp]),
    "drt_scene_bvh_export": (C.c_int, [_vp, _f, _u32, _u32, _u32, _i32]),
    "drt_scene_grid_export_dims": (C.c_int, [_vp, _i32, _f, _f, _i64]),
    "drt_scene_grid_export": (C.c_int, [_vp, _i64, _i32]),
    "drt_scene_camera_frame": (C.c_int, [_vp, C.POINTER(DrtCamera)]),
    "drt_scene_upload": (C.c_int, [_vp, _vp]),
    "drt_scene_set_eye": (C.c_int, [_vp, _f]),
    "drt_scene_upload_camera": (C.c_int, [_vp, _vp]),
    "drt_group_scene_upload_camera": (C.c_int, [_vp, _vp]),
    "drt_set_image_decoder": (C.c_int, [_vp, _vp]),
    "drt_scene_load_skybox": (C.c_int, [_vp, C.c_char_p]),
    "drt_scene_trace_cpu": (C.c_int, [_vp, C.c_int, _f, C.c_int64, _f, _f, _i32, _u8]),
    "drt_scene_skybox_color_cpu": (C.c_int, [_vp, _f, C.c_int64, _f]),
    "drt_image_rgb8": (C.c_int, [_vp, C.c_int32, C.c_int32, _vp]),
    "drt_image_write_png": (C.c_int, [C.c_char_p, _vp, C.c_int32, C.c_int32]),
}


def build(force: bool = False, jobs: int = 8) -> Path:
    """Compile libdrt.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    args = ["make", "-C", str(CSRC), f"-j{jobs}"]
    if force:
        subprocess.run(["make", "-C", str(CSRC), "clean"], check=True, capture_output=True)
    r = subprocess.run(args, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("libdrt.so build failed:\n" + r.stdout[-4000:] + r.stderr[-4000:])
    return LIB_PATH


_lib = None


def load():
    """Load libdrt.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process.  PyTorch ships its own libamdhip64 (DT_NEEDED
        # "libamdhip64.so", SONAME "libamdhip64.so.7"); loading torch first makes libdrt.so's
        # DT_NEEDED "libamdhip64.so.7" resolve to that same runtime, so device pointers,
        # streams and RCCL collectives from torch.distributed interoperate with our kernels.
        import torch  # noqa: F401

        # DRT_LIBRARY: an alternative build of the same library (A/B runs in tools/ab.sh)
        path = Path(os.environ.get("DRT_LIBRARY") or LIB_PATH)
        if not path.exists():
            raise RuntimeError(f"{path} is missing: run distributionraytracer_amd._lib.build() "
                               "(make -C distributionraytracer_amd/csrc)")
        L = C.CDLL(str(path))
        alt = bool(os.environ.get("DRT_LIBRARY"))
        for name, (res, args) in SIGNATURES.items():
            if alt and not hasattr(L, name):
                continue  # an older A/B build may predate an entry point the run does not call
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, ctx=None, what=""):
    if rc != DRT_OK:
        msg = ""
        if ctx is not None:
            try:
                msg = load().drt_last_error(ctx).decode()
            except Exception:
                pass
        raise RuntimeError(f"{what} failed: {STATUS.get(rc, rc)} {msg}".strip())
