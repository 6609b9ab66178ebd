"""MI355X-native distribution ray tracer (drop-in for rita-mota/DistributionRayTracer's hot path).

Python host layer over libdrt.so:

  Scene     — P3F scenes (Scene::load_p3f, scene.cpp:474) or programmatic scenes; the host
              BVH / Grid build (bvh.cpp:27-227, grid.cpp:30-97) runs in C++.
  Renderer  — one HIP context on one gfx950 device: upload, render (renderScene,
              main.cpp:525-738), batched BVH/Grid Traverse queries, tile-sharded frames.

Everything that touches a ray runs in hand-written HIP kernels; there is no CPU render path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

from . import _lib
from ._lib import ACCEL, FRAME_REFERENCE_ORDER, FRAME_STATS, DrtCamera, DrtFrameParams, DrtFrameStats, DrtOptions, DrtSceneInfo, check

__all__ = ["Scene", "Renderer", "RendererGroup", "ACCEL", "load_skybox_dir", "SKY_FACES", "build"]

SKY_FACES = ("right", "left", "top", "bottom", "front", "back")  # scene.cpp:333, CubeMap enum


def build(force=False):
    return _lib.build(force=force)


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _fp(a):
    return a.ctypes.data_as(_lib._f)


def image_rgb8(frame):
    """u8fromfloat of a (RES_Y, RES_X, 3) float frame, row 0 = bottom (main.cpp:716-718)."""
    f = np.ascontiguousarray(frame, np.float32)
    out = np.empty(f.shape, np.uint8)
    check(_lib.load().drt_image_rgb8(f.ctypes.data, f.shape[1], f.shape[0], out.ctypes.data), what="drt_image_rgb8")
    return out


def write_png(path, frame):
    """saveImgFile (main.cpp:251-266): 8-bit RGB PNG, displayed upright (top row = frame row RES_Y-1)."""
    f = np.ascontiguousarray(frame, np.float32)
    check(_lib.load().drt_image_write_png(str(path).encode(), f.ctypes.data, f.shape[1], f.shape[0]),
          what="drt_image_write_png")


def load_skybox_dir(path, max_size=None):
    """Decode the six cube faces (DevIL in the reference, scene.cpp:329-378) with PIL, rows
    bottom-up (IL_ORIGIN_LOWER_LEFT)."""
    from PIL import Image

    faces = []
    for name in SKY_FACES:
        im = Image.open(os.path.join(path, name + ".jpg")).convert("RGB")
        if max_size is not None and im.width > max_size:
            im = im.resize((max_size, max_size), Image.NEAREST)
        faces.append(np.asarray(im, dtype=np.uint8)[::-1].copy())
    return faces


class Scene:
    """Host scene (drt_scene*): the reference's Scene + its accelerator."""

    def __init__(self, handle=None):
        L = _lib.load()
        self.h = C.c_void_p(handle if handle is not None else L.drt_scene_new())
        if not self.h:
            raise RuntimeError("scene creation failed")

    def __del__(self):
        try:
            if getattr(self, "h", None):
                _lib.load().drt_scene_free(self.h)
                self.h = None
        except Exception:
            pass

    @classmethod
    def load_p3f(cls, path, skybox_root=None, skybox_faces=None, skybox_max_size=None):
        L = _lib.load()
        h = L.drt_scene_load_p3f(str(path).encode())
        if not h:
            raise FileNotFoundError(path)
        s = cls(h)
        env = s.env
        if env:
            if skybox_faces is None and s.info().skybox_loaded:
                return s  # Scene::load_p3f's LoadSkybox found the faces (PPM / registered decoder)
            if skybox_faces is None:
                root = Path(skybox_root) if skybox_root else Path(path).resolve().parent.parent
                skybox_faces = load_skybox_dir(root / env, skybox_max_size)
            s.set_skybox(skybox_faces)
        return s

    @property
    def env(self):
        return _lib.load().drt_scene_env(self.h).decode()

    def set_skybox(self, faces):
        for i, a in enumerate(faces):
            a = np.ascontiguousarray(a, dtype=np.uint8)
            h, w, bpp = a.shape
            check(_lib.load().drt_scene_set_skybox_face(self.h, i, w, h, bpp, a.ctypes.data_as(_lib._u8)),
                  what="set_skybox")

    def info(self):
        i = DrtSceneInfo()
        check(_lib.load().drt_scene_info(self.h, C.byref(i)), what="scene_info")
        return i

    def set_camera(self, eye, at, up, fovy, hither, res_x, res_y, aperture=0.0, focal=1.0):
        check(_lib.load().drt_scene_set_camera(self.h, _fp(_f32(eye)), _fp(_f32(at)), _fp(_f32(up)), fovy, hither,
                                               res_x, res_y, aperture, focal), what="set_camera")

    def set_eye(self, eye):
        """Camera::SetEye (camera.h:63-72): the interactive camera motion of main.cpp:530-533."""
        check(_lib.load().drt_scene_set_eye(self.h, _fp(_f32(eye))), what="set_eye")

    def set_background(self, rgb):
        _lib.load().drt_scene_set_background(self.h, _fp(_f32(rgb)))

    def set_accel(self, accel):
        check(_lib.load().drt_scene_set_accel(self.h, ACCEL[accel] if isinstance(accel, str) else int(accel)),
              what="set_accel")

    def set_spp(self, spp):
        _lib.load().drt_scene_set_spp(self.h, int(spp))

    def add_material(self, diff, kd, spec, ks, shine, t, ior):
        return _lib.load().drt_scene_add_material(self.h, _fp(_f32(diff)), kd, _fp(_f32(spec)), ks, shine, t, ior)

    def add_sphere(self, c, r):
        return _lib.load().drt_scene_add_sphere(self.h, _fp(_f32(c)), r)

    def add_triangles(self, verts):
        v = _f32(verts).reshape(-1, 9)
        return _lib.load().drt_scene_add_triangles(self.h, _fp(v), len(v))

    def add_plane_pts(self, a, b, c):
        return _lib.load().drt_scene_add_plane_pts(self.h, _fp(_f32(a)), _fp(_f32(b)), _fp(_f32(c)))

    def add_plane_nd(self, n, d):
        return _lib.load().drt_scene_add_plane_nd(self.h, _fp(_f32(n)), d)

    def add_box(self, mn, mx):
        return _lib.load().drt_scene_add_box(self.h, _fp(_f32(mn)), _fp(_f32(mx)))

    def add_light_point(self, pos, rgb=(1, 1, 1)):
        return _lib.load().drt_scene_add_light_point(self.h, _fp(_f32(pos)), _fp(_f32(rgb)))

    def add_light_quad(self, pos, rgb, v1, v2, grid_res):
        return _lib.load().drt_scene_add_light_quad(self.h, _fp(_f32(pos)), _fp(_f32(rgb)), _fp(_f32(v1)),
                                                    _fp(_f32(v2)), grid_res)

    def build(self):
        check(_lib.load().drt_scene_build(self.h), what="scene_build")

    def camera_frame(self):
        c = DrtCamera()
        check(_lib.load().drt_scene_camera_frame(self.h, C.byref(c)), what="camera_frame")
        return c

    def bvh_export(self):
        n = self.info().bvh_nodes
        no = self.info().n_objects
        boxes = np.zeros((n, 6), np.float32)
        leaf = np.zeros(n, np.uint32)
        index = np.zeros(n, np.uint32)
        nobj = np.zeros(n, np.uint32)
        order = np.zeros(no, np.int32)
        check(_lib.load().drt_scene_bvh_export(self.h, _fp(boxes), leaf.ctypes.data_as(_lib._u32),
                                               index.ctypes.data_as(_lib._u32), nobj.ctypes.data_as(_lib._u32),
                                               order.ctypes.data_as(_lib._i32)), what="bvh_export")
        return dict(boxes=boxes, leaf=leaf, index=index, nobjs=nobj, order=order)

    def trace_cpu(self, rays, shadow=False):
        """The scalar host path (BVH::Traverse / Grid::Traverse / the NONE scan on the CPU, one ray
        at a time): closest -> (t, normal, object); shadow -> occluded (uint8)."""
        r = _f32(rays).reshape(-1, 6)
        n = len(r)
        L = _lib.load()
        if shadow:
            occ = np.zeros(n, np.uint8)
            check(L.drt_scene_trace_cpu(self.h, 1, _fp(r), n, None, None, None, occ.ctypes.data_as(_lib._u8)),
                  what="trace_cpu")
            return occ
        t = np.zeros(n, np.float32)
        nrm = np.zeros((n, 3), np.float32)
        obj = np.zeros(n, np.int32)
        check(L.drt_scene_trace_cpu(self.h, 0, _fp(r), n, _fp(t), _fp(nrm), obj.ctypes.data_as(_lib._i32), None),
              what="trace_cpu")
        return t, nrm, obj

    def skybox_color_cpu(self, dirs):
        """Scene::GetSkyboxColor for n directions (n x 3 floats)."""
        d = _f32(dirs).reshape(-1, 3)
        out = np.zeros((len(d), 3), np.float32)
        check(_lib.load().drt_scene_skybox_color_cpu(self.h, _fp(d), len(d), _fp(out)), what="skybox_color_cpu")
        return out

    def load_skybox(self, sky_dir):
        """Scene::LoadSkybox: <dir>/<face>.ppm (or .jpg through a registered decoder)."""
        check(_lib.load().drt_scene_load_skybox(self.h, str(sky_dir).encode()), what="load_skybox")

    def grid_export(self):
        L = _lib.load()
        dims = np.zeros(3, np.int32)
        bmin = np.zeros(3, np.float32)
        bmax = np.zeros(3, np.float32)
        nref = C.c_int64()
        check(L.drt_scene_grid_export_dims(self.h, dims.ctypes.data_as(_lib._i32), _fp(bmin), _fp(bmax),
                                           C.byref(nref)), what="grid_export")
        cs = np.zeros(int(np.prod(dims)) + 1, np.int64)
        co = np.zeros(nref.value, np.int32)
        check(L.drt_scene_grid_export(self.h, cs.ctypes.data_as(_lib._i64), co.ctypes.data_as(_lib._i32)),
              what="grid_export")
        return dict(dims=tuple(int(d) for d in dims), bmin=bmin, bmax=bmax, cell_start=cs, cell_objs=co)


class Renderer:
    """One HIP context (drt_ctx*) on one gfx950 device."""

    def __init__(self, device=0):
        L = _lib.load()
        opt = DrtOptions()
        opt.device = int(device)
        h = C.c_void_p()
        rc = L.drt_create(C.byref(h), C.byref(opt))
        if rc != 0:
            raise RuntimeError(f"drt_create(device={device}) failed: {_lib.STATUS.get(rc, rc)} "
                               "(a gfx950 / MI355X device is required; there is no CPU path)")
        self.h = h
        self.scene = None

    def close(self):
        if getattr(self, "h", None):
            _lib.load().drt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene: Scene):
        check(_lib.load().drt_scene_upload(self.h, scene.h), self.h, "drt_scene_upload")
        self.scene = scene
        return self

    def set_camera(self, camera=None):
        """drt_set_camera: the uploaded scene's camera alone (the per-frame SetEye of the interactive
        renderer, main.cpp:530-533); `camera` is a Scene (its current camera) or a DrtCamera frame,
        default the uploaded Scene.  Primitives and the accelerator stay resident."""
        cam = self.scene if camera is None else camera
        if isinstance(cam, Scene):
            check(_lib.load().drt_scene_upload_camera(self.h, cam.h), self.h, "drt_scene_upload_camera")
        else:
            check(_lib.load().drt_set_camera(self.h, C.byref(cam)), self.h, "drt_set_camera")
        return self

    def frame_params(self, seed=1, max_depth=4, roughness=0.0, shard=0, n_shards=1, tile=16, stats=False,
                     light_spp=1, progressive_frame=0, slot=0, reference_order=False):
        p = DrtFrameParams()
        p.slot = slot
        p.light_spp = light_spp
        p.progressive_frame = progressive_frame
        p.seed = seed
        p.max_depth = max_depth
        p.roughness = roughness
        p.shard = shard
        p.n_shards = n_shards
        p.tile = tile
        p.flags = (FRAME_STATS if stats else 0) | (FRAME_REFERENCE_ORDER if reference_order else 0)
        return p

    def render(self, seed=1, max_depth=4, roughness=0.0, stats=False, tile=16, light_spp=1, progressive_frame=0,
               accum=None, reference_order=False):
        """Whole frame to host memory.  progressive_frame n >= 1: zone A frame n lerped into
        `accum` (updated in place and returned).  reference_order: shadow queries walk the
        reference's binary tree in its visit order (DRT_FRAME_REFERENCE_ORDER), so stats() counts
        the reference's shadow work; the frame is the same either way."""
        info = self.scene.info()
        if accum is not None:
            if accum.dtype != np.float32 or accum.shape != (info.res_y, info.res_x, 3) or not accum.flags.c_contiguous:
                raise ValueError("accum must be a C-contiguous float32 (res_y, res_x, 3) array")
            out = accum
        else:
            out = np.zeros((info.res_y, info.res_x, 3), np.float32)
        p = self.frame_params(seed, max_depth, roughness, tile=tile, stats=stats, light_spp=light_spp,
                              progressive_frame=progressive_frame, reference_order=reference_order)
        check(_lib.load().drt_render(self.h, C.byref(p), _fp(out)), self.h, "drt_render")
        return out

    def plan(self, params):
        """drt_plan_frame: work items, sample slots, mode and kernel choice of a frame (no device work)."""
        out = _lib.DrtFramePlan()
        check(_lib.load().drt_plan_frame(self.h, C.byref(params), C.byref(out)), self.h, "drt_plan_frame")
        return dict(work_items=int(out.work_items), sample_slots=int(out.sample_slots), mode=int(out.mode),
                    persistent=bool(out.persistent), tiles_in_shard=int(out.tiles_in_shard), passes=int(out.passes), wavefront=bool(out.wavefront))

    def render_device(self, params, d_out_ptr, stream=None):
        """Asynchronous: shard (or whole frame) into a device pointer on `stream` (int handle)."""
        check(_lib.load().drt_render_device(self.h, C.byref(params), C.c_void_p(d_out_ptr),
                                            C.c_void_p(stream or 0)), self.h, "drt_render_device")

    def shard_layout(self, params):
        tiles = C.c_int64()
        floats = C.c_int64()
        check(_lib.load().drt_shard_layout(self.h, C.byref(params), C.byref(tiles), C.byref(floats)), self.h,
              "drt_shard_layout")
        return tiles.value, floats.value

    def unshard_device(self, params, d_shards_ptr, d_frame_ptr, stream=None):
        check(_lib.load().drt_unshard_device(self.h, C.byref(params), C.c_void_p(d_shards_ptr),
                                             C.c_void_p(d_frame_ptr), C.c_void_p(stream or 0)), self.h,
              "drt_unshard_device")

    def stats(self):
        s = DrtFrameStats()
        check(_lib.load().drt_get_stats(self.h, C.byref(s)), self.h, "drt_get_stats")
        return s.as_dict()

    def frame_times(self, max_frames=512):
        """(path-kernel ms, kernel+reduce ms) per recent frame, oldest first (HIP events)."""
        a = (C.c_double * max_frames)()
        b = (C.c_double * max_frames)()
        n = _lib.load().drt_frame_times(self.h, max_frames, a, b)
        if n < 0:
            check(n, self.h, "drt_frame_times")
        return np.array(a[:n]), np.array(b[:n])

    def frame_pass_times(self, max_frames=512):
        """(pass-1 ms, pass-2 ms) per recent frame, oldest first (HIP events): a two-pass frame's
        closest-chain and replay launches; a one-pass frame's kernel and 0."""
        a = (C.c_double * max_frames)()
        b = (C.c_double * max_frames)()
        n = _lib.load().drt_frame_pass_times(self.h, max_frames, a, b)
        if n < 0:
            check(n, self.h, "drt_frame_pass_times")
        return np.array(a[:n]), np.array(b[:n])

    def frame_stage_times(self):
        """{wf_gen, stream, wf_combine} ms of the last wavefront frame's pass-2 launches (drt_frame_stage_times)."""
        out = (C.c_double * 3)()
        n = _lib.load().drt_frame_stage_times(self.h, out)
        if n < 0:
            check(n, self.h, "drt_frame_stage_times")
        return {"wf_gen": out[0], "stream": out[1], "wf_combine": out[2], "chunks": n}

    def wave_times(self, pass_index=0, max_waves=1 << 14):
        """Per resident wave of the last stats frame's persistent launch (pass 0 or 1): (start, end)
        s_memrealtime stamps in us (100 MHz clock), rows of waves that ran; (drt_frame_wave_times)."""
        buf = (C.c_uint64 * (2 * max_waves))()
        n = _lib.load().drt_frame_wave_times(self.h, pass_index, buf, max_waves)
        if n < 0:
            check(n, self.h, "drt_frame_wave_times")
        a = np.frombuffer(buf, dtype=np.uint64, count=2 * n).reshape(n, 2)
        a = a[(a[:, 0] > 0) & (a[:, 1] > 0)]
        return a.astype(np.float64) / 100.0

    def frame_spans(self, max_frames=512):
        """(path start, path end, frame end) of recent frames in ms on one device clock, from the
        oldest frame's path-kernel start (HIP events on each frame's stream)."""
        a, b, e = ((C.c_double * max_frames)() for _ in range(3))
        n = _lib.load().drt_frame_spans(self.h, max_frames, a, b, e)
        if n < 0:
            check(n, self.h, "drt_frame_spans")
        return np.array(a[:n]), np.array(b[:n]), np.array(e[:n])

    def trace_closest(self, rays):
        r = _f32(rays).reshape(-1, 6)
        n = len(r)
        t = np.zeros(n, np.float32)
        nrm = np.zeros((n, 3), np.float32)
        obj = np.zeros(n, np.int32)
        check(_lib.load().drt_trace_closest(self.h, _fp(r), n, _fp(t), _fp(nrm), obj.ctypes.data_as(_lib._i32)),
              self.h, "drt_trace_closest")
        return t, nrm, obj

    def trace_shadow(self, rays):
        r = _f32(rays).reshape(-1, 6)
        occ = np.zeros(len(r), np.uint8)
        check(_lib.load().drt_trace_shadow(self.h, _fp(r), len(r), occ.ctypes.data_as(_lib._u8)), self.h,
              "drt_trace_shadow")
        return occ

    def trace_device(self, shadow, d_rays, n, d_t=0, d_normal=0, d_object=0, d_occluded=0, stream=None):
        """Asynchronous batched queries on device pointers (ints), on `stream` (int handle)."""
        v = C.c_void_p
        check(_lib.load().drt_trace_device(self.h, int(bool(shadow)), v(d_rays), int(n), v(d_t), v(d_normal),
                                           v(d_object), v(d_occluded), v(stream or 0)), self.h, "drt_trace_device")

    def set_trace_stats(self, on=True, reference_order=False):
        """Count traversal work (rays, nodes, leaves, primitives) of later batched queries;
        reference_order: later shadow queries walk the reference's binary tree."""
        flags = (FRAME_STATS if on else 0) | (FRAME_REFERENCE_ORDER if reference_order else 0)
        check(_lib.load().drt_set_trace_flags(self.h, flags), self.h, "drt_set_trace_flags")

    def trace_stats(self):
        """Streaming-kernel time (kernel_ms) and counters of the last BVH batched query."""
        s = DrtFrameStats()
        check(_lib.load().drt_trace_stats(self.h, C.byref(s)), self.h, "drt_trace_stats")
        return s.as_dict()


class RendererGroup:
    """Several GPUs behind one handle (drt_group_*, include/drt.h): the scene replicated on every
    device, each frame tile-sharded over them, all-gathered over RCCL and reassembled on the first
    device — a single process, no torch.distributed."""

    def __init__(self, devices):
        L = _lib.load()
        devs = list(devices)
        arr = (C.c_int32 * len(devs))(*devs)
        h = C.c_void_p()
        rc = L.drt_group_create(C.byref(h), len(devs), arr)
        if rc != 0:
            raise RuntimeError(f"drt_group_create({devs}) failed: {_lib.STATUS.get(rc, rc)}")
        self.h = h
        self.devices = devs
        self.scene = None

    def close(self):
        if getattr(self, "h", None):
            _lib.load().drt_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: {_lib.STATUS.get(rc, rc)} "
                               f"{_lib.load().drt_group_last_error(self.h).decode()}".strip())

    def upload(self, scene: Scene):
        self._check(_lib.load().drt_group_scene_upload(self.h, scene.h), "drt_group_scene_upload")
        self.scene = scene
        return self

    def set_camera(self, camera=None):
        """drt_group_set_camera on every device (see Renderer.set_camera)."""
        cam = self.scene if camera is None else camera
        if isinstance(cam, Scene):
            self._check(_lib.load().drt_group_scene_upload_camera(self.h, cam.h), "drt_group_scene_upload_camera")
        else:
            self._check(_lib.load().drt_group_set_camera(self.h, C.byref(cam)), "drt_group_set_camera")
        return self

    def render(self, seed=1, max_depth=4, roughness=0.0, light_spp=1, progressive_frame=0, accum=None, slot=0):
        info = self.scene.info()
        out = accum if accum is not None else np.zeros((info.res_y, info.res_x, 3), np.float32)
        p = DrtFrameParams()
        p.seed, p.max_depth, p.roughness, p.light_spp, p.progressive_frame = seed, max_depth, roughness, light_spp, \
            progressive_frame
        p.slot = slot
        self._check(_lib.load().drt_group_render(self.h, C.byref(p), _fp(out)), "drt_group_render")
        return out

    def render_device(self, d_frame_ptr, seed=1, max_depth=4, roughness=0.0, light_spp=1, stream=None, slot=0):
        p = DrtFrameParams()
        p.seed, p.max_depth, p.roughness, p.light_spp = seed, max_depth, roughness, light_spp
        p.slot = slot
        self._check(_lib.load().drt_group_render_device(self.h, C.byref(p), C.c_void_p(d_frame_ptr),
                                                        C.c_void_p(stream or 0)), "drt_group_render_device")

    def synchronize(self):
        self._check(_lib.load().drt_group_synchronize(self.h), "drt_group_synchronize")
