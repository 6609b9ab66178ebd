// drt_group.hip — several GPUs behind one C-ABI handle (include/drt.h, drt_group_*).
//
// pixels are independent (main.cpp:603) and the keyed RNG depends only on (seed,
// pixel, k), so a frame splits into interleaved 16x16 tiles dealt over the GPUs (the dealing of
// drt_frame_params.shard / n_shards).  A group holds one drt_ctx per device, one HIP stream per
// device and one RCCL communicator clique (ncclCommInitAll: one process drives every device).
// A frame is: every device renders its shard into an equal-size shard buffer on its own stream;
// one ncclAllGather of the shard buffers over xGMI (12 B x pixels / N per device); device 0
// reassembles the frame (drt_unshard_device).  The scene is replicated: the caller uploads it to
// every context (drt_group_ctx), or through drt_group_scene_upload (include/drt_host.h).
//
// RCCL is opened at run time (dlopen "librccl.so.1") the first time a group is created, so
// libdrt.so does not link it and shares the process's copy when one is already loaded
// (PyTorch's).  A one-device group takes the same path (its all-gather is a local copy), so the
// collective path is exercised on a one-GPU machine too; only progressive frames skip it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/drt.h"

namespace {

struct Rccl {  // the few RCCL entry points the group needs
  decltype(&ncclCommInitAll) commInitAll = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclAllGather) allGather = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  bool ok = false;
  std::string err;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      r.err = std::string("cannot load RCCL: ") + dlerror();
      return;
    }
    r.commInitAll = (decltype(r.commInitAll))dlsym(h, "ncclCommInitAll");
    r.commDestroy = (decltype(r.commDestroy))dlsym(h, "ncclCommDestroy");
    r.allGather = (decltype(r.allGather))dlsym(h, "ncclAllGather");
    r.groupStart = (decltype(r.groupStart))dlsym(h, "ncclGroupStart");
    r.groupEnd = (decltype(r.groupEnd))dlsym(h, "ncclGroupEnd");
    r.errorString = (decltype(r.errorString))dlsym(h, "ncclGetErrorString");
    r.ok = r.commInitAll && r.commDestroy && r.allGather && r.groupStart && r.groupEnd && r.errorString;
    if (!r.ok) r.err = "RCCL is missing an entry point";
  });
  return r;
}

}  // namespace

struct drt_group {
  int n = 0;
  std::vector<int> dev;
  std::vector<drt_ctx*> ctx;
  std::vector<hipStream_t> stream;
  std::vector<ncclComm_t> comm;     // one per device
  // per frame slot (drt_frame_params.slot) and device: its shard buffer, the all-gathered shards.
  // Frames on different slots own different buffers; a frame on a slot whose last frame ran on
  // another stream0 waits (on device 0) for that frame's reassembly, which reads them.
  std::vector<float*> shard[DRT_FRAME_SLOTS], gathered[DRT_FRAME_SLOTS];
  std::vector<size_t> shard_floats[DRT_FRAME_SLOTS];  // current allocation (floats per shard)
  hipEvent_t slot_done[DRT_FRAME_SLOTS] = {};          // device 0: after the slot's last unshard
  hipStream_t slot_stream[DRT_FRAME_SLOTS] = {};
  float* d_frame = nullptr;            // device 0: reassembled frame for drt_group_render
  size_t frame_floats = 0;
  std::string err;
};

#define G_FAIL(g, code, ...)                      \
  do {                                            \
    char _b[512];                                 \
    snprintf(_b, sizeof(_b), __VA_ARGS__);        \
    (g)->err = _b;                                \
    return (code);                                \
  } while (0)
#define G_HIP(g, expr)                                                                                 \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) G_FAIL(g, _e == hipErrorOutOfMemory ? DRT_E_OOM : DRT_E_HIP, "%s: %s", #expr, \
                                 hipGetErrorString(_e));                                               \
  } while (0)

extern "C" {

void drt_group_destroy(drt_group* g) {
  if (!g) return;
  for (int r = 0; r < g->n; r++) {
    (void)hipSetDevice(g->dev[r]);
    if (r < (int)g->stream.size() && g->stream[r]) (void)hipStreamSynchronize(g->stream[r]);
  }
  if (!g->comm.empty() && rccl().ok)
    for (ncclComm_t c : g->comm)
      if (c) rccl().commDestroy(c);
  for (int r = 0; r < g->n; r++) {
    (void)hipSetDevice(g->dev[r]);
    for (int k = 0; k < DRT_FRAME_SLOTS; k++) {
      if (r < (int)g->shard[k].size() && g->shard[k][r]) (void)hipFree(g->shard[k][r]);
      if (r < (int)g->gathered[k].size() && g->gathered[k][r]) (void)hipFree(g->gathered[k][r]);
      if (r == 0 && g->slot_done[k]) (void)hipEventDestroy(g->slot_done[k]);
    }
    if (r < (int)g->stream.size() && g->stream[r]) (void)hipStreamDestroy(g->stream[r]);
    if (r < (int)g->ctx.size() && g->ctx[r]) drt_destroy(g->ctx[r]);
  }
  if (g->d_frame) {
    (void)hipSetDevice(g->dev[0]);
    (void)hipFree(g->d_frame);
  }
  delete g;
}

int drt_group_create(drt_group** out, int n_devices, const int32_t* devices) {
  if (!out || n_devices <= 0) return DRT_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DRT_E_NODEVICE;
  std::vector<int> dev(n_devices);
  for (int r = 0; r < n_devices; r++) {
    dev[r] = devices ? devices[r] : r;
    if (dev[r] < 0 || dev[r] >= ndev) return DRT_E_INVALID;
    for (int q = 0; q < r; q++)
      if (dev[q] == dev[r]) return DRT_E_INVALID;  // RCCL: one rank per device
  }
  drt_group* g = new drt_group();
  g->n = n_devices;
  g->dev = dev;
  g->ctx.assign(n_devices, nullptr);
  g->stream.assign(n_devices, nullptr);
  for (int k = 0; k < DRT_FRAME_SLOTS; k++) {
    g->shard[k].assign(n_devices, nullptr);
    g->gathered[k].assign(n_devices, nullptr);
    g->shard_floats[k].assign(n_devices, 0);
  }
  for (int r = 0; r < n_devices; r++) {
    drt_options opt{};
    opt.device = dev[r];
    int rc = drt_create(&g->ctx[r], &opt);
    if (rc) {
      drt_group_destroy(g);
      return rc;
    }
    if (hipSetDevice(dev[r]) != hipSuccess || hipStreamCreateWithFlags(&g->stream[r], hipStreamNonBlocking) != hipSuccess) {
      drt_group_destroy(g);
      return DRT_E_HIP;
    }
  }
  (void)hipSetDevice(dev[0]);
  for (int k = 0; k < DRT_FRAME_SLOTS; k++)
    if (hipEventCreateWithFlags(&g->slot_done[k], hipEventDisableTiming) != hipSuccess) {
      drt_group_destroy(g);
      return DRT_E_HIP;
    }
  {  // every group, one device included, runs the same shard -> all-gather -> unshard path
    const Rccl& R = rccl();
    if (!R.ok) {
      drt_group_destroy(g);
      return DRT_E_UNSUPPORTED;
    }
    g->comm.assign(n_devices, nullptr);
    if (R.commInitAll(g->comm.data(), n_devices, dev.data()) != ncclSuccess) {
      g->comm.clear();
      drt_group_destroy(g);
      return DRT_E_HIP;
    }
  }
  *out = g;
  return DRT_OK;
}

const char* drt_group_last_error(const drt_group* g) { return g ? g->err.c_str() : "null group"; }

int drt_group_size(const drt_group* g) { return g ? g->n : DRT_E_INVALID; }

drt_ctx* drt_group_ctx(drt_group* g, int rank) { return (g && rank >= 0 && rank < g->n) ? g->ctx[rank] : nullptr; }

int drt_group_set_camera(drt_group* g, const drt_camera* camera) {
  if (!g || !camera) return DRT_E_INVALID;
  // validated once for every device before any device changes, so that a refusal leaves every
  // device on the old camera (a group frame never mixes tiles of two cameras); drt_set_camera's
  // checks are these
  if (camera->res_x <= 0 || camera->res_y <= 0) G_FAIL(g, DRT_E_INVALID, "camera resolution must be positive");
  for (int r = 0; r < g->n; r++) {
    int32_t res[2] = {0, 0};
    if (drt_frame_resolution(g->ctx[r], res) != DRT_OK) G_FAIL(g, DRT_E_STATE, "device %d: no scene uploaded", g->dev[r]);
    if (res[0] != camera->res_x || res[1] != camera->res_y)
      G_FAIL(g, DRT_E_INVALID, "device %d: camera resolution %dx%d differs from the resident %dx%d", g->dev[r],
             camera->res_x, camera->res_y, res[0], res[1]);
  }
  for (int r = 0; r < g->n; r++) {
    const int rc = drt_set_camera(g->ctx[r], camera);
    if (rc) G_FAIL(g, rc, "device %d: %s", g->dev[r], drt_last_error(g->ctx[r]));
  }
  return DRT_OK;
}

int drt_group_render_device(drt_group* g, const drt_frame_params* params, float* d_frame, void* stream0) {
  if (!g || !params || !d_frame) return DRT_E_INVALID;
  if (params->n_shards > 1) G_FAIL(g, DRT_E_INVALID, "the group deals the tiles itself: pass n_shards 0 or 1");
  // a progressive frame lerps into the previous one (main.cpp:574-586), which a sharded frame
  // would need scattered to the devices first: interactive zone A stays on one device
  if (g->n > 1 && params->progressive_frame > 0)
    G_FAIL(g, DRT_E_UNSUPPORTED, "progressive frames run on a one-device group");
  hipStream_t s0 = stream0 ? (hipStream_t)stream0 : g->stream[0];
  if (g->n == 1 && params->progressive_frame > 0) {  // zone A: the whole frame on the one device
    drt_frame_params p = *params;
    p.shard = 0;
    p.n_shards = 1;
    const int rc = drt_render_device(g->ctx[0], &p, d_frame, s0);
    if (rc) G_FAIL(g, rc, "device %d: %s", g->dev[0], drt_last_error(g->ctx[0]));
    return DRT_OK;
  }
  std::vector<drt_frame_params> p(g->n, *params);
  int64_t floats = 0;
  for (int r = 0; r < g->n; r++) {
    p[r].shard = r;
    p[r].n_shards = g->n;
    p[r].flags |= DRT_FRAME_SHARD_LAYOUT;  // shard-compact even when n == 1
    int64_t tiles = 0, f = 0;
    const int rc = drt_shard_layout(g->ctx[r], &p[r], &tiles, &f);
    if (rc) G_FAIL(g, rc, "device %d: %s", g->dev[r], drt_last_error(g->ctx[r]));
    if (r == 0) floats = f;
    else if (f != floats) G_FAIL(g, DRT_E_STATE, "devices hold different scenes (shard sizes %lld vs %lld)",
                                 (long long)f, (long long)floats);
  }
  const int slot = params->slot;
  if (slot < 0 || slot >= DRT_FRAME_SLOTS) G_FAIL(g, DRT_E_INVALID, "frame slot out of range");
  std::vector<float*>& shard = g->shard[slot];
  std::vector<float*>& gathered = g->gathered[slot];
  // the slot's buffers: the last frame on this slot may still be gathering / reassembling them on
  // another stream0 (devices r > 0 always use the group's own stream, which orders them)
  G_HIP(g, hipSetDevice(g->dev[0]));
  if (g->slot_stream[slot] && g->slot_stream[slot] != s0) G_HIP(g, hipStreamWaitEvent(s0, g->slot_done[slot], 0));
  // the frame's shards, each device on its own stream (device 0 on the caller's stream)
  for (int r = 0; r < g->n; r++) {
    G_HIP(g, hipSetDevice(g->dev[r]));
    if (g->shard_floats[slot][r] < (size_t)floats) {
      // regrowing: the slot's previous frame must be done with the old buffers on this device
      G_HIP(g, hipStreamSynchronize(r == 0 ? s0 : g->stream[r]));
      if (shard[r]) G_HIP(g, hipFree(shard[r]));
      if (gathered[r]) G_HIP(g, hipFree(gathered[r]));
      shard[r] = gathered[r] = nullptr;
      g->shard_floats[slot][r] = 0;
      G_HIP(g, hipMalloc(&shard[r], sizeof(float) * (size_t)floats));
      G_HIP(g, hipMalloc(&gathered[r], sizeof(float) * (size_t)floats * g->n));
      g->shard_floats[slot][r] = (size_t)floats;
    }
    const int rc = drt_render_device(g->ctx[r], &p[r], shard[r], r == 0 ? s0 : g->stream[r]);
    if (rc) G_FAIL(g, rc, "device %d: %s", g->dev[r], drt_last_error(g->ctx[r]));
  }
  // one all-gather of the shard buffers (each stream orders it after its device's shard)
  const Rccl& R = rccl();
  if (R.groupStart() != ncclSuccess) G_FAIL(g, DRT_E_HIP, "ncclGroupStart failed");
  for (int r = 0; r < g->n; r++) {
    const ncclResult_t e = R.allGather(shard[r], gathered[r], (size_t)floats, ncclFloat, g->comm[r],
                                       r == 0 ? s0 : g->stream[r]);
    if (e != ncclSuccess) {
      R.groupEnd();
      G_FAIL(g, DRT_E_HIP, "ncclAllGather: %s", R.errorString(e));
    }
  }
  const ncclResult_t e = R.groupEnd();
  if (e != ncclSuccess) G_FAIL(g, DRT_E_HIP, "ncclGroupEnd: %s", R.errorString(e));
  // device 0 reassembles the frame
  G_HIP(g, hipSetDevice(g->dev[0]));
  const int rc = drt_unshard_device(g->ctx[0], &p[0], gathered[0], d_frame, s0);
  if (rc) G_FAIL(g, rc, "unshard: %s", drt_last_error(g->ctx[0]));
  G_HIP(g, hipEventRecord(g->slot_done[slot], s0));
  g->slot_stream[slot] = s0;
  return DRT_OK;
}

int drt_group_render(drt_group* g, const drt_frame_params* params, float* rgb_out) {
  if (!g || !params || !rgb_out) return DRT_E_INVALID;
  drt_frame_plan plan;
  drt_frame_params p0 = *params;
  p0.n_shards = 1;
  p0.shard = 0;
  int rc = drt_plan_frame(g->ctx[0], &p0, &plan);  // fails without a scene
  if (rc) G_FAIL(g, rc, "device %d: %s", g->dev[0], drt_last_error(g->ctx[0]));
  if (params->progressive_frame >= 10000) return DRT_OK;  // MAX_SAMPLES: output untouched
  int32_t res[2];
  rc = drt_frame_resolution(g->ctx[0], res);
  if (rc) G_FAIL(g, rc, "%s", drt_last_error(g->ctx[0]));
  const size_t n = (size_t)res[0] * res[1] * 3;  // RES_Y * RES_X * 3 floats (main.cpp:710)
  G_HIP(g, hipSetDevice(g->dev[0]));
  if (g->frame_floats < n) {
    if (g->d_frame) G_HIP(g, hipFree(g->d_frame));
    g->d_frame = nullptr;
    g->frame_floats = 0;
    G_HIP(g, hipMalloc(&g->d_frame, sizeof(float) * n));
    g->frame_floats = n;
  }
  if (params->progressive_frame > 1)  // the lerp reads the previous frame
    G_HIP(g, hipMemcpyAsync(g->d_frame, rgb_out, sizeof(float) * n, hipMemcpyHostToDevice, g->stream[0]));
  rc = drt_group_render_device(g, params, g->d_frame, g->stream[0]);
  if (rc) return rc;
  G_HIP(g, hipSetDevice(g->dev[0]));
  G_HIP(g, hipMemcpyAsync(rgb_out, g->d_frame, sizeof(float) * n, hipMemcpyDeviceToHost, g->stream[0]));
  for (int r = 0; r < g->n; r++) {
    G_HIP(g, hipSetDevice(g->dev[r]));
    G_HIP(g, hipStreamSynchronize(g->stream[r]));
  }
  return DRT_OK;
}

int drt_group_synchronize(drt_group* g) {
  if (!g) return DRT_E_INVALID;
  for (int r = 0; r < g->n; r++) {
    G_HIP(g, hipSetDevice(g->dev[r]));
    G_HIP(g, hipStreamSynchronize(g->stream[r]));
  }
  return DRT_OK;
}

}  // extern "C"
