// drt_capi.hip — the C ABI of include/drt.h: device memory, uploads, frame orchestration.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "drt_kernels.hpp"
#include "drt_layout.hpp"

namespace drt {
void launch_path(const SceneArgs& S, const FrameArgs& F, int accel, bool tri_only, bool stats, hipStream_t st);
void launch_shuffle(const FrameArgs& F, int res_x, int res_y, uint8_t* perm, hipStream_t st);
void launch_reduce(const ReduceArgs& A, hipStream_t st);
void launch_unshard(const float* shards, float* frame, int tile, int tiles_x, int n_tiles, int n_shards,
                    int tiles_per_shard, int res_x, int res_y, hipStream_t st);
bool persistent_supported(int accel, const int gdim[3]);
void launch_path_persistent(const SceneArgs& S, const FrameArgs& F, int accel, bool tri_only, bool stats,
                            hipStream_t st);
void launch_trace_stream(const SceneArgs& S, const TraceArgs& A, bool shadow, bool tri_only, bool stats, int waves,
                         hipStream_t st);
void launch_trace_prep(const float* rays, int n, int shadow, float4* out, hipStream_t st);
void launch_wf_gen(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, hipStream_t st);
void launch_grid_stream(const SceneArgs& S, const TraceArgs& A, bool tri_only, bool stats, int waves, int walk, int pairs,
                        hipStream_t st);
void launch_grid_tree_stream(const SceneArgs& ST_, const SceneArgs& SG, const TraceArgs& A, bool stats, int waves,
                             int walk, int pairs, unsigned int* fb_counter, hipStream_t st);
void launch_wf_combine(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, hipStream_t st);
void launch_wf_combine_reduce(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, const ReduceArgs& R,
                              hipStream_t st);
void launch_trace_finish(const SceneArgs& S, const float4* q, int n, float* t, const uint32_t* prim, float* nrm,
                         int32_t* obj, hipStream_t st);
void launch_trace(const SceneArgs& S, int accel, bool tri_only, const float* rays, int n, int shadow, float* t,
                  float* nrm, int32_t* obj, uint8_t* occ, hipStream_t st);
}  // namespace drt

using namespace drt;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  hipError_t ensure(size_t n) {  // grow-only
    if (n <= bytes && p) return hipSuccess;
    release();
    hipError_t e = hipMalloc(&p, n ? n : 16);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  hipError_t fit(size_t n) {  // grow, and give back a buffer far larger than this use needs
    if (p && bytes > 4 * n + (256u << 20)) release();
    if (n <= bytes && p) return hipSuccess;
    release();
    hipError_t e = hipMalloc(&p, n ? n : 16);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

}  // namespace

struct drt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // per-frame HIP events (path-kernel start, path-kernel end / reduce start, frame end),
  // a ring so every frame of a timed loop can be read back afterwards
  static constexpr int kRing = 512;
  static constexpr int kEv = 4;  // events per frame: start, path end, frame end, end of pass 1
  std::vector<hipEvent_t> ring;
  uint64_t frames = 0;
  std::string err;
  // scene
  bool has_scene = false;
  drt_camera cam{};
  int accel = DRT_ACCEL_NONE;
  uint32_t spp = 0;
  float bg[3] = {0, 0, 0};
  bool tri_only = true;
  int n_prims = 0;
  std::vector<PrimRecord> prims_scene;  // scene order
  std::vector<drt_light> lights;
  std::vector<drt_material> mats;
  DevBuf d_prims, d_lights, d_mats, d_sky[6];
  int has_sky = 0, sky_w[6] = {0}, sky_h[6] = {0}, sky_bpp[6] = {0};
  // BVH
  bool has_bvh = false;
  DevBuf d_nodes, d_big;
  float root_box[6] = {0};
  uint32_t root_desc = 0;
  int bvh_depth = 0;
  // 4-ary shadow tree collapsed from the BVH (drt_layout.hpp); absent for a leaf root, a tree too
  // deep for the shadow stack, coordinates no record can quantise, or DRT_WIDE_SHADOW=0
  bool has_wide = false;
  DevBuf d_wnodes, d_wleaf;
  // stats frames: per resident wave of each path_persistent launch (pass 1, then pass 2) its (start, end)
  // s_memrealtime stamps (drt_frame_wave_times); wave_slots = waves per pass
  DevBuf d_wave_times;
  uint32_t wave_slots = 0;
  // the last wavefront frame's launches: per chunk (<= kStageChunks) the events after its wf_gen, its
  // shadow-query stream and its wf_combine (drt_frame_stage_times); stage_chunks = chunks recorded
  static constexpr int kStageChunks = 64;
  std::vector<hipEvent_t> stage_ev;
  int stage_chunks = 0;
  int stage_frame_ev = -1;  // ring slot of that frame (its end-of-pass-1 event opens chunk 0)
  uint32_t wroot = 0, n_wide = 0;
  // grid
  bool has_grid = false;
  int gdim[3] = {0, 0, 0};
  float gmin[3] = {0}, gmax[3] = {0};
  DevBuf d_cell_start, d_cell_objs, d_macro, d_cell_recs;
  DevBuf d_gprims, d_cell_pos;  // indexed Grid layout (experiment): Morton-ordered records, per-reference positions
  DevBuf d_cell_tris, d_cell_tpos;  // triangle scenes: 40-B triangles in pairs per cell, pair-aligned cell starts
  int gmacro_shift = 0, gmacro_dim[3] = {0, 0, 0}, gmacro_words = 0;
  // per scene object its cell range (ix_min, iy_min, iz_min, ix_max, iy_max, iz_max), from the cell lists
  std::vector<int32_t> grid_cells;
  // the Grid scene's shadow tree (drt_upload_grid_shadow_bvh, triangle scenes): 4-ary records with
  // widened child boxes, the primitives in its BVH's order, per such primitive its cell range (32-B
  // LeafBoxRecord-shaped records read by the certificate), its big-leaf table
  bool has_gv = false;
  DevBuf d_gv_wnodes, d_gv_range, d_gv_prims, d_gv_big;
  uint32_t gv_wroot = 0;
  // frame scratch
  DevBuf d_frame, d_rays, d_out, d_counter;
  // frame scratch per slot (drt_frame_params.slot): frames on different slots may be in flight
  // together on different streams
  DevBuf d_samples_s[DRT_FRAME_SLOTS], d_stats_s[DRT_FRAME_SLOTS], d_counter_s[DRT_FRAME_SLOTS], d_perm_s[DRT_FRAME_SLOTS];
  // MODE_SEQ tail continuation slots per frame slot (FrameArgs::seq_cont), one per resident lane
  DevBuf d_cont_s[DRT_FRAME_SLOTS];
  // two-pass in-order frames: per sample slot its stream position, per slot and bounce its closest hit
  DevBuf d_skel_rk_s[DRT_FRAME_SLOTS], d_skel_hits_s[DRT_FRAME_SLOTS];
  DevBuf d_heads_s[DRT_FRAME_SLOTS];  // replay passes: frame heads, max_depth + 1 per resident lane
  // wavefront replay (WfArgs): shadow queries, their Phong factors and answers, per-level records
  DevBuf d_wf_rays_s[DRT_FRAME_SLOTS], d_wf_nl_s[DRT_FRAME_SLOTS], d_wf_occ_s[DRT_FRAME_SLOTS], d_wf_lvl_s[DRT_FRAME_SLOTS];
  DevBuf d_wf_cnt_s[DRT_FRAME_SLOTS];  // compact queries: per (band, level, 64-slot group) the group's query count
  DevBuf d_wf_fb_s[DRT_FRAME_SLOTS];   // the Grid shadow tree's undecided queries (TraceArgs::fb_rays)
  int cus = 0;  // compute units of the device (sizes the continuation slots)
  int stats_slot = 0;  // slot of the last frame (drt_get_stats reads its counters)
  drt_frame_stats last{};
  bool stats_valid = false;  // the last frame ran with DRT_FRAME_STATS
  // batched queries: streaming-query records, primitive results, timing of the last call
  DevBuf d_tq, d_tprim, d_tstats;
  // tev: streaming-kernel start / end, query done.  Batched queries on one context share these
  // buffers and the claim counter, so each query waits for the previous one (tev[2]) on its own
  // stream, and a buffer is only regrown once that query has finished.
  hipEvent_t tev[3] = {nullptr, nullptr, nullptr};
  bool trace_issued = false;  // tev[2] has been recorded
  int trace_flags = 0;        // DRT_FRAME_STATS: count traversal work of batched queries
  bool trace_timed = false;   // the last batched query ran the streaming kernel
  bool trace_stats_valid = false;
  // A frame's shuffle and reduce kernels run on a high-priority auxiliary stream per slot, linked
  // to the caller's stream by events: with frames in flight, the persistent kernels of the other
  // frames hold every CU, and on the caller's stream these small kernels queued behind their
  // pending blocks for milliseconds, stalling the next frame of that stream (kernel trace of
  // 8-way shard frames).  ev_path marks the slot's last path kernel (the next
  // shuffle of that slot rewrites the permutation it reads).
  hipStream_t aux[DRT_FRAME_SLOTS] = {};
  hipEvent_t ev_shuf[DRT_FRAME_SLOTS] = {}, ev_path[DRT_FRAME_SLOTS] = {}, ev_red[DRT_FRAME_SLOTS] = {};
  // ev_path[slot] is recorded after EVERY path kernel of the slot (aux frame or not), so an aux
  // shuffle that rewrites the slot's permutation always waits for the last kernel reading it
  bool path_issued[DRT_FRAME_SLOTS] = {};
  // The slot's last frame: its ring entry (frame number) and the stream it ran on.  A frame on the
  // same slot from another stream waits for that frame's end event first (its samples, counters
  // and permutation are the slot's scratch).
  uint64_t slot_frame[DRT_FRAME_SLOTS] = {};
  hipStream_t slot_stream[DRT_FRAME_SLOTS] = {};
  bool slot_used[DRT_FRAME_SLOTS] = {};
  // MODE_SEQ hand-over of the slot's last frame (drt_frame_stats.seq_handover)
  bool slot_handover[DRT_FRAME_SLOTS] = {};
  // The auxiliary streams cost each frame ~0.17 ms of cross-stream event latency, which only
  // pays for itself on long frames: they are used once a completed frame's path kernel took
  // >= kAuxMinMs (DRT_AUX_STREAMS=0 / 1 forces them off / on).  -1 = no completed frame yet.
  static constexpr double kAuxMinMs = 4.0;
  double last_path_ms = -1.0;
};

#define DRT_FAIL(ctx, code, ...)                                        \
  do {                                                                  \
    char _b[512];                                                       \
    snprintf(_b, sizeof(_b), __VA_ARGS__);                              \
    (ctx)->err = _b;                                                    \
    return (code);                                                      \
  } while (0)
#define DRT_HIP(ctx, expr)                                                                            \
  do {                                                                                                \
    hipError_t _e = (expr);                                                                           \
    if (_e != hipSuccess) DRT_FAIL(ctx, _e == hipErrorOutOfMemory ? DRT_E_OOM : DRT_E_HIP, "%s: %s", \
                                   #expr, hipGetErrorString(_e));                                     \
  } while (0)

static int env_int(const char* name, int dflt) {  // tuning knobs for A/B runs
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}
static uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  return (v && *v) ? strtoull(v, nullptr, 0) : dflt;
}

static PrimRecord pack_prim(const drt_prim& p, uint32_t mat, uint32_t obj) {
  PrimRecord r{};
  float* q = r.q;
  q[0] = p.a[0]; q[1] = p.a[1]; q[2] = p.a[2];
  q[3] = bits_as_float((uint32_t)(p.type & 3) | (mat << 2));
  q[7] = bits_as_float(obj);
  switch (p.type) {
    case DRT_PRIM_TRIANGLE:  // edge1 = P1 - P0, edge2 = P2 - P0 (scene.cpp:59-60)
      q[4] = p.b[0] - p.a[0]; q[5] = p.b[1] - p.a[1]; q[6] = p.b[2] - p.a[2];
      q[8] = p.c[0] - p.a[0]; q[9] = p.c[1] - p.a[1]; q[10] = p.c[2] - p.a[2];
      break;
    case DRT_PRIM_SPHERE:
    case DRT_PRIM_PLANE:
      q[4] = p.r;
      break;
    default:
      q[4] = p.b[0]; q[5] = p.b[1]; q[6] = p.b[2];
      break;
  }
  return r;
}

// ---- 4-ary shadow tree (drt_layout.hpp) -------------------------------------------------------
// One axis of a wide node: the coarsest-needed power-of-two scale s = 2^E and anchor p = k * s such
// that every child's [lo, hi] is covered by [p + ql * s, p + qh * s] with 0 <= ql, qh <= 255 and
// every such plane an exact float (|k| + 255 < 2^24).  False if no exponent fits (non-finite or
// enormous coordinates): the scene then keeps the binary tree for its shadow queries.
static bool quantize_axis(const double* lo, const double* hi, int n, float& p, uint32_t& ebits, uint32_t* qlo,
                          uint32_t* qhi) {
  double nlo = lo[0], nhi = hi[0];
  for (int k = 1; k < n; k++) {
    nlo = std::min(nlo, lo[k]);
    nhi = std::max(nhi, hi[k]);
  }
  if (!std::isfinite(nlo) || !std::isfinite(nhi) || nhi < nlo) return false;
  // the device's one-fma child test assumes |anchor| <= 2^60 and scale <= 2^50 (node_step)
  if (std::fabs(nlo) > 0x1p59 || std::fabs(nhi) > 0x1p59) return false;
  int e0 = -126;
  if (nhi > nlo) e0 = std::max(-126, std::ilogb((nhi - nlo) / 255.0) - 1);
  for (int E = e0; E <= 120; E++) {
    const double s = std::ldexp(1.0, E);
    const double k0 = std::floor(nlo / s);
    if (std::fabs(k0) + 256.0 >= 16777216.0) continue;
    uint32_t L[kWideW] = {}, H[kWideW] = {};  // byte k & 3 of word k >> 2: child k
    bool ok = true;
    const float pf = (float)(k0 * s), sf = (float)s;
    if ((double)pf != k0 * s) continue;
    if (E > 50) return false;
    for (int k = 0; k < kWideK && ok; k++) {
      if (k >= n) {  // unused slot: an inverted box (lo 255 > hi 0)
        L[k >> 2] |= 255u << (8 * (k & 3));
        continue;
      }
      const double ql = std::floor(lo[k] / s) - k0, qh = std::ceil(hi[k] / s) - k0;
      if (ql < 0.0 || qh > 255.0) {
        ok = false;
        break;
      }
      // the device decodes with one FMA; every value here is exact, so check it as the device does
      const float dl = std::fma((float)ql, sf, pf), dh = std::fma((float)qh, sf, pf);
      if (!((double)dl <= lo[k]) || !((double)dh >= hi[k]) || !std::isfinite(dl) || !std::isfinite(dh)) {
        ok = false;
        break;
      }
      L[k >> 2] |= (uint32_t)ql << (8 * (k & 3));
      H[k >> 2] |= (uint32_t)qh << (8 * (k & 3));
    }
    if (!ok) continue;
    p = pf;
    ebits = (uint32_t)(E + 127);
    for (int w = 0; w < kWideW; w++) {
      qlo[w] = L[w];
      qhi[w] = H[w];
    }
    return true;
  }
  return false;
}

// The shadow tree answers exactly as the reference's tree only if every child box lies inside its
// parent's box and every primitive sits in exactly one leaf.  The reference's build
// guarantees both (bvh.cpp:206-220: a node's box is the union of its objects' boxes); a caller's
// tree that breaks either — or shares a subtree between two parents, which the collapse would copy
// once per parent — keeps the binary tree for its shadow queries.
static bool wide_tree_valid(const drt_bvh_node* nodes, uint32_t n_nodes, uint32_t n_obj) {
  std::vector<uint8_t> seen(n_nodes, 0), covered(n_obj, 0);
  std::vector<uint32_t> st{0u};
  seen[0] = 1;
  uint64_t leaf_objs = 0;
  while (!st.empty()) {
    const uint32_t i = st.back();
    st.pop_back();
    const drt_bvh_node& nd = nodes[i];
    if (nd.leaf) {
      for (uint32_t k = 0; k < nd.n_objs; k++) {
        if (covered[nd.index + k]) return false;
        covered[nd.index + k] = 1;
      }
      leaf_objs += nd.n_objs;
      continue;
    }
    for (uint32_t c = nd.index; c < nd.index + 2; c++) {
      if (seen[c]) return false;
      seen[c] = 1;
      for (int a = 0; a < 3; a++)
        if (!(nodes[c].bmin[a] >= nd.bmin[a]) || !(nodes[c].bmax[a] <= nd.bmax[a])) return false;
      st.push_back(c);
    }
  }
  return leaf_objs == n_obj;
}

// Collapse the reference's binary tree (nodes, leaf descriptors per node) into 4-ary records: a
// wide node's children are its binary node's two children, the inner one with the largest box
// surface replaced by its two children until there are four (or only leaves).  Records in depth-
// first order.  False if a record cannot be quantised or 3 * depth would overflow the shadow stack.
// widen > 0 (the Grid scene's tree, drt_upload_grid_shadow_bvh): every child box grown by widen on each side.
static bool build_wide(const drt_bvh_node* nodes, const std::vector<uint32_t>& leaf_descs,
                       std::vector<WideNodeRecord>& out, uint32_t& root, double widen = 0.0) {
  out.clear();
  if (nodes[0].leaf) return false;
  auto area = [&](uint32_t i) {
    const drt_bvh_node& nd = nodes[i];
    const double x = (double)nd.bmax[0] - nd.bmin[0], y = (double)nd.bmax[1] - nd.bmin[1],
                 z = (double)nd.bmax[2] - nd.bmin[2];
    return x * y + y * z + z * x;
  };
  struct Item {
    uint32_t node, slot;
    int depth;
  };
  std::vector<Item> st{{0u, 0u, 1}};
  const int order = env_int("DRT_WIDE_ORDER", 2);
  out.emplace_back();
  int maxd = 1;
  while (!st.empty()) {
    const Item it = st.back();
    st.pop_back();
    maxd = std::max(maxd, it.depth);
    uint32_t ch[kWideK];
    int n = 2;
    ch[0] = nodes[it.node].index;
    ch[1] = ch[0] + 1;
    while (n < kWideK) {
      int best = -1;
      double ba = -1.0;
      for (int k = 0; k < n; k++)
        if (!nodes[ch[k]].leaf && area(ch[k]) > ba) {
          ba = area(ch[k]);
          best = k;
        }
      if (best < 0) break;
      const uint32_t c = ch[best];
      ch[best] = nodes[c].index;
      ch[n++] = nodes[c].index + 1;
    }
    // child slot order: the device enters the first hit slot, then the others in slot order.  Default
    // 2, ascending box surface (0: as collapsed, 1: descending, 3: leaves first, then descending)
    if (order == 1 || order == 2 || order == 3) {
      std::stable_sort(ch, ch + n, [&](uint32_t a, uint32_t b) {
        if (order == 3 && nodes[a].leaf != nodes[b].leaf) return nodes[a].leaf > nodes[b].leaf;
        return order == 2 ? area(a) < area(b) : area(a) > area(b);
      });
    }
    WideNodeRecord r{};
    for (int a = 0; a < 3; a++) {
      double lo[kWideK], hi[kWideK];
      for (int k = 0; k < n; k++) {
        lo[k] = (double)nodes[ch[k]].bmin[a] - widen;
        hi[k] = (double)nodes[ch[k]].bmax[a] + widen;
      }
      uint32_t e = 0;
      if (!quantize_axis(lo, hi, n, r.p[a], e, r.q + kWideW * (2 * a), r.q + kWideW * (2 * a + 1))) return false;
      r.ebits |= e << (8 * a);
    }
    // children pushed in reverse so the first child's subtree follows its parent in memory
    for (int k = n - 1; k >= 0; k--) {
      if (nodes[ch[k]].leaf) {
        r.desc[k] = leaf_descs[ch[k]];
      } else {
        r.desc[k] = (uint32_t)out.size();
        out.emplace_back();
        st.push_back({ch[k], r.desc[k], it.depth + 1});
      }
    }
    out[it.slot] = r;
  }
  if ((kWideK - 1) * maxd > kWideMaxStack) return false;  // a node pushes at most kWideK - 1 children
  root = 0;
  return true;
}

extern "C" {

int drt_abi_version(void) { return DRT_ABI_VERSION; }

int drt_create(drt_ctx** out, const drt_options* opt) {
  if (!out) return DRT_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DRT_E_NODEVICE;
  int dev = opt ? opt->device : 0;
  if (dev < 0 || dev >= ndev) return DRT_E_INVALID;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return DRT_E_HIP;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DRT_E_NODEVICE;
  drt_ctx* c = new drt_ctx();
  c->device = dev;
  if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return DRT_E_HIP;
  }
  c->ring.assign(drt_ctx::kEv * drt_ctx::kRing, nullptr);
  for (auto& e : c->ring)
    if (hipEventCreate(&e) != hipSuccess) {
      drt_destroy(c);
      return DRT_E_HIP;
    }
  for (auto& e : c->tev)
    if (hipEventCreate(&e) != hipSuccess) {
      drt_destroy(c);
      return DRT_E_HIP;
    }
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
  for (int k = 0; k < DRT_FRAME_SLOTS; k++) {
    if (hipStreamCreateWithPriority(&c->aux[k], hipStreamNonBlocking, greatest) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_shuf[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_path[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_red[k], hipEventDisableTiming) != hipSuccess) {
      drt_destroy(c);
      return DRT_E_HIP;
    }
  }
  *out = c;
  return DRT_OK;
}

void drt_destroy(drt_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& e : c->ring)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->tev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->stage_ev)
    if (e) (void)hipEventDestroy(e);
  for (int k = 0; k < DRT_FRAME_SLOTS; k++) {
    if (c->aux[k]) {
      (void)hipStreamSynchronize(c->aux[k]);
      (void)hipStreamDestroy(c->aux[k]);
    }
    for (hipEvent_t e : {c->ev_shuf[k], c->ev_path[k], c->ev_red[k]})
      if (e) (void)hipEventDestroy(e);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* drt_last_error(const drt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int drt_upload_scene(drt_ctx* c, const drt_scene_desc* s) {
  if (!c || !s) return DRT_E_INVALID;
  // Nothing renders against a half-replaced scene: the context's scene and accelerator are
  // invalid from here until this upload has committed every buffer.
  c->has_scene = c->has_bvh = c->has_grid = c->has_gv = false;
  if (s->camera.res_x <= 0 || s->camera.res_y <= 0) DRT_FAIL(c, DRT_E_INVALID, "camera resolution must be positive");
  if (s->n_prims < 0 || (s->n_prims > 0 && !s->prims)) DRT_FAIL(c, DRT_E_INVALID, "bad primitive array");
  if (s->n_lights < 0 || (s->n_lights > 0 && !s->lights)) DRT_FAIL(c, DRT_E_INVALID, "bad light array");
  if (s->n_materials < 0 || (s->n_materials > 0 && !s->materials)) DRT_FAIL(c, DRT_E_INVALID, "bad material array");
  if (s->accel < DRT_ACCEL_NONE || s->accel > DRT_ACCEL_BVH) DRT_FAIL(c, DRT_E_INVALID, "bad accel %d", s->accel);
  for (int i = 0; i < s->n_lights; i++)
    if (s->lights[i].type != DRT_LIGHT_POINT && s->lights[i].type != DRT_LIGHT_QUAD)
      DRT_FAIL(c, DRT_E_INVALID, "light %d: bad type %d", i, s->lights[i].type);
  if (s->has_skybox)
    for (int f = 0; f < 6; f++)
      if (!s->skybox[f] || s->sky_w[f] <= 0 || s->sky_h[f] <= 0 || (s->sky_bpp[f] != 3 && s->sky_bpp[f] != 4))
        DRT_FAIL(c, DRT_E_INVALID, "skybox face %d missing or malformed", f);
  // Objects without a material are UB upstream (m_Material uninitialised); they get the
  // default Material() (scene.h:38) appended at the end of the table.
  std::vector<drt_material> mats(s->materials, s->materials + s->n_materials);
  const uint32_t dflt = (uint32_t)mats.size();
  mats.push_back(drt_material{{0.2f, 0.2f, 0.2f}, 0.2f, {1.f, 1.f, 1.f}, 0.8f, 20.f, 1.0f, 0.0f, 1.0f});
  std::vector<PrimRecord> prims((size_t)s->n_prims);
  bool tri_only = true;
  for (int i = 0; i < s->n_prims; i++) {
    const drt_prim& p = s->prims[i];
    if (p.type < 0 || p.type > 3) DRT_FAIL(c, DRT_E_INVALID, "prim %d: bad type %d", i, p.type);
    if (p.material >= s->n_materials) DRT_FAIL(c, DRT_E_INVALID, "prim %d: material %d out of range", i, p.material);
    if (p.type != DRT_PRIM_TRIANGLE) tri_only = false;
    prims[i] = pack_prim(p, p.material < 0 ? dflt : (uint32_t)p.material, (uint32_t)i);
  }
  std::vector<drt_light> lights(s->lights, s->lights + s->n_lights);
  // validated: device buffers next (a failure here leaves the context without a scene)
  DRT_HIP(c, hipSetDevice(c->device));
  // + 64 B: the BVH node step reads four 16-B slots from a leaf's first record and, for leaves of
  // two or more, two more; the tail slots of the last record must stay inside the allocation
  DRT_HIP(c, c->d_prims.ensure(sizeof(PrimRecord) * prims.size() + kPrimPadBytes));
  DRT_HIP(c, hipMemset(c->d_prims.p, 0, sizeof(PrimRecord) * prims.size() + kPrimPadBytes));
  DRT_HIP(c, hipMemcpy(c->d_prims.p, prims.data(), sizeof(PrimRecord) * prims.size(), hipMemcpyHostToDevice));
  DRT_HIP(c, c->d_lights.ensure(sizeof(drt_light) * std::max<size_t>(1, lights.size())));
  if (!lights.empty())
    DRT_HIP(c, hipMemcpy(c->d_lights.p, lights.data(), sizeof(drt_light) * lights.size(), hipMemcpyHostToDevice));
  DRT_HIP(c, c->d_mats.ensure(sizeof(drt_material) * mats.size()));
  DRT_HIP(c, hipMemcpy(c->d_mats.p, mats.data(), sizeof(drt_material) * mats.size(), hipMemcpyHostToDevice));
  for (int f = 0; f < 6; f++) {
    c->sky_w[f] = c->sky_h[f] = c->sky_bpp[f] = 0;
    if (!s->has_skybox) continue;
    size_t n = (size_t)s->sky_w[f] * s->sky_h[f] * s->sky_bpp[f];
    DRT_HIP(c, c->d_sky[f].ensure(n));
    DRT_HIP(c, hipMemcpy(c->d_sky[f].p, s->skybox[f], n, hipMemcpyHostToDevice));
    c->sky_w[f] = s->sky_w[f]; c->sky_h[f] = s->sky_h[f]; c->sky_bpp[f] = s->sky_bpp[f];
  }
  // commit
  c->has_sky = s->has_skybox ? 1 : 0;
  c->cam = s->camera;
  c->accel = s->accel;
  c->spp = s->spp;
  memcpy(c->bg, s->background, sizeof(c->bg));
  c->lights = std::move(lights);
  c->mats = std::move(mats);
  c->n_prims = s->n_prims;
  c->prims_scene = std::move(prims);
  c->tri_only = tri_only;
  c->has_scene = true;
  return DRT_OK;
}

int drt_set_camera(drt_ctx* c, const drt_camera* k) {
  if (!c || !k) return DRT_E_INVALID;
  if (!c->has_scene) DRT_FAIL(c, DRT_E_STATE, "set the camera of an uploaded scene");
  if (k->res_x <= 0 || k->res_y <= 0) DRT_FAIL(c, DRT_E_INVALID, "camera resolution must be positive");
  // Camera::SetEye moves the eye and keeps the resolution (camera.h:63-72); the caller's frame
  // buffers are sized by it, so a different one is refused (re-upload the scene to change it)
  if (k->res_x != c->cam.res_x || k->res_y != c->cam.res_y)
    DRT_FAIL(c, DRT_E_INVALID, "camera resolution %dx%d differs from the resident %dx%d", k->res_x, k->res_y,
             c->cam.res_x, c->cam.res_y);
  // the frame reaches the kernels by value (SceneArgs, copied at launch): frames already issued
  // keep the camera they were launched with
  c->cam = *k;
  return DRT_OK;
}

int drt_upload_bvh(drt_ctx* c, const drt_bvh_node* nodes, uint32_t n_nodes, const uint32_t* order, uint32_t n_obj) {
  if (!c || !nodes || n_nodes == 0) return DRT_E_INVALID;
  if (!c->has_scene) DRT_FAIL(c, DRT_E_STATE, "upload the scene before its BVH");
  c->has_bvh = c->has_grid = c->has_gv = false;  // until this upload commits
  if ((int)n_obj != c->n_prims || (n_obj && !order)) DRT_FAIL(c, DRT_E_INVALID, "object_order must cover all %d objects", c->n_prims);
  std::vector<uint8_t> seen(n_obj, 0);
  for (uint32_t i = 0; i < n_obj; i++) {
    if (order[i] >= n_obj || seen[order[i]]) DRT_FAIL(c, DRT_E_INVALID, "object_order is not a permutation");
    seen[order[i]] = 1;
  }
  // inner records in reference node order
  std::vector<int64_t> rec(n_nodes, -1);
  uint32_t n_inner = 0;
  for (uint32_t i = 0; i < n_nodes; i++) {
    const drt_bvh_node& nd = nodes[i];
    if (nd.leaf) {
      if ((uint64_t)nd.index + nd.n_objs > n_obj) DRT_FAIL(c, DRT_E_INVALID, "leaf %u out of range", i);
    } else {
      if ((uint64_t)nd.index + 1 >= n_nodes || nd.index <= i) DRT_FAIL(c, DRT_E_INVALID, "inner node %u: bad children", i);
      rec[i] = n_inner++;
    }
  }
  if (n_obj > kFirstMask) DRT_FAIL(c, DRT_E_UNSUPPORTED, "more than %u objects", kFirstMask);
  // Where each inner record sits in memory (DRT_NODE_LAYOUT; the tree, its descriptors' meaning and
  // every traversal are unchanged): 0 = reference node order; 1 (default) = a record and, in the
  // same 128-B line, the record of its child with the larger box surface (the child a ray more
  // often visits next), each such pair starting a line; 2 = a node's two inner children side by
  // side, the pair starting a line.  Headline frame: fabric line reads 2.12 -> 1.89 G per launch
  // with 1 (2: 2.11 G), 89.4 against 89.7 ms; C4 610-623 against 625 ms.
  const int layout = env_int("DRT_NODE_LAYOUT", 1);
  std::vector<uint32_t> slot_of(n_inner);
  uint32_t n_slots = n_inner;
  if ((layout == 1 || layout == 2) && n_inner > 0) {  // (a leaf root has no inner record)
    auto area = [&](uint32_t i) {
      const drt_bvh_node& nd = nodes[i];
      const double x = (double)nd.bmax[0] - nd.bmin[0], y = (double)nd.bmax[1] - nd.bmin[1],
                   z = (double)nd.bmax[2] - nd.bmin[2];
      return x * y + y * z + z * x;
    };
    auto inner_children = [&](uint32_t n, uint32_t& a, uint32_t& b) {  // a: larger surface
      const uint32_t l = nodes[n].index, r = l + 1;
      a = b = UINT32_MAX;
      const bool li = !nodes[l].leaf, ri = !nodes[r].leaf;
      if (li && ri) {
        a = area(l) >= area(r) ? l : r;
        b = a == l ? r : l;
      } else if (li) {
        a = l;
      } else if (ri) {
        a = r;
      }
    };
    uint32_t pos = 0;
    std::vector<uint32_t> st;
    if (layout == 1) {
      st.push_back(0u);
      while (!st.empty()) {
        const uint32_t n = st.back();
        st.pop_back();
        pos += pos & 1u;  // a line starts
        slot_of[rec[n]] = pos++;
        uint32_t a, b;
        inner_children(n, a, b);
        if (a == UINT32_MAX) continue;
        slot_of[rec[a]] = pos++;
        if (b != UINT32_MAX) st.push_back(b);
        uint32_t aa, ab;
        inner_children(a, aa, ab);
        if (ab != UINT32_MAX) st.push_back(ab);
        if (aa != UINT32_MAX) st.push_back(aa);
      }
    } else {
      slot_of[rec[0]] = pos++;
      st.push_back(0u);
      while (!st.empty()) {
        const uint32_t n = st.back();
        st.pop_back();
        uint32_t a, b;
        inner_children(n, a, b);
        if (a == UINT32_MAX) continue;
        pos += pos & 1u;
        const uint32_t l = nodes[n].index;  // left, right order within the pair
        if (!nodes[l].leaf) slot_of[rec[l]] = pos++;
        if (!nodes[l + 1].leaf) slot_of[rec[l + 1]] = pos++;
        if (b != UINT32_MAX) st.push_back(b);
        st.push_back(a);
      }
    }
    n_slots = pos;
  } else {
    for (uint32_t k = 0; k < n_inner; k++) slot_of[k] = k;
  }
  std::vector<uint2> big;
  auto desc_of = [&](uint32_t i) -> uint32_t {
    const drt_bvh_node& nd = nodes[i];
    if (!nd.leaf) return slot_of[(size_t)rec[i]];
    if (nd.n_objs < kBigLeaf) return leaf_desc(nd.index, nd.n_objs);
    big.push_back(make_uint2(nd.index, nd.n_objs));
    return leaf_desc((uint32_t)big.size() - 1, kBigLeaf);
  };
  std::vector<uint32_t> dsc(n_nodes);  // every node's descriptor, once (big leaves get one table entry)
  for (uint32_t i = 0; i < n_nodes; i++) dsc[i] = desc_of(i);
  std::vector<NodeRecord> recs(n_slots);  // padding slots stay zero (never referenced)
  for (uint32_t i = 0; i < n_nodes; i++) {
    if (nodes[i].leaf) continue;
    const drt_bvh_node& L = nodes[nodes[i].index];
    const drt_bvh_node& R = nodes[nodes[i].index + 1];
    NodeRecord& r = recs[slot_of[(size_t)rec[i]]];
    const float b[12] = {L.bmin[0], L.bmin[1], L.bmin[2], L.bmax[0], L.bmax[1], L.bmax[2],
                         R.bmin[0], R.bmin[1], R.bmin[2], R.bmax[0], R.bmax[1], R.bmax[2]};
    memcpy(r.box, b, sizeof(b));
    r.desc[0] = dsc[nodes[i].index];
    r.desc[1] = dsc[nodes[i].index + 1];
    r.desc[2] = r.desc[3] = 0;
  }
  // 4-ary shadow tree and the exact reference leaf box of every primitive (DRT_WIDE_SHADOW=0: none)
  std::vector<WideNodeRecord> wide;
  uint32_t wroot = 0;
  const bool has_wide = env_int("DRT_WIDE_SHADOW", 1) != 0 && wide_tree_valid(nodes, n_nodes, n_obj) &&
                        build_wide(nodes, dsc, wide, wroot);
  std::vector<LeafBoxRecord> lbox;
  if (has_wide) {
    lbox.assign((size_t)n_obj + 2, LeafBoxRecord{});  // + 2: the node step's tail slot reads
    for (uint32_t i = 0; i < n_nodes; i++) {
      const drt_bvh_node& nd = nodes[i];
      if (!nd.leaf) continue;
      LeafBoxRecord b{};
      memcpy(b.box, nd.bmin, 12);
      memcpy(b.box + 3, nd.bmax, 12);
      for (uint32_t k = 0; k < nd.n_objs; k++) lbox[nd.index + k] = b;
    }
  }
  // depth (= bound on the traversal stack), iterative
  int maxd = 0;
  {
    std::vector<std::pair<uint32_t, int>> st{{0u, 1}};
    while (!st.empty()) {
      auto [i, d] = st.back();
      st.pop_back();
      maxd = std::max(maxd, d);
      if (!nodes[i].leaf) {
        st.push_back({nodes[i].index, d + 1});
        st.push_back({nodes[i].index + 1, d + 1});
      }
    }
  }
  if (maxd >= kMaxBvhDepth) DRT_FAIL(c, DRT_E_UNSUPPORTED, "BVH depth %d exceeds the %d-entry traversal stack", maxd, kMaxBvhDepth);
  c->bvh_depth = maxd;
  memcpy(c->root_box, nodes[0].bmin, 3 * sizeof(float));
  memcpy(c->root_box + 3, nodes[0].bmax, 3 * sizeof(float));
  c->root_desc = dsc[0];
  DRT_HIP(c, hipSetDevice(c->device));
  DRT_HIP(c, c->d_nodes.ensure(sizeof(NodeRecord) * std::max<size_t>(1, recs.size())));
  if (!recs.empty()) DRT_HIP(c, hipMemcpy(c->d_nodes.p, recs.data(), sizeof(NodeRecord) * recs.size(), hipMemcpyHostToDevice));
  c->has_wide = false;
  if (has_wide) {
    DRT_HIP(c, c->d_wnodes.ensure(sizeof(WideNodeRecord) * wide.size()));
    DRT_HIP(c, hipMemcpy(c->d_wnodes.p, wide.data(), sizeof(WideNodeRecord) * wide.size(), hipMemcpyHostToDevice));
    DRT_HIP(c, c->d_wleaf.ensure(sizeof(LeafBoxRecord) * lbox.size()));
    DRT_HIP(c, hipMemcpy(c->d_wleaf.p, lbox.data(), sizeof(LeafBoxRecord) * lbox.size(), hipMemcpyHostToDevice));
    c->wroot = wroot;
    c->n_wide = (uint32_t)wide.size();
    c->has_wide = true;
  }
  DRT_HIP(c, c->d_big.ensure(sizeof(uint2) * std::max<size_t>(1, big.size())));
  if (!big.empty()) DRT_HIP(c, hipMemcpy(c->d_big.p, big.data(), sizeof(uint2) * big.size(), hipMemcpyHostToDevice));
  // primitive records in BVH object order: every leaf is one contiguous run
  std::vector<PrimRecord> perm(n_obj);
  for (uint32_t i = 0; i < n_obj; i++) perm[i] = c->prims_scene[order[i]];
  DRT_HIP(c, hipMemcpy(c->d_prims.p, perm.data(), sizeof(PrimRecord) * perm.size(), hipMemcpyHostToDevice));
  c->has_bvh = true;
  c->has_grid = false;
  return DRT_OK;
}

int drt_upload_grid(drt_ctx* c, const int32_t dims[3], const float bmin[3], const float bmax[3], const int64_t* cs,
                    const int32_t* co, int64_t n_refs) {
  if (!c || !dims || !bmin || !bmax || !cs || (n_refs > 0 && !co)) return DRT_E_INVALID;
  if (!c->has_scene) DRT_FAIL(c, DRT_E_STATE, "upload the scene before its grid");
  c->has_bvh = c->has_grid = c->has_gv = false;  // until this upload commits
  // A scene without objects: Grid::Build's widths overflow (float FLT_MAX - -FLT_MAX), the cell
  // counts come out NaN -> INT_MIN and the grid has no cells (grid.cpp:56-67); its box is
  // inverted, so every ray misses it.  Same here with one empty cell under that box.
  static const int64_t kEmptyStart[2] = {0, 0};
  static const int32_t kOneCell[3] = {1, 1, 1};
  if (n_refs == 0 && (dims[0] <= 0 || dims[1] <= 0 || dims[2] <= 0)) {
    dims = kOneCell;
    cs = kEmptyStart;
  }
  if (dims[0] <= 0 || dims[1] <= 0 || dims[2] <= 0) DRT_FAIL(c, DRT_E_INVALID, "bad grid dims");
  if (n_refs >= (int64_t)0xFFFFFFFF) DRT_FAIL(c, DRT_E_UNSUPPORTED, "too many grid references");
  const size_t ncell = (size_t)dims[0] * dims[1] * dims[2];
  std::vector<uint32_t> s32(ncell + 1), o32((size_t)n_refs);
  for (size_t i = 0; i <= ncell; i++) {
    if (cs[i] < 0 || cs[i] > n_refs || (i && cs[i] < cs[i - 1])) DRT_FAIL(c, DRT_E_INVALID, "bad cell_start");
    s32[i] = (uint32_t)cs[i];
  }
  for (int64_t i = 0; i < n_refs; i++) {
    if (co[i] < 0 || co[i] >= c->n_prims) DRT_FAIL(c, DRT_E_INVALID, "bad cell object");
    o32[i] = (uint32_t)co[i];
  }
  // every object's cell range: Grid::Build registers an object in every cell of its box's range
  // (grid.cpp:78-92), so the range is the min / max over the cells that list it
  std::vector<int32_t> cells_of((size_t)c->n_prims * 6);
  for (int i = 0; i < c->n_prims; i++) {
    int32_t* r = &cells_of[(size_t)i * 6];
    r[0] = r[1] = r[2] = INT32_MAX;
    r[3] = r[4] = r[5] = -1;
  }
  for (int z = 0; z < dims[2]; z++)
    for (int y = 0; y < dims[1]; y++)
      for (int x = 0; x < dims[0]; x++) {
        const size_t ci = (size_t)x + (size_t)dims[0] * y + (size_t)dims[0] * dims[1] * z;
        for (uint32_t k = s32[ci]; k < s32[ci + 1]; k++) {
          int32_t* r = &cells_of[(size_t)o32[k] * 6];
          r[0] = std::min(r[0], x); r[1] = std::min(r[1], y); r[2] = std::min(r[2], z);
          r[3] = std::max(r[3], x); r[4] = std::max(r[4], y); r[5] = std::max(r[5], z);
        }
      }
  DRT_HIP(c, hipSetDevice(c->device));
  DRT_HIP(c, c->d_cell_start.ensure(4 * s32.size()));
  DRT_HIP(c, hipMemcpy(c->d_cell_start.p, s32.data(), 4 * s32.size(), hipMemcpyHostToDevice));
  DRT_HIP(c, c->d_cell_objs.ensure(4 * std::max<size_t>(1, o32.size())));
  if (!o32.empty()) DRT_HIP(c, hipMemcpy(c->d_cell_objs.p, o32.data(), 4 * o32.size(), hipMemcpyHostToDevice));
  // Triangle scenes (round 5): the referenced triangles inline in cell order as 40-B records
  // (v0, e1, e2, scene index), two per 80-B pair = five 16-B loads instead of six for two 48-B
  // records (the stepper is bound by the per-lane loads of the vector-memory path), and
  // 132 instead of 158 MB at 1M triangles.  A cell's list starts on a pair boundary: cell_tpos[i] is
  // its first record (even), bit 31 set when cell i - 1's list ended on a padding slot, so a cell's
  // range is [tpos[i], tpos[i + 1] - pad) from one 8-B load.
#if defined(DRT_GRID_RECS48) || defined(DRT_GRID_INDEXED)
  const bool packed = false;  // (A/B) the 48-B records for every scene (the indexed layout's too)
#else
  const bool packed = c->tri_only;
#endif
  if (packed) {
    std::vector<uint32_t> tpos(ncell + 1);
    uint64_t pos = 0;
    uint32_t pad = 0;
    for (size_t i = 0; i < ncell; i++) {
      const uint32_t cnt = s32[i + 1] - s32[i];
      tpos[i] = (uint32_t)pos | (pad << 31);
      pos += cnt + (cnt & 1u);
      pad = cnt & 1u;
    }
    if (pos >= 0x80000000ull) DRT_FAIL(c, DRT_E_UNSUPPORTED, "too many grid references");
    tpos[ncell] = (uint32_t)pos | (pad << 31);
    std::vector<float> tris((size_t)(pos / 2 + 1) * 20, 0.0f);
    for (size_t i = 0; i < ncell; i++)
      for (uint32_t k = s32[i], j = 0; k < s32[i + 1]; k++, j++) {
        const uint32_t at = (tpos[i] & 0x7fffffffu) + j;  // record position
        float* f = &tris[(size_t)(at >> 1) * 20 + (at & 1u) * 10];
        const PrimRecord& r = c->prims_scene[o32[k]];  // (v0, .), (e1, .), (e2, .)
        memcpy(f, &r.q[0], 12);
        memcpy(f + 3, &r.q[4], 12);
        memcpy(f + 6, &r.q[8], 12);
        memcpy(f + 9, &o32[k], 4);
      }
    DRT_HIP(c, c->d_cell_tpos.ensure(4 * tpos.size()));
    DRT_HIP(c, hipMemcpy(c->d_cell_tpos.p, tpos.data(), 4 * tpos.size(), hipMemcpyHostToDevice));
    DRT_HIP(c, c->d_cell_tris.ensure(4 * tris.size() + kPrimPadBytes));
    DRT_HIP(c, hipMemset(c->d_cell_tris.p, 0, 4 * tris.size() + kPrimPadBytes));
    DRT_HIP(c, hipMemcpy(c->d_cell_tris.p, tris.data(), 4 * tris.size(), hipMemcpyHostToDevice));
    c->d_cell_recs.release();
  } else {
    c->d_cell_tris.release();
    c->d_cell_tpos.release();
  }
  // other scenes' persistent Grid stepper reads the referenced records inline, in cell order (48 B
  // per reference; q2.w = the scene-order primitive index), so a cell's objects are one hop away
  if (!packed) {
    std::vector<PrimRecord> recs((size_t)std::max<int64_t>(1, n_refs));
    for (int64_t i = 0; i < n_refs; i++) {
      recs[i] = c->prims_scene[o32[i]];
      memcpy(&recs[i].q[11], &o32[i], 4);
    }
    DRT_HIP(c, c->d_cell_recs.ensure(sizeof(PrimRecord) * recs.size() + kPrimPadBytes));
    DRT_HIP(c, hipMemset(c->d_cell_recs.p, 0, sizeof(PrimRecord) * recs.size() + kPrimPadBytes));
    DRT_HIP(c, hipMemcpy(c->d_cell_recs.p, recs.data(), sizeof(PrimRecord) * recs.size(), hipMemcpyHostToDevice));
  }
  // Indexed layout (experiment, drt_kernels.hip DRT_GRID_INDEXED): every object's record once, in the
  // order a Morton walk of the non-empty cells first meets it (q2.w = the scene-order index), and per
  // reference its position there — so that objects of neighbouring cells share lines.  Built and
  // uploaded only by builds that read it.
#ifdef DRT_GRID_INDEXED
  {
    auto part = [](uint32_t v) {  // 10 bits -> every third bit
      v &= 0x3ffu;
      v = (v | (v << 16)) & 0x030000FFu;
      v = (v | (v << 8)) & 0x0300F00Fu;
      v = (v | (v << 4)) & 0x030C30C3u;
      v = (v | (v << 2)) & 0x09249249u;
      return v;
    };
    std::vector<std::pair<uint32_t, uint32_t>> cells;  // (Morton code, cell)
    for (int z = 0; z < dims[2]; z++)
      for (int y = 0; y < dims[1]; y++)
        for (int x = 0; x < dims[0]; x++) {
          const size_t ci = (size_t)x + (size_t)dims[0] * y + (size_t)dims[0] * dims[1] * z;
          if (s32[ci + 1] != s32[ci])
            cells.push_back({part((uint32_t)x) | (part((uint32_t)y) << 1) | (part((uint32_t)z) << 2), (uint32_t)ci});
        }
    std::sort(cells.begin(), cells.end());
    std::vector<uint32_t> rank((size_t)c->n_prims, UINT32_MAX);
    uint32_t next = 0;
    for (auto& mc : cells)
      for (uint32_t k = s32[mc.second]; k < s32[mc.second + 1]; k++)
        if (rank[o32[k]] == UINT32_MAX) rank[o32[k]] = next++;
    for (auto& r : rank)
      if (r == UINT32_MAX) r = next++;
    std::vector<PrimRecord> g((size_t)std::max(1, c->n_prims));
    for (int i = 0; i < c->n_prims; i++) {
      g[rank[i]] = c->prims_scene[i];
      memcpy(&g[rank[i]].q[11], &i, 4);
    }
    std::vector<uint32_t> pos((size_t)n_refs + 2, 0u);  // + 2: the stepper reads pairs
    for (int64_t i = 0; i < n_refs; i++) pos[i] = rank[o32[i]];
    DRT_HIP(c, c->d_gprims.ensure(sizeof(PrimRecord) * g.size() + kPrimPadBytes));
    DRT_HIP(c, hipMemset(c->d_gprims.p, 0, sizeof(PrimRecord) * g.size() + kPrimPadBytes));
    DRT_HIP(c, hipMemcpy(c->d_gprims.p, g.data(), sizeof(PrimRecord) * g.size(), hipMemcpyHostToDevice));
    DRT_HIP(c, c->d_cell_pos.ensure(4 * pos.size()));
    DRT_HIP(c, hipMemcpy(c->d_cell_pos.p, pos.data(), 4 * pos.size(), hipMemcpyHostToDevice));
  }
#endif
  // grid references index scene-order primitive records
  DRT_HIP(c, hipMemcpy(c->d_prims.p, c->prims_scene.data(), sizeof(PrimRecord) * c->prims_scene.size(),
                       hipMemcpyHostToDevice));
  // macro-cell occupancy bitmap (2^ms cells per side, <= kMacroBits bits): the Grid stepper keeps it
  // in LDS and steps through empty macro-cells without touching memory
  int ms = 0;
  auto mdim = [&](int d, int m) { return (d + (1 << m) - 1) >> m; };
  while ((size_t)mdim(dims[0], ms) * mdim(dims[1], ms) * mdim(dims[2], ms) > kMacroBits) ms++;
  const int mx = mdim(dims[0], ms), my = mdim(dims[1], ms), mz = mdim(dims[2], ms);
  std::vector<uint32_t> bits(((size_t)mx * my * mz + 31) / 32, 0u);
  for (int z = 0; z < dims[2]; z++)
    for (int y = 0; y < dims[1]; y++)
      for (int x = 0; x < dims[0]; x++) {
        const size_t ci = (size_t)x + (size_t)dims[0] * y + (size_t)dims[0] * dims[1] * z;
        if (s32[ci + 1] == s32[ci]) continue;
        const size_t mi = (size_t)(x >> ms) + (size_t)mx * (y >> ms) + (size_t)mx * my * (z >> ms);
        bits[mi >> 5] |= 1u << (mi & 31);
      }
  DRT_HIP(c, c->d_macro.ensure(4 * bits.size()));
  DRT_HIP(c, hipMemcpy(c->d_macro.p, bits.data(), 4 * bits.size(), hipMemcpyHostToDevice));
  c->gmacro_shift = ms;
  c->gmacro_dim[0] = mx; c->gmacro_dim[1] = my; c->gmacro_dim[2] = mz;
  c->gmacro_words = (int)bits.size();
  memcpy(c->gdim, dims, sizeof(c->gdim));
  memcpy(c->gmin, bmin, sizeof(c->gmin));
  memcpy(c->gmax, bmax, sizeof(c->gmax));
  c->grid_cells = std::move(cells_of);
  c->has_grid = true;
  c->has_bvh = false;
  return DRT_OK;
}

int drt_upload_grid_shadow_bvh(drt_ctx* c, const drt_bvh_node* nodes, uint32_t n_nodes, const uint32_t* order,
                               uint32_t n_obj) {
  if (!c || !nodes || n_nodes == 0) return DRT_E_INVALID;
  if (!c->has_grid) DRT_FAIL(c, DRT_E_STATE, "upload the grid before its shadow tree");
  c->has_gv = false;  // until this upload commits
  if ((int)n_obj != c->n_prims || (n_obj && !order)) DRT_FAIL(c, DRT_E_INVALID, "object_order must cover all %d objects", c->n_prims);
  if (!c->tri_only) DRT_FAIL(c, DRT_E_UNSUPPORTED, "the Grid's shadow tree serves triangle scenes");
  if (n_obj > kFirstMask) DRT_FAIL(c, DRT_E_UNSUPPORTED, "more than %u objects", kFirstMask);
  std::vector<uint8_t> seen(n_obj, 0);
  for (uint32_t i = 0; i < n_obj; i++) {
    if (order[i] >= n_obj || seen[order[i]]) DRT_FAIL(c, DRT_E_INVALID, "object_order is not a permutation");
    seen[order[i]] = 1;
  }
  for (uint32_t i = 0; i < n_nodes; i++) {
    const drt_bvh_node& nd = nodes[i];
    if (nd.leaf ? (uint64_t)nd.index + nd.n_objs > n_obj : ((uint64_t)nd.index + 1 >= n_nodes || nd.index <= i))
      DRT_FAIL(c, DRT_E_INVALID, "node %u out of range", i);
  }
  if (!wide_tree_valid(nodes, n_nodes, n_obj)) DRT_FAIL(c, DRT_E_INVALID, "not a tree of nested boxes over every object");
  // leaf descriptors (oversized leaves through the big-leaf table, as drt_upload_bvh)
  std::vector<uint2> big;
  std::vector<uint32_t> dsc(n_nodes, 0u);
  for (uint32_t i = 0; i < n_nodes; i++) {
    const drt_bvh_node& nd = nodes[i];
    if (!nd.leaf) continue;
    if (nd.n_objs < kBigLeaf) {
      dsc[i] = leaf_desc(nd.index, nd.n_objs);
    } else {
      big.push_back(make_uint2(nd.index, nd.n_objs));
      dsc[i] = leaf_desc((uint32_t)big.size() - 1, kBigLeaf);
    }
  }
  // Child boxes grown by 2^-19 M, M the scene's largest coordinate (DRT_GRID_TREE_WIDEN_LOG2 = -19): every
  // primitive whose test reports a hit at t < range lies inside its grown box, and a ray through a grown
  // box passes its slab test — the slab values (P - o) * inv carry 3 eps of relative error, under 4 eps D
  // of the ray's length to the box (D <= 2 sqrt(3) M the scene's diagonal: 14 eps M), and a reported hit
  // lies within a few eps M of its triangle — so the walk is an any-hit over every object, and a query
  // it finds no hit for is one Grid::Traverse(Ray&) finds none for either.
  // (2^-16 M measured 14 % more node visits on the Grid headline, whose floor sets M.)
  double m = 0.0;
  for (int a = 0; a < 3; a++) m = std::max(m, std::max(std::fabs((double)nodes[0].bmin[a]), std::fabs((double)nodes[0].bmax[a])));
  const double widen = std::ldexp(m, std::min(-17, env_int("DRT_GRID_TREE_WIDEN_LOG2", -19)));
  std::vector<WideNodeRecord> wide;
  uint32_t wroot = 0;
  if (!build_wide(nodes, dsc, wide, wroot, widen)) DRT_FAIL(c, DRT_E_UNSUPPORTED, "no shadow tree for this grid scene");
  // primitives in the tree's order, and per such primitive its cell range (grid_certificate)
  std::vector<PrimRecord> perm(n_obj);
  std::vector<LeafBoxRecord> rng((size_t)n_obj + 2, LeafBoxRecord{});  // + 2: the node step's tail slot reads
  const bool nocert = env_int("DRT_GRID_TREE_NOCERT", 0) != 0;  // (tests) every hit to the Grid walk
  for (uint32_t i = 0; i < n_obj; i++) {
    perm[i] = c->prims_scene[order[i]];
    const int32_t* r = &c->grid_cells[(size_t)order[i] * 6];
    LeafBoxRecord& b = rng[i];
    if (r[3] < 0 || nocert) {  // listed in no cell: an inverted range, never certified
      b.box[0] = b.box[1] = b.box[2] = 1.0f;
      b.box[3] = b.box[4] = b.box[5] = 0.0f;
    } else {
      for (int k = 0; k < 6; k++) b.box[k] = (float)r[k];
    }
  }
  DRT_HIP(c, hipSetDevice(c->device));
  DRT_HIP(c, c->d_gv_wnodes.ensure(sizeof(WideNodeRecord) * wide.size()));
  DRT_HIP(c, hipMemcpy(c->d_gv_wnodes.p, wide.data(), sizeof(WideNodeRecord) * wide.size(), hipMemcpyHostToDevice));
  DRT_HIP(c, c->d_gv_range.ensure(sizeof(LeafBoxRecord) * rng.size()));
  DRT_HIP(c, hipMemcpy(c->d_gv_range.p, rng.data(), sizeof(LeafBoxRecord) * rng.size(), hipMemcpyHostToDevice));
  DRT_HIP(c, c->d_gv_prims.ensure(sizeof(PrimRecord) * perm.size() + kPrimPadBytes));
  DRT_HIP(c, hipMemset(c->d_gv_prims.p, 0, sizeof(PrimRecord) * perm.size() + kPrimPadBytes));
  DRT_HIP(c, hipMemcpy(c->d_gv_prims.p, perm.data(), sizeof(PrimRecord) * perm.size(), hipMemcpyHostToDevice));
  DRT_HIP(c, c->d_gv_big.ensure(sizeof(uint2) * std::max<size_t>(1, big.size())));
  if (!big.empty()) DRT_HIP(c, hipMemcpy(c->d_gv_big.p, big.data(), sizeof(uint2) * big.size(), hipMemcpyHostToDevice));
  c->gv_wroot = wroot;
  c->has_gv = true;
  return DRT_OK;
}

}  // extern "C"

// reference_order: every shadow query walks the reference's binary tree in its visit order
// (DRT_FRAME_REFERENCE_ORDER: node / leaf / primitive counts equal the reference's)
static int scene_args(drt_ctx* c, int accel, SceneArgs& S, bool reference_order) {
  memset(&S, 0, sizeof(S));
  const drt_camera& k = c->cam;
  memcpy(S.eye, k.eye, 12); memcpy(S.u, k.u, 12); memcpy(S.v, k.v, 12); memcpy(S.n, k.n, 12);
  S.w = k.w; S.h = k.h; S.plane_dist = k.plane_dist; S.focal_ratio = k.focal_ratio; S.aperture = k.aperture;
  S.res_x = k.res_x; S.res_y = k.res_y;
  S.lights = c->d_lights.as<drt_light>();
  S.n_lights = (int)c->lights.size();
  S.mats = c->d_mats.as<drt_material>();
  S.n_mats = (int)c->mats.size();
  S.prims = c->d_prims.as<float4>();
  S.n_prims = c->n_prims;
  memcpy(S.bg, c->bg, 12);
  S.has_sky = c->has_sky;
  for (int f = 0; f < 6; f++) {
    S.sky[f] = c->d_sky[f].as<uint8_t>();
    S.sky_w[f] = c->sky_w[f]; S.sky_h[f] = c->sky_h[f]; S.sky_bpp[f] = c->sky_bpp[f];
  }
  if (accel == ACC_BVH) {
    if (!c->has_bvh) DRT_FAIL(c, DRT_E_STATE, "scene uses a BVH but none was uploaded");
    S.big_leaves = c->d_big.as<uint2>();
    S.nodes = c->d_nodes.as<float4>();
    memcpy(S.root_box, c->root_box, sizeof(S.root_box));
    S.root_desc = c->root_desc;
    if (c->has_wide && !reference_order) {
      S.wnodes = c->d_wnodes.as<float4>();
      S.wleaf = c->d_wleaf.as<float4>();
      S.wroot = c->wroot;
    }
  } else if (accel == ACC_GRID) {
    if (!c->has_grid) DRT_FAIL(c, DRT_E_STATE, "scene uses a grid but none was uploaded");
    memcpy(S.gdim, c->gdim, sizeof(S.gdim));
    memcpy(S.gmin, c->gmin, sizeof(S.gmin));
    memcpy(S.gmax, c->gmax, sizeof(S.gmax));
    // the shadow tree's cell certificate (grid_certificate): n / width per axis, and 128 eps K n_max
    double K = 1.0;
    int nm = 1;
    for (int a = 0; a < 3; a++) {
      const double w = (double)c->gmax[a] - (double)c->gmin[a];
      S.gscale[a] = (float)((double)c->gdim[a] / w);
      K = std::max(K, 1.0 + (std::fabs((double)c->gmin[a]) + std::fabs((double)c->gmax[a])) / w);
      nm = std::max(nm, c->gdim[a]);
    }
    const double margin = 128.0 * std::ldexp(1.0, -23) * K * nm;
    S.gmargin = margin < 0.25 ? (float)margin : 1.0f;  // (1: no certificate, every hit to the Grid walk)
    S.cell_start = c->d_cell_start.as<uint32_t>();
    S.gmacro = c->d_macro.as<uint32_t>();
    S.cell_recs = c->d_cell_recs.as<float4>();
    S.cell_tris = c->d_cell_tris.as<float4>();
    S.cell_tpos = c->d_cell_tpos.as<uint32_t>();
    S.gprims = c->d_gprims.as<float4>();
    S.cell_pos = c->d_cell_pos.as<uint32_t>();
    S.gmacro_shift = c->gmacro_shift;
    memcpy(S.gmacro_dim, c->gmacro_dim, sizeof(S.gmacro_dim));
    S.gmacro_words = c->gmacro_words;
    S.cell_objs = c->d_cell_objs.as<uint32_t>();
  }
  return DRT_OK;
}

struct Plan {
  FrameArgs F;
  ReduceArgs R;
  int tiles_y, n_tiles;
  bool persistent;      // path_persistent (BVH) instead of path_kernel
  bool two_pass;        // in-order frame as MODE_SKEL + MODE_REPLAY (no refraction in the scene)
  bool aa_chain;        // ... or an AA frame as MODE_CHAIN + MODE_REPLAY (BVH, shadow tree uploaded)
  uint32_t chain_div;   // two-pass Whitted frame: replay sample slots per closest-chain record (grid_res)
  bool tree;            // ... of a scene with a refracting material: MODE_TCHAIN + MODE_TREPLAY
  uint32_t recs;        // closest-hit records per (shared) sample: max_depth + 1, or 2^(max_depth+1) - 1
  bool wavefront;       // two-pass frame without refraction: pass 2 as wf_gen + shadow-query stream + wf_combine
  uint64_t wf_chunk;    // ... over chunks of this many sample slots
  uint32_t wf_chunks;
  bool wf_fold;         // ... with the reduce folded into wf_combine (no reduce launch, no sample buffer)
  bool skip;            // progressive frame past MAX_SAMPLES: nothing to render
  uint64_t n_slots;     // float4 sample slots of the frame (reduce reads nsub per pixel)
};

static void note_last_path_ms(drt_ctx* c);
// Query slots a chunk's buffers hold beyond its sample slots: each of <= 8 bands rounded up to 256 slots.
constexpr uint64_t kWfPad = 8u * 256u;
// Wavefront frames pack each 64-slot group's queries (WfArgs::compact, round 6): the BVH's trace_stream and
// the Grid's grid_stream refill from the group counts.  DRT_WAVEFRONT_COMPACT=0 keeps the thr = -1 markers
// (and on the Grid the path kernel's MODE_QSTREAM, as DRT_GRID_STREAM=0 does).
static bool wf_compact(const drt_ctx* c) {
#ifdef DRT_WF_PIECEWISE
  (void)c;
  return false;
#else
  if (env_int("DRT_WAVEFRONT_COMPACT", 1) == 0) return false;
  return c->accel == DRT_ACCEL_BVH || (c->accel == DRT_ACCEL_GRID && env_int("DRT_GRID_STREAM", 1) != 0);
#endif
}
// Shadow-query slots per level of a wavefront replay: the (light, k) pairs the light loop visits — every
// k of a quad light, k = 0 of a point light (next_light_pair).
static uint64_t wf_pairs(const drt_ctx* c, int light_spp) {
  uint64_t n = 0;
  for (const drt_light& l : c->lights) n += l.type == DRT_LIGHT_QUAD ? (uint64_t)std::max(1, light_spp) : 1u;
  return n;
}
static int plan_frame(drt_ctx* c, const drt_frame_params* p, Plan& P) {
  if (!c->has_scene) DRT_FAIL(c, DRT_E_STATE, "no scene uploaded");
  const int shards = p->n_shards <= 0 ? 1 : p->n_shards;
  if (p->shard < 0 || p->shard >= shards) DRT_FAIL(c, DRT_E_INVALID, "shard %d of %d", p->shard, shards);
  const int md = p->max_depth <= 0 ? 4 : p->max_depth;
  if (md >= kMaxFrames) DRT_FAIL(c, DRT_E_UNSUPPORTED, "max_depth %d > %d", md, kMaxFrames - 1);
  FrameArgs& F = P.F;
  memset(&F, 0, sizeof(F));
  F.seed = p->seed;
  F.max_depth = md;
  F.roughness = p->roughness;
  F.spp = c->spp;
  F.tile = p->tile > 0 ? p->tile : 16;
  const int RX = c->cam.res_x, RY = c->cam.res_y;
  F.tiles_x = (RX + F.tile - 1) / F.tile;
  P.tiles_y = (RY + F.tile - 1) / F.tile;
  P.n_tiles = F.tiles_x * P.tiles_y;
  F.shard = p->shard;
  F.n_shards = shards;
  F.n_my_tiles = P.n_tiles > p->shard ? (P.n_tiles - p->shard + shards - 1) / shards : 0;
  if (p->light_spp < 0 || p->light_spp > 4096) DRT_FAIL(c, DRT_E_INVALID, "light_spp %d out of [0, 4096]", p->light_spp);
  F.light_spp = p->light_spp > 1 ? p->light_spp : 1;
  F.light_grid = 1;
  while ((F.light_grid + 1) * (F.light_grid + 1) <= F.light_spp) F.light_grid++;
  F.light_inv = 1.0f / (float)F.light_spp;
  if (p->progressive_frame < 0) DRT_FAIL(c, DRT_E_INVALID, "progressive_frame %d < 0", p->progressive_frame);
  const int prog = p->progressive_frame;
  P.skip = prog >= 10000;  // FrameCount == MAX_SAMPLES (main.cpp:39, :537)
  const bool AA = c->spp != 0;                           // main.cpp:1005-1010
  F.dof = (c->cam.aperture != 0.0f && AA) ? 1 : 0;       // main.cpp:1013-1017
  const bool seq = F.dof || p->roughness != 0.0f;
  float scale = 1.0f;
  const bool quad0 = !c->lights.empty() && c->lights[0].type == DRT_LIGHT_QUAD;
  if (prog > 0) {  // zone A: one jittered sample per pixel whatever spp is (main.cpp:540-572)
    F.mode = MODE_PROG;
    F.nsub = 1;
  } else if (AA) {
    F.n_sqrt = (int)std::sqrt((double)c->spp);
    F.mode = seq ? MODE_SEQ : MODE_AA;
    F.nsub = seq ? 1 : (int)c->spp;
    scale = (float)(1.0 / (double)(float)c->spp);
  } else if (quad0) {
    F.grid_res = c->lights[0].grid_res;
    F.grid_size = (int)std::sqrt((double)F.grid_res);
    F.mode = seq ? MODE_SEQ : MODE_WHITTED_QUAD;
    F.nsub = seq ? 1 : (int)F.grid_res;
    scale = 1.0f / (float)(int)F.grid_res;
  } else {
    F.mode = seq ? MODE_SEQ : MODE_WHITTED_POINT;
    F.nsub = 1;
  }
  const int per_pixel = F.mode == MODE_SEQ ? 1 : F.nsub;  // work items per pixel
  F.n_items = (uint64_t)F.n_my_tiles * F.tile * F.tile * per_pixel;
  // The persistent kernels claim items with 32-bit partition counters that overshoot the end by
  // at most one refill per resident wave (< 2^20); frames with more items run path_kernel, whose
  // item index is 64-bit (e.g. 8192^2 x 64 spp AA = 2^32 items).
  P.persistent = persistent_supported(c->accel, c->gdim) && env_int("DRT_PERSISTENT", 1) != 0 &&
                 F.n_items < kPersistentMaxItems;
  int slots = per_pixel;                                   // sample slots per pixel
  if (P.persistent && F.mode == MODE_SEQ) {  // a lane runs a pixel's samples in order, one slot each
    slots = c->spp ? (int)c->spp : (F.grid_res ? (int)F.grid_res : 1);
    F.nsub = slots;
  }
  P.n_slots = (uint64_t)F.n_my_tiles * F.tile * F.tile * slots;
  // In-order keyed-stream frames in two passes (FrameMode MODE_SKEL / MODE_REPLAY): a random draw's
  // position in a pixel's stream depends only on the closest-hit chain of the samples before it,
  // because shadow rays draw nothing.  Pass 1 runs the pixels' samples in order but traces only
  // those chains; pass 2 runs every sample independently from its recorded position.  Without
  // refraction a sample's chain is linear (one closest hit per bounce), so the record is max_depth
  // + 1 hits per sample; a scene with a refracting material (trans == 1, main.cpp:471) keeps the
  // one-pass MODE_SEQ frame, and so do frames whose record would pass kTwoPassMaxBytes.
  P.two_pass = false;
  if (P.persistent && F.mode == MODE_SEQ && env_int("DRT_SEQ_TWO_PASS", 1) != 0 &&
      P.n_slots < kPersistentMaxItems && P.n_slots * (uint64_t)(md + 1) * 8u <= kTwoPassMaxBytes) {
    bool refr = false;
    for (const drt_material& m : c->mats) refr = refr || m.trans == 1.0f;
    P.two_pass = !refr;
  }
  // AA frames in two passes (round 4): the samples' closest-hit chains (MODE_CHAIN, one lane per
  // sample), then every sample's shading with its closest hits read back (MODE_REPLAY), whose waves
  // then hold shadow queries only and walk them on the 4-ary shadow tree.  In one pass the lanes of a
  // wave mix both query kinds and the shadow tree measured slower.  Same conditions
  // as above (no refraction, the record fits), a BVH with its shadow tree, and not a reference-order
  // frame (DRT_FRAME_REFERENCE_ORDER keeps the one-pass frame); DRT_AA_TWO_PASS=0 keeps one pass.
  // Scenes of few objects keep one pass too: their traversal is short, so the pass boundary costs
  // more than the shadow tree saves (C2, balls_low's 11 objects: 17 500 against 23 300 Mrays/s in two
  // passes; DRT_AA_TWO_PASS_MIN_PRIMS, default 1024).
  P.aa_chain = false;
  // Short frames keep one pass too: each pass ends in a tail where most CUs wait for the last lanes,
  // and the second pass adds ~0.5 ms to a frame rendered alone (shipped dragon scene, 800x600 x 16
  // spp: 2.72 / 2.15 ms Grid / BVH in two passes against 2.02 / 1.63 in one; balls_high 512^2 x 16:
  // BVH 5.21 against 4.79 ms), while longer frames gain (the 1M-triangle scene at 512^2 x 16 spp:
  // 22.3 against 24.3 ms; profiles/r04_two_pass_small_frames_ab.txt, r04_two_pass_frame_time_ab.jsonl).
  // The plan depends on the params and the scene only (round 5; round 4 read the context's last frame
  // time, so equal frames could plan differently): two passes for whole frames of >= 2^23 samples
  // (C3, the headline, their shards) or scenes of >= 2^19 objects (the 1M-triangle scene at 16 spp);
  // the shipped scenes' 16-spp frames (<= 800x600 x 16 = 7.7 M samples, <= 100 005 objects) keep one.
  // DRT_AA_TWO_PASS: 0 one pass, 1 this rule (default), 2 two passes at any size.  Both plans render
  // the same frame.
  const int aa2 = env_int("DRT_AA_TWO_PASS", 1);
  const uint64_t frame_samples = (uint64_t)P.n_tiles * F.tile * F.tile * (uint64_t)per_pixel;
  const bool big_frame = aa2 >= 2 || frame_samples >= (env_u64("DRT_AA_TWO_PASS_MIN_SAMPLES", 1ull << 23)) ||
                         (uint64_t)c->n_prims >= env_u64("DRT_AA_TWO_PASS_BIG_SCENE", 1ull << 19);
  // The Grid's AA frames too (its shadow queries stay on the Grid: Grid::Traverse(Ray&)'s answer is
  // tied to the cells its walk visits): 1 381 against 1 295 Mrays/s on the Grid headline scene.
  const bool grid_chain = c->accel == DRT_ACCEL_GRID && c->has_grid && env_int("DRT_AA_TWO_PASS_GRID", 1) != 0;
  // Scenes of mixed primitives without a refracting material take two passes at any size (round 5): their
  // one-pass kernel is the mixed-primitive path kernel (BVH 67, Grid 79 VGPR spills), while the chain pass
  // and the wavefront's shadow stream run at 7 waves/SIMD — the shipped balls_high (7 383 spheres) AA16
  // frame: BVH 5 275 -> 6 287, Grid 2 254 -> 2 415 Mrays/s; its Whitted frame on the Grid 3.48 -> 2.05
  // ms.  Triangle scenes' small frames and glass scenes' tree frames measured slower in two passes
  // (dragon AA16: BVH 5 887 -> 3 277; profiles/r05_whitted_two_pass_wavefront.jsonl, r05_gvb_aa_two_pass.jsonl).
  bool mixed_noglass = !c->tri_only;
  for (const drt_material& m : c->mats) mixed_noglass = mixed_noglass && m.trans != 1.0f;
  if (P.persistent && F.mode == MODE_AA && (big_frame || mixed_noglass) && (grid_chain || (c->accel == DRT_ACCEL_BVH && c->has_bvh && c->has_wide)) &&
      c->n_prims >= env_int("DRT_AA_TWO_PASS_MIN_PRIMS", 1024) &&
      !(p->flags & DRT_FRAME_REFERENCE_ORDER) && aa2 != 0 &&
      P.n_slots < kPersistentMaxItems && P.n_slots * (uint64_t)(md + 1) * 8u <= kTwoPassMaxBytes) {
    P.two_pass = P.aa_chain = true;
  }
  // Whitted frames in two passes too (round 5): the closest-chain pass traces ONE chain per pixel —
  // its grid_res light samples share the pixel-centre primary ray and every mirror bounce
  // (main.cpp:683-696; roughness 0, or the frame is MODE_SEQ) — and the replay pass runs every
  // (pixel, light sample) with that pixel's hits read back, its shadow queries on the shadow tree
  // (BVH) or the Grid.  Same conditions as the AA frames'; a quad-light frame of >= 4 light samples
  // at any size (the closest work shrinks grid_res times), a point-light frame by the AA size rule.
  // DRT_WHITTED_TWO_PASS=0 keeps one pass.
  // (A Grid scene of mixed primitives without a refracting material: point-light Whitted frames in two
  // passes at any size too, mixed_noglass above; measured on the Grid only.)
  P.chain_div = 1;
  const bool whitted = F.mode == MODE_WHITTED_QUAD || F.mode == MODE_WHITTED_POINT;
  const bool grid_mixed = grid_chain && mixed_noglass;
  if (P.persistent && whitted && env_int("DRT_WHITTED_TWO_PASS", 1) != 0 && aa2 != 0 &&
      (grid_chain || (c->accel == DRT_ACCEL_BVH && c->has_bvh && c->has_wide)) &&
      (F.mode == MODE_WHITTED_QUAD ? F.grid_res >= 4 || aa2 >= 2 : big_frame || grid_mixed) &&
      c->n_prims >= env_int("DRT_AA_TWO_PASS_MIN_PRIMS", 1024) && !(p->flags & DRT_FRAME_REFERENCE_ORDER) &&
      P.n_slots < kPersistentMaxItems && P.n_slots * (uint64_t)(md + 1) * 8u <= kTwoPassMaxBytes) {
    P.two_pass = P.aa_chain = true;
    P.chain_div = F.mode == MODE_WHITTED_QUAD ? (uint32_t)F.nsub : 1u;
  }
  // A scene with a refracting material (trans == 1, main.cpp:471) makes a sample's closest hits a
  // binary tree (refraction child first, then reflection): its AA / Whitted frames take two passes as
  // MODE_TCHAIN (every closest hit of the tree, recorded in rayTracing()'s query order, no shadow
  // rays) + MODE_TREPLAY (the whole rayTracing() with the hits read back in that order), when the
  // record — up to 2^(max_depth + 1) - 1 hits per sample — fits (round 5; DRT_TREE_TWO_PASS=0: one
  // pass).  Otherwise one pass, as before.
  P.tree = false;
  P.recs = (uint32_t)md + 1u;
  if (P.aa_chain) {
    bool refr = false;
    for (const drt_material& m : c->mats) refr = refr || m.trans == 1.0f;
    if (refr) {
      const uint64_t recs = (1ull << (md + 1)) - 1ull;
      const uint64_t shared = P.n_slots / P.chain_div;
      if (env_int("DRT_TREE_TWO_PASS", 1) != 0 && md <= 12 && shared * recs * 8u <= kTwoPassMaxBytes &&
          shared * recs < 0xFFFFFFFFull) {
        P.tree = true;
        P.recs = (uint32_t)recs;
      } else {
        P.two_pass = P.aa_chain = false;
        P.chain_div = 1;
      }
    }
  }
  // Pass 2 of an AA / Whitted BVH frame without refraction as a wavefront (round 5, WfArgs): every
  // shadow query of the frame generated from the recorded chains, answered by the streaming kernel,
  // combined per sample — 78.7 -> 69.3 ms on the headline (profiles/r05_ab_wavefront_replay.jsonl).
  // DRT_WAVEFRONT=0 keeps the persistent MODE_AREPLAY pass, and so does a frame of >= 2^32 query slots
  // or whose query buffers cannot be allocated (run_frame).  Both render the same frame.
  // In-order (DoF / glossy) two-pass frames too: wf_gen draws each sample's lens and reflectDir samples
  // from its recorded stream position as MODE_REPLAY does.  The frame's sample slots go through pass 2 in
  // chunks of DRT_WAVEFRONT_CHUNK_SLOTS (default 2^24: the headline in one, C4's 67 M slots in four), so
  // the query buffers stay at (max_depth + 1) x pairs x 41 B + (max_depth + 1) x 16 B per chunk slot
  // (C4: 14.8 GB per frame slot).
  P.wavefront = false;
  P.wf_chunk = 0;
  P.wf_chunks = 0;
  P.wf_fold = false;
  if (P.two_pass && !P.tree && (c->accel == DRT_ACCEL_BVH || c->accel == DRT_ACCEL_GRID) &&
      env_int("DRT_WAVEFRONT", 1) != 0 && (c->accel == DRT_ACCEL_BVH || env_int("DRT_WAVEFRONT_GRID", 1) != 0) &&
      (P.aa_chain || env_int("DRT_WAVEFRONT_INORDER", 1) != 0)) {
    // the chunk: at most DRT_WAVEFRONT_CHUNK_SLOTS slots and DRT_WAVEFRONT_CHUNK_BYTES of query buffers
    // (round 6, ADVICE r5: many lights x light_spp made a fixed 2^24-slot chunk ask for ~160 GB), whole
    // pixels (a multiple of nsub, so that wf_combine can fold the reduce)
    const uint64_t pairs = wf_pairs(c, F.light_spp);
    const uint64_t slot_bytes = ((uint64_t)md + 1u) * (pairs * 41u + 16u);
    const uint64_t budget = env_u64("DRT_WAVEFRONT_CHUNK_BYTES", 24ull << 30);
    uint64_t chunk = std::min<uint64_t>(P.n_slots, env_u64("DRT_WAVEFRONT_CHUNK_SLOTS", 1ull << 24));
    chunk = std::min<uint64_t>(chunk, budget / std::max<uint64_t>(1, slot_bytes));
    const uint64_t px = (uint64_t)std::max(1, slots);
    if (chunk > px) chunk -= chunk % px;
    chunk = std::max<uint64_t>(1, chunk);
    const uint64_t q = ((uint64_t)md + 1u) * pairs * (chunk + kWfPad);
    const uint64_t chunks = (P.n_slots + chunk - 1) / chunk;
    if (P.n_slots < 0xFFFFFFFFull && q < kPersistentMaxItems && chunks <= 4096) {
      P.wavefront = true;
      P.wf_chunk = chunk;
      P.wf_chunks = (uint32_t)chunks;
      // the reduce folded into wf_combine (whole pixels per chunk, <= 1024 samples per pixel; a wavefront
      // frame is never progressive); DRT_WAVEFRONT_FOLD=0 keeps the separate reduce launch
      P.wf_fold = chunk % px == 0 && px <= 1024 && prog == 0 && env_int("DRT_WAVEFRONT_FOLD", 1) != 0;
    }
  }
  ReduceArgs& R = P.R;
  R.nsub = slots;
  R.scale = scale;
  R.tile = F.tile; R.tiles_x = F.tiles_x; R.shard = F.shard; R.n_shards = F.n_shards; R.n_my_tiles = F.n_my_tiles;
  R.res_x = RX; R.res_y = RY;
  R.prog_frame = prog;
  return DRT_OK;
}

// Path-kernel time of the newest frame whose path kernel has finished (no waiting).
static void note_last_path_ms(drt_ctx* c) {
  const uint64_t look = std::min<uint64_t>(c->frames, 4);
  for (uint64_t k = 0; k < look; k++) {
    hipEvent_t* ev = &c->ring[drt_ctx::kEv * ((c->frames - 1 - k) % drt_ctx::kRing)];
    if (hipEventQuery(ev[1]) != hipSuccess) continue;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) c->last_path_ms = ms;
    return;
  }
}

static int run_frame(drt_ctx* c, const drt_frame_params* p, float* d_out, bool full_frame, hipStream_t st) {
  Plan P;
  int rc = plan_frame(c, p, P);
  if (rc) return rc;
  if (P.skip) return DRT_OK;
  SceneArgs S;
  rc = scene_args(c, c->accel, S, (p->flags & DRT_FRAME_REFERENCE_ORDER) != 0);
  if (rc) return rc;
  DRT_HIP(c, hipSetDevice(c->device));
  // frames on different scratch slots may run concurrently on different streams
  if (p->slot < 0 || p->slot >= DRT_FRAME_SLOTS) DRT_FAIL(c, DRT_E_INVALID, "frame slot out of range");
  const int slot = p->slot;
  DevBuf& d_samples = c->d_samples_s[slot];
  DevBuf& d_stats = c->d_stats_s[slot];
  DevBuf& d_counter = c->d_counter_s[slot];
  // The slot's scratch is reused: a frame from another stream than the slot's last frame waits for
  // that frame to end (on the device).  Frames of one stream are ordered by the stream itself.
  if (c->slot_used[slot] && c->slot_stream[slot] != st && c->frames - c->slot_frame[slot] < drt_ctx::kRing)
    DRT_HIP(c, hipStreamWaitEvent(st, c->ring[drt_ctx::kEv * (c->slot_frame[slot] % drt_ctx::kRing) + 2], 0));
  // Two-pass in-order frame: its closest-hit record is allocated first; a frame whose record does not
  // fit in device memory runs as the one-pass MODE_SEQ frame, which renders the same pixels.
  if (P.F.n_items && P.two_pass) {
    // the in-order BVH replay pass's frame heads (kReplayHeads): max_depth + 1 per lane of every block
    // the device can hold (<= 2048 threads per CU), indexed by the global thread id of the persistent grid
    if (!c->cus) DRT_HIP(c, hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device));
    const bool heads = !P.aa_chain && c->accel == DRT_ACCEL_BVH;
    const uint64_t head_bytes = sizeof(float4) * (uint64_t)std::max(1, c->cus) * 2048u * (uint64_t)(P.F.max_depth + 1);
    if ((!P.aa_chain && c->d_skel_rk_s[slot].ensure(sizeof(uint32_t) * P.n_slots) != hipSuccess) ||
        c->d_skel_hits_s[slot].ensure(sizeof(uint2) * (P.n_slots / P.chain_div) * (uint64_t)P.recs) != hipSuccess ||
        (heads && c->d_heads_s[slot].ensure(head_bytes) != hipSuccess)) {
      (void)hipGetLastError();
      c->d_skel_rk_s[slot].release();
      c->d_skel_hits_s[slot].release();
      c->d_heads_s[slot].release();
      P.two_pass = P.aa_chain = P.tree = false;
    }
  }
  // MODE_SEQ tail hand-over (DRT_SEQ_DONATE: 0 off, 1 on, default auto).  It frees whole blocks
  // at the frame's tail for the NEXT frame's blocks, but makes a frame alone slower (a handed-over
  // pixel waits for a lane of a kept wave: C4 820-828 -> 853-902 ms).  Auto turns it
  // on when another frame of this context is still in flight on another stream at issue time —
  // the pipelined case, where a frame follows on the freed CUs.
  bool handover = false;
  c->slot_handover[slot] = false;
  {
    const int dm = env_int("DRT_SEQ_DONATE", -1);
    if (dm >= 0) {
      handover = dm != 0;
    } else {
      for (int k = 0; k < DRT_FRAME_SLOTS && !handover; k++) {
        if (k == slot || !c->slot_used[k] || c->slot_stream[k] == st) continue;
        if (c->frames - c->slot_frame[k] >= drt_ctx::kRing) continue;
        handover = hipEventQuery(c->ring[drt_ctx::kEv * (c->slot_frame[k] % drt_ctx::kRing) + 2]) == hipErrorNotReady;
      }
    }
  }
  c->stats_slot = slot;
  DRT_HIP(c, d_samples.ensure(sizeof(float4) * std::max<uint64_t>(1, P.n_slots)));
  DRT_HIP(c, d_stats.ensure(sizeof(unsigned long long) * ST_COUNT));
  const bool stats = (p->flags & DRT_FRAME_STATS) != 0;
  c->stats_valid = stats;
  if (stats) DRT_HIP(c, hipMemsetAsync(d_stats.p, 0, sizeof(unsigned long long) * ST_COUNT, st));
  if (stats && P.persistent) {  // per-wave start / end stamps of the persistent launches (<= 32 waves per CU)
    if (!c->cus) DRT_HIP(c, hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device));
    c->wave_slots = (uint32_t)std::max(1, c->cus) * 32u;
    const size_t wt_bytes = sizeof(unsigned long long) * 2u * 2u * c->wave_slots;
    DRT_HIP(c, c->d_wave_times.ensure(wt_bytes));
    DRT_HIP(c, hipMemsetAsync(c->d_wave_times.p, 0, wt_bytes, st));
    P.F.wave_times = c->d_wave_times.as<unsigned long long>();
  }
  P.F.samples = d_samples.as<float4>();
  P.F.stats = d_stats.as<unsigned long long>();
  P.R.samples = P.F.samples;
  P.R.full_frame = full_frame ? 1 : 0;
  P.R.out = d_out;
  // per-pixel sample shuffle, once per pixel instead of once per sample (spp < 2: no shuffle); ahead
  // of the frame's first event, so that the path-kernel time is the persistent kernel's own
  const bool shuffled = P.F.mode == MODE_AA || (P.F.mode == MODE_SEQ && P.F.spp > 0);
  const int aux_mode = env_int("DRT_AUX_STREAMS", -1);
  if (aux_mode < 0) note_last_path_ms(c);
  const bool use_aux = aux_mode > 0 || (aux_mode < 0 && c->last_path_ms >= drt_ctx::kAuxMinMs);
  hipStream_t ax = use_aux ? c->aux[slot] : st;
  if (P.persistent && shuffled && P.F.spp >= 2 && P.F.spp <= 256 && P.F.n_items && env_int("DRT_PERM", 1)) {
    DevBuf& d_perm = c->d_perm_s[slot];
    DRT_HIP(c, d_perm.ensure((size_t)P.F.n_my_tiles * P.F.tile * P.F.tile * P.F.spp));
    // the slot's previous path kernel reads the permutation this shuffle rewrites (on the caller's
    // stream that order is the stream's own, or the slot wait above)
    if (use_aux && c->path_issued[slot]) DRT_HIP(c, hipStreamWaitEvent(ax, c->ev_path[slot], 0));
    launch_shuffle(P.F, c->cam.res_x, c->cam.res_y, d_perm.as<uint8_t>(), ax);
    P.F.perm = d_perm.as<uint8_t>();
    DRT_HIP(c, hipGetLastError());
    if (use_aux) {
      DRT_HIP(c, hipEventRecord(c->ev_shuf[slot], ax));
      DRT_HIP(c, hipStreamWaitEvent(st, c->ev_shuf[slot], 0));
    }
  }
  hipEvent_t* ev = &c->ring[drt_ctx::kEv * (c->frames % drt_ctx::kRing)];
  c->slot_frame[slot] = c->frames;
  c->slot_stream[slot] = st;
  c->slot_used[slot] = true;
  c->frames++;
  DRT_HIP(c, hipEventRecord(ev[0], st));
  const bool persistent = P.persistent;
  if (persistent) {
    // 8 partition counters, 64 B apart, per pass: a two-pass frame's second pass uses the second
    // KiB, zeroed here too, so that no fill kernel sits between the passes (a fill waits for a CU
    // slot behind the other frames' persistent blocks, and the second pass behind it)
    // (a wavefront pass 2: one KiB of counters per chunk, from the second KiB on)
    const size_t counter_bytes = 1024u * (1u + (P.two_pass ? std::max<uint32_t>(1u, P.wf_chunks) : 0u));
    DRT_HIP(c, d_counter.ensure(std::max<size_t>(2048, counter_bytes)));
    DRT_HIP(c, hipMemsetAsync(d_counter.p, 0, counter_bytes, st));
    P.F.work_counter = d_counter.as<unsigned int>();
    P.F.part_items = (uint32_t)((P.F.n_items + 7) / 8);
    P.F.refill_min = env_int("DRT_REFILL_MIN", 8);
    P.F.process_min = env_int("DRT_PROCESS_MIN", 24);
    P.F.waves = env_int("DRT_WAVES", c->accel == DRT_ACCEL_GRID ? 5 : 6);
    P.F.grid_pairs = std::max(1, env_int("DRT_GRID_PAIRS", 3));  // >= 1: a lane must make progress
    P.F.grid_walk = std::max(0, env_int("DRT_GRID_WALK", 5));
    // MODE_SEQ tail hand-over (`handover` above)
    if (P.F.mode == MODE_SEQ && handover && !P.two_pass) {
      c->slot_handover[slot] = true;
      if (!c->cus) DRT_HIP(c, hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device));
      const uint32_t cap = (uint32_t)std::max(1, c->cus) * 2048u;  // 32 waves of 64 lanes per CU at most
      DevBuf& d_cont = c->d_cont_s[slot];
      DRT_HIP(c, d_cont.ensure(sizeof(unsigned long long) * cap));
      DRT_HIP(c, hipMemsetAsync(d_cont.p, 0, sizeof(unsigned long long) * cap, st));
      P.F.seq_cont = d_cont.as<unsigned long long>();
      P.F.seq_cap = cap;
      // Kept waves: exactly what the unfinished pixels need.  More (slack above 100 %) and a higher
      // idle-lane threshold for pops measured 1.5-4x slower frames (contention on the one push/pop
      // line): the slack is fixed and the threshold clamped to the range that measured
      // sane.
      P.F.seq_slack = 100;
      P.F.seq_pop_min = std::min(32, std::max(1, env_int("DRT_SEQ_POP_MIN", 8)));
      P.F.seq_backlog = (uint32_t)std::max(0, env_int("DRT_SEQ_BACKLOG", 0));
    }  // with pairs 3, 5 waves: 1 300 Mrays/s; (walk, pairs) = (8, 4) 1 228, (6, 3) 1 272, (4, 3) 1 235-1 319, (5, 2) 1 275
  }
  bool folded = false;  // the reduce ran inside wf_combine
  if (P.F.n_items && P.two_pass) {
    DevBuf& d_rk = c->d_skel_rk_s[slot];  // allocated above
    DevBuf& d_hits = c->d_skel_hits_s[slot];
    // pass 2 as a wavefront (plan_frame): the query buffers, or the persistent replay if they do not fit
    bool wavefront = false;
    WfArgs W{};
    if (P.wavefront) {
      const uint64_t levels = (uint64_t)P.F.max_depth + 1u, pairs = wf_pairs(c, P.F.light_spp);
      const uint64_t q = levels * pairs * (P.wf_chunk + kWfPad);  // (+ the bands' padding, wf_q)
      const bool compact = wf_compact(c);
      const uint64_t cnt_bytes = levels * ((P.wf_chunk + kWfPad) / 64u + 8u) + 4u;
      if (c->d_wf_rays_s[slot].fit(2 * sizeof(float4) * std::max<uint64_t>(q, 1)) == hipSuccess &&
          c->d_wf_nl_s[slot].fit(sizeof(float2) * std::max<uint64_t>(q, 1)) == hipSuccess &&
          c->d_wf_occ_s[slot].fit(std::max<uint64_t>(q, 1)) == hipSuccess &&
          c->d_wf_lvl_s[slot].fit(sizeof(float4) * levels * P.wf_chunk) == hipSuccess &&
          (!compact || c->d_wf_cnt_s[slot].fit(cnt_bytes) == hipSuccess) &&
          (!(compact && c->accel == DRT_ACCEL_GRID && c->has_gv) ||
           c->d_wf_fb_s[slot].fit(2 * sizeof(float4) * std::max<uint64_t>(q, 1)) == hipSuccess)) {
        wavefront = true;
        W.rays = c->d_wf_rays_s[slot].as<float4>();
        W.rays_b = W.rays + std::max<uint64_t>(q, 1);
        W.nl = c->d_wf_nl_s[slot].as<float2>();
        W.occ = c->d_wf_occ_s[slot].as<uint8_t>();
        W.lvl = c->d_wf_lvl_s[slot].as<float4>();
        W.pairs = (int)pairs;
        W.levels = (int)levels;
        W.grid = c->accel == DRT_ACCEL_GRID ? 1 : 0;
        W.inorder = P.aa_chain ? 0 : 1;
        W.compact = compact ? 1 : 0;
        W.cnt = compact ? c->d_wf_cnt_s[slot].as<uint8_t>() : nullptr;
      } else {
        (void)hipGetLastError();
        for (DevBuf* b : {&c->d_wf_rays_s[slot], &c->d_wf_nl_s[slot], &c->d_wf_occ_s[slot], &c->d_wf_lvl_s[slot],
                          &c->d_wf_cnt_s[slot], &c->d_wf_fb_s[slot]})
          b->release();
      }
    }
    FrameArgs F1 = P.F;  // pass 1: the pixels' closest-hit chains, samples in order (AA: any order)
    F1.mode = P.tree ? MODE_TCHAIN : (P.aa_chain ? MODE_CHAIN : MODE_SKEL);
    F1.tree_recs = (int)P.recs;
    F1.skel_rk = P.aa_chain ? nullptr : d_rk.as<uint32_t>();
    F1.skel_hits = d_hits.as<uint2>();
    F1.aa_chain = P.aa_chain ? 1 : 0;
    F1.chain_div = (int)P.chain_div;
    if (P.chain_div > 1) {  // a Whitted frame's closest-chain pass: one lane per pixel
      F1.nsub = 1;
      F1.n_items = P.F.n_items / P.chain_div;
      F1.part_items = (uint32_t)((F1.n_items + 7) / 8);
    }
    if (P.aa_chain) {  // the closest-chain pass carries little state
      // its "shading" is recording a hit and starting the mirror ray: batches of 8 ready lanes
      // measured 1 927 against 1 897 Mrays/s for 24 (1: 1 842, 48: 1 725; profiles/r04_pass_knobs_ab.jsonl)
      // (Grid: 5 waves, 1 381 against 1 318 Mrays/s at 6 on the Grid headline scene;
      // profiles/r04_grid_two_pass_wide_order_ab.jsonl)
      // (7 waves since round 5 — the chain pass has its own instantiation and no spills at 6 since
      // MODE_AREPLAY split off: BVH 2 534-2 545 against 2 483-2 488 Mrays/s, C3 3 471-3 473 against 3 425;
      // Grid 1 963-1 967 against 1 872-1 876 at 5 (6: 1 930); round 4 measured 1 785 against 1 897 at 7 on
      // the BVH; profiles/r05_chain_knobs.jsonl, r05_grid_waves.jsonl)
      F1.waves = env_int("DRT_CHAIN_WAVES", 7);
      F1.process_min = env_int("DRT_CHAIN_PROCESS_MIN", 8);
      F1.refill_min = env_int("DRT_CHAIN_REFILL_MIN", P.F.refill_min);  // 16 measured 1 868
      // Grid: 3 empty cells per call in both passes of an AA two-pass frame (1 420 against 1 383 Mrays/s
      // at the one-pass frame's 5; 2: 1 413; profiles/r04_hit_normals_grid_walk_ab.jsonl)
      F1.grid_walk = std::max(0, env_int("DRT_CHAIN_GRID_WALK", 3));
      F1.grid_pairs = std::max(1, env_int("DRT_CHAIN_GRID_PAIRS", P.F.grid_pairs));
    } else {
      F1.process_min = env_int("DRT_SKEL_PROCESS_MIN", P.F.process_min);
    }
    F1.seq_cont = nullptr;
    // (Measured alternative, kept out: the AA closest-chain pass writing each level's shadow queries and
    // record itself instead of wf_gen reading the hits back — its code in the chain loop cost 14 VGPR
    // spills, 2 339 against 2 380 Mrays/s fused / unfused in that build and 2 475 without it;
    // profiles/r05_ab_fused_chain_gen.jsonl.)
    launch_path_persistent(S, F1, c->accel, c->tri_only, stats, st);
    DRT_HIP(c, hipGetLastError());
    DRT_HIP(c, hipEventRecord(ev[3], st));  // end of pass 1 (drt_frame_pass_times)
    FrameArgs F2 = F1;  // pass 2: every sample on its own, closest hits read back
    F2.mode = P.tree ? MODE_TREPLAY : (P.aa_chain ? MODE_AREPLAY : MODE_REPLAY);
    F2.heads = (!P.aa_chain && c->accel == DRT_ACCEL_BVH) ? c->d_heads_s[slot].as<float4>() : nullptr;
    F2.nsub = P.F.nsub;
    F2.waves = env_int("DRT_REPLAY_WAVES", P.F.waves);
    F2.process_min = env_int("DRT_REPLAY_PROCESS_MIN", P.F.process_min);  // 12 / 40: 1 861 / 1 764 vs 1 897
    F2.refill_min = env_int("DRT_REPLAY_REFILL_MIN", P.F.refill_min);
    F2.grid_walk = std::max(0, env_int("DRT_REPLAY_GRID_WALK", P.aa_chain ? 3 : P.F.grid_walk));
    F2.grid_pairs = std::max(1, env_int("DRT_REPLAY_GRID_PAIRS", P.F.grid_pairs));
    F2.n_items = P.n_slots;
    F2.part_items = (uint32_t)((F2.n_items + 7) / 8);
    F2.work_counter = d_counter.as<unsigned int>() + 256;
    if (F2.wave_times) F2.wave_times += 2u * c->wave_slots;  // pass 2's launches (persistent replay / MODE_QSTREAM)
    if (wavefront) {  // drt_frame_stage_times: this frame's launches
      if (c->stage_ev.empty()) {
        c->stage_ev.assign(3 * drt_ctx::kStageChunks, nullptr);
        for (auto& e : c->stage_ev) DRT_HIP(c, hipEventCreate(&e));
      }
      c->stage_chunks = 0;
      c->stage_frame_ev = (int)(drt_ctx::kEv * ((c->frames - 1) % drt_ctx::kRing));
    }
    for (uint32_t k = 0; wavefront && k < P.wf_chunks; k++) {
      W.slot0 = (uint32_t)(k * P.wf_chunk);
      W.n_slots = (uint32_t)std::min<uint64_t>(P.wf_chunk, P.n_slots - W.slot0);
      // XCD bands (wf_q): DRT_WAVEFRONT_BANDS (1 or 8) consecutive ranges of the chunk's sample slots, each
      // streamed first by one XCD.  BVH 8: headline +0.2 %, C3 +0.8 %; the Grid's MODE_QSTREAM measured
      // 6 % slower with them and keeps 1 (profiles/r05_ab_wavefront_bands.jsonl); the Grid's grid_stream
      // (round 6, compact queries) gains 2.7 % with them: 2 079 / 2 066 against 2 023 / 2 020 Mrays/s
      // (profiles/r06_ab_grid_stream.jsonl)
      W.bands = env_int("DRT_WAVEFRONT_BANDS", (W.grid && !W.compact) ? 1 : 8) >= 8 ? 8 : 1;
      W.band = (W.n_slots + (uint32_t)W.bands - 1u) / (uint32_t)W.bands;
      if (W.compact) W.band = (W.band + 255u) & ~255u;  // 64-slot groups, 256-query chunks, one (level, pair) row each
      launch_wf_gen(S, F2, W, st);
      DRT_HIP(c, hipGetLastError());
      const bool stage = k < (uint32_t)drt_ctx::kStageChunks && !c->stage_ev.empty();
      if (stage) DRT_HIP(c, hipEventRecord(c->stage_ev[3 * k], st));
      const uint64_t q = (uint64_t)W.levels * (uint64_t)W.pairs * W.band * (uint64_t)W.bands;
      const uint32_t part_len = (uint32_t)((uint64_t)W.levels * W.pairs * W.band);
      unsigned int* counter = d_counter.as<unsigned int>() + 256u * (1u + k);
      if (q && W.grid && W.compact) {
        // the Grid's shadow queries on its own streaming kernel (grid_stream, round 6): the Grid stepper,
        // refilled from the compact query array like trace_stream
        TraceArgs A{};
        A.rays = W.rays;
        A.rays_b = W.rays_b;
        A.stride = 1;
        A.n = (uint32_t)q;
        A.counter = counter;
        A.occ_out = W.occ;
        A.stats = F2.stats;
        A.refill_min = env_int("DRT_WAVEFRONT_GRID_REFILL_MIN", 16);
        A.sparse = 2;
        A.cnt = W.cnt;
        A.levels = W.levels;
        A.pairs = W.pairs;
        A.band = W.band;
        A.parts = W.bands;
        A.part_len = W.bands == 8 ? part_len : (uint32_t)q;
        // (round 6) the Grid scene's shadow tree answers the queries it can certify, the Grid walk the rest
        // (trace_stream GV + grid_fallback).  Stats frames keep the walk, so that their work
        // counters stay the reference's cell / object counts (DRT_GRID_SHADOW_TREE=2: the tree there too,
        // its work in the wide_* counters); DRT_GRID_SHADOW_TREE=0: the walk for every frame.
        const int gv = env_int("DRT_GRID_SHADOW_TREE", 1);
        if (c->has_gv && c->tri_only && c->d_wf_fb_s[slot].p && (gv >= 2 || (gv == 1 && !stats))) {
          SceneArgs ST = S;
          ST.prims = c->d_gv_prims.as<float4>();
          ST.wnodes = c->d_gv_wnodes.as<float4>();
          ST.wleaf = c->d_gv_range.as<float4>();
          ST.wroot = c->gv_wroot;
          ST.big_leaves = c->d_gv_big.as<uint2>();
          // refill at 16 idle lanes: 2 162-2 165 against 2 148 Mrays/s at the BVH stream's 12 (8: 2 098; 6 waves
          // instead of 7: 2 138-2 145; profiles/r06_ab_grid_shadow_tree_knobs.jsonl)
          A.refill_min = env_int("DRT_GRID_TREE_REFILL_MIN", 16);
          A.fb_rays = c->d_wf_fb_s[slot].as<float4>();
          A.fb_count = counter + 224;  // (zeroed with the chunk's claim counters)
          launch_grid_tree_stream(ST, S, A, stats, env_int("DRT_WAVEFRONT_WAVES", 7), F2.grid_walk, F2.grid_pairs,
                                  counter + 240, st);
        } else {
          launch_grid_stream(S, A, c->tri_only, stats, env_int("DRT_WAVEFRONT_GRID_WAVES", 7), F2.grid_walk, F2.grid_pairs, st);
        }
        DRT_HIP(c, hipGetLastError());
      } else if (q && W.grid) {
        // the Grid's shadow queries on its persistent stepper (MODE_QSTREAM): Grid::Traverse(Ray&)'s answer
        // is tied to the cells its walk visits, so they stay on the Grid
        FrameArgs FQ = F2;
        FQ.mode = MODE_QSTREAM;
        FQ.n_items = q;
        FQ.part_items = W.bands == 8 ? part_len : (uint32_t)((q + 7) / 8);
        FQ.q_rays = W.rays;
        FQ.q_rays_b = W.rays_b;
        FQ.q_occ = W.occ;
        FQ.work_counter = counter;
        FQ.process_min = 1;
        // refill at 16 idle lanes: 1 875 against 1 758 Mrays/s at the path kernel's 8 (24: 1 874-1 878,
        // 32: 1 809, 4: 1 576; profiles/r05_grid_qstream_knobs*.jsonl)
        FQ.refill_min = env_int("DRT_WAVEFRONT_GRID_REFILL_MIN", 16);
        FQ.waves = env_int("DRT_WAVEFRONT_GRID_WAVES", 7);  // 7: +0.7 % against 5 (r05_grid_waves.jsonl)
        launch_path_persistent(S, FQ, c->accel, c->tri_only, stats, st);
        DRT_HIP(c, hipGetLastError());
      } else if (q) {
        TraceArgs A{};
        A.rays = W.rays;
        A.rays_b = W.rays_b;
        A.stride = 1;
        A.n = (uint32_t)q;
        A.counter = counter;
        A.occ_out = W.occ;
        A.stats = F2.stats;
        // 7 waves / SIMD and refill at 12 idle lanes: 2 487-2 491 Mrays/s on the headline against 2 235 at
        // the batched queries' 6 / 24 (7 / 16: 2 475-2 480, 7 / 10: 2 479-2 489, 8 / 16: 2 393-2 400,
        // 6 / 16: 2 431; C3 at 12 / 16: 3 430 / 3 425-3 427; r05_wavefront_knobs_*.jsonl)
        A.refill_min = env_int("DRT_WAVEFRONT_REFILL_MIN", 12);
        A.sparse = W.compact ? 2 : 1;
        A.cnt = W.cnt;
        A.levels = W.levels;
        A.pairs = W.pairs;
        A.band = W.band;
        A.parts = W.bands;
        A.part_len = W.bands == 8 ? part_len : (uint32_t)q;
        launch_trace_stream(S, A, true, c->tri_only, stats, env_int("DRT_WAVEFRONT_WAVES", 7), st);
        DRT_HIP(c, hipGetLastError());
      }
      if (stage) DRT_HIP(c, hipEventRecord(c->stage_ev[3 * k + 1], st));
      if (P.wf_fold) launch_wf_combine_reduce(S, F2, W, P.R, st);
      else launch_wf_combine(S, F2, W, st);
      DRT_HIP(c, hipGetLastError());
      if (stage) DRT_HIP(c, hipEventRecord(c->stage_ev[3 * k + 2], st));
      if (stage) c->stage_chunks = (int)k + 1;
    }
    folded = wavefront && P.wf_fold;
    if (!wavefront) launch_path_persistent(S, F2, c->accel, c->tri_only, stats, st);
  } else if (P.F.n_items) {
    if (persistent) launch_path_persistent(S, P.F, c->accel, c->tri_only, stats, st);
    else launch_path(S, P.F, c->accel, c->tri_only, stats, st);
  }
  DRT_HIP(c, hipGetLastError());
  if (!(P.F.n_items && P.two_pass)) DRT_HIP(c, hipEventRecord(ev[3], st));  // one pass: pass 1 is the frame
  DRT_HIP(c, hipEventRecord(ev[1], st));
  DRT_HIP(c, hipEventRecord(c->ev_path[slot], st));  // every frame: the slot's last path kernel
  c->path_issued[slot] = true;
  if (P.F.n_my_tiles && !folded) {
    if (use_aux) DRT_HIP(c, hipStreamWaitEvent(ax, c->ev_path[slot], 0));
    launch_reduce(P.R, ax);
    DRT_HIP(c, hipGetLastError());
    if (use_aux) {
      DRT_HIP(c, hipEventRecord(c->ev_red[slot], ax));
      DRT_HIP(c, hipStreamWaitEvent(st, c->ev_red[slot], 0));
    }
  }
  DRT_HIP(c, hipEventRecord(ev[2], st));
  return DRT_OK;
}

extern "C" {

int drt_shard_layout(const drt_ctx* c, const drt_frame_params* p, int64_t* tiles, int64_t* floats) {
  if (!c || !p) return DRT_E_INVALID;
  Plan P;
  int rc = plan_frame(const_cast<drt_ctx*>(c), p, P);
  if (rc) return rc;
  const int shards = P.F.n_shards;
  const int64_t per_shard = (P.n_tiles + shards - 1) / shards;  // equal-size shard buffers
  if (tiles) *tiles = P.F.n_my_tiles;
  if (floats) *floats = per_shard * P.F.tile * P.F.tile * 3;
  return DRT_OK;
}

int drt_plan_frame(const drt_ctx* c, const drt_frame_params* p, drt_frame_plan* out) {
  if (!c || !p || !out) return DRT_E_INVALID;
  Plan P;
  int rc = plan_frame(const_cast<drt_ctx*>(c), p, P);
  if (rc) return rc;
  memset(out, 0, sizeof(*out));
  out->work_items = P.F.n_items;
  out->sample_slots = P.n_slots;
  out->mode = P.F.mode;
  out->persistent = P.persistent ? 1 : 0;
  out->tiles_in_shard = P.F.n_my_tiles;
  out->passes = P.two_pass ? 2 : 1;
  out->wavefront = P.wavefront ? 1 : 0;
  return DRT_OK;
}

int drt_frame_resolution(const drt_ctx* c, int32_t res_xy[2]) {
  if (!c || !res_xy) return DRT_E_INVALID;
  if (!c->has_scene) return DRT_E_STATE;
  res_xy[0] = c->cam.res_x;
  res_xy[1] = c->cam.res_y;
  return DRT_OK;
}

int drt_render_device(drt_ctx* c, const drt_frame_params* p, float* d_out, void* stream) {
  if (!c || !p || !d_out) return DRT_E_INVALID;
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  const bool full = (p->n_shards <= 1) && !(p->flags & DRT_FRAME_SHARD_LAYOUT);
  return run_frame(c, p, d_out, full, st);
}

int drt_unshard_device(drt_ctx* c, const drt_frame_params* p, const float* d_shards, float* d_frame, void* stream) {
  if (!c || !p || !d_shards || !d_frame) return DRT_E_INVALID;
  Plan P;
  int rc = plan_frame(c, p, P);
  if (rc) return rc;
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  const int shards = P.F.n_shards;
  const int per_shard = (P.n_tiles + shards - 1) / shards;
  DRT_HIP(c, hipSetDevice(c->device));
  launch_unshard(d_shards, d_frame, P.F.tile, P.F.tiles_x, P.n_tiles, shards, per_shard, c->cam.res_x, c->cam.res_y, st);
  DRT_HIP(c, hipGetLastError());
  return DRT_OK;
}

int drt_render(drt_ctx* c, const drt_frame_params* p, float* rgb_out) {
  if (!c || !p || !rgb_out) return DRT_E_INVALID;
  if (p->n_shards > 1) DRT_FAIL(c, DRT_E_INVALID, "drt_render renders whole frames; use drt_render_device for shards");
  const size_t n = (size_t)c->cam.res_x * c->cam.res_y * 3;
  if (p->progressive_frame >= 10000) return DRT_OK;  // MAX_SAMPLES reached: output untouched
  DRT_HIP(c, hipSetDevice(c->device));
  DRT_HIP(c, c->d_frame.ensure(sizeof(float) * n));
  if (p->progressive_frame > 1)  // the lerp reads the previous frame
    DRT_HIP(c, hipMemcpyAsync(c->d_frame.p, rgb_out, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  int rc = run_frame(c, p, c->d_frame.as<float>(), true, c->stream);
  if (rc) return rc;
  DRT_HIP(c, hipMemcpyAsync(rgb_out, c->d_frame.p, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  DRT_HIP(c, hipStreamSynchronize(c->stream));
  return DRT_OK;
}

int drt_frame_times(drt_ctx* c, int max_frames, double* path_ms, double* total_ms) {
  if (!c || max_frames < 0) return DRT_E_INVALID;
  const uint64_t have = std::min<uint64_t>(c->frames, (uint64_t)drt_ctx::kRing);
  const int n = (int)std::min<uint64_t>(have, (uint64_t)max_frames);
  for (int i = 0; i < n; i++) {
    const uint64_t f = c->frames - (uint64_t)n + (uint64_t)i;
    hipEvent_t* ev = &c->ring[drt_ctx::kEv * (f % drt_ctx::kRing)];
    DRT_HIP(c, hipEventSynchronize(ev[2]));
    float a = 0, b = 0;
    DRT_HIP(c, hipEventElapsedTime(&a, ev[0], ev[1]));
    DRT_HIP(c, hipEventElapsedTime(&b, ev[0], ev[2]));
    if (path_ms) path_ms[i] = a;
    if (total_ms) total_ms[i] = b;
  }
  return n;
}

int drt_frame_pass_times(drt_ctx* c, int max_frames, double* pass1_ms, double* pass2_ms) {
  if (!c || max_frames < 0) return DRT_E_INVALID;
  const uint64_t have = std::min<uint64_t>(c->frames, (uint64_t)drt_ctx::kRing);
  const int n = (int)std::min<uint64_t>(have, (uint64_t)max_frames);
  if (n) DRT_HIP(c, hipSetDevice(c->device));
  for (int i = 0; i < n; i++) {
    const uint64_t f = c->frames - (uint64_t)n + (uint64_t)i;
    hipEvent_t* ev = &c->ring[drt_ctx::kEv * (f % drt_ctx::kRing)];
    DRT_HIP(c, hipEventSynchronize(ev[2]));
    float a = 0, b = 0;
    DRT_HIP(c, hipEventElapsedTime(&a, ev[0], ev[3]));
    DRT_HIP(c, hipEventElapsedTime(&b, ev[3], ev[1]));
    if (pass1_ms) pass1_ms[i] = a;
    if (pass2_ms) pass2_ms[i] = b;
  }
  return n;
}

int drt_frame_stage_times(drt_ctx* c, double out_ms[3]) {
  if (!c || !out_ms) return DRT_E_INVALID;
  if (c->stage_chunks <= 0 || c->stage_frame_ev < 0) DRT_FAIL(c, DRT_E_STATE, "no wavefront frame recorded");
  DRT_HIP(c, hipSetDevice(c->device));
  out_ms[0] = out_ms[1] = out_ms[2] = 0.0;
  hipEvent_t prev = c->ring[c->stage_frame_ev + 3];  // end of pass 1
  for (int k = 0; k < c->stage_chunks; k++) {
    hipEvent_t* e = &c->stage_ev[3 * k];
    DRT_HIP(c, hipEventSynchronize(e[2]));
    float a = 0, b = 0, d = 0;
    DRT_HIP(c, hipEventElapsedTime(&a, prev, e[0]));
    DRT_HIP(c, hipEventElapsedTime(&b, e[0], e[1]));
    DRT_HIP(c, hipEventElapsedTime(&d, e[1], e[2]));
    out_ms[0] += a; out_ms[1] += b; out_ms[2] += d;
    prev = e[2];
  }
  return c->stage_chunks;
}

int drt_frame_wave_times(drt_ctx* c, int pass, uint64_t* start_end, int64_t max_waves) {
  if (!c || pass < 0 || pass > 1 || max_waves < 0 || (max_waves && !start_end)) return DRT_E_INVALID;
  if (!c->stats_valid || !c->d_wave_times.p) DRT_FAIL(c, DRT_E_STATE, "no stats frame with wave stamps");
  DRT_HIP(c, hipSetDevice(c->device));
  DRT_HIP(c, hipDeviceSynchronize());
  const int64_t n = std::min<int64_t>(max_waves, (int64_t)c->wave_slots);
  if (n) {
    DRT_HIP(c, hipMemcpy(start_end, c->d_wave_times.as<unsigned long long>() + 2u * c->wave_slots * (uint32_t)pass,
                         sizeof(uint64_t) * 2u * (size_t)n, hipMemcpyDeviceToHost));
  }
  return (int)n;
}

int drt_frame_spans(drt_ctx* c, int max_frames, double* path_start, double* path_end, double* frame_end) {
  if (!c || max_frames < 0) return DRT_E_INVALID;
  const uint64_t have = std::min<uint64_t>(c->frames, (uint64_t)drt_ctx::kRing);
  const int n = (int)std::min<uint64_t>(have, (uint64_t)max_frames);
  if (n == 0) return 0;
  DRT_HIP(c, hipSetDevice(c->device));
  const uint64_t f0 = c->frames - (uint64_t)n;
  hipEvent_t base = c->ring[drt_ctx::kEv * (f0 % drt_ctx::kRing)];
  for (int i = 0; i < n; i++) {
    hipEvent_t* ev = &c->ring[drt_ctx::kEv * ((f0 + (uint64_t)i) % drt_ctx::kRing)];
    DRT_HIP(c, hipEventSynchronize(ev[2]));
    float a = 0, b = 0, e = 0;
    DRT_HIP(c, hipEventElapsedTime(&a, base, ev[0]));
    DRT_HIP(c, hipEventElapsedTime(&b, base, ev[1]));
    DRT_HIP(c, hipEventElapsedTime(&e, base, ev[2]));
    if (path_start) path_start[i] = a;
    if (path_end) path_end[i] = b;
    if (frame_end) frame_end[i] = e;
  }
  return n;
}

int drt_get_stats(drt_ctx* c, drt_frame_stats* out) {
  if (!c || !out) return DRT_E_INVALID;
  memset(&c->last, 0, sizeof(c->last));
  if (c->frames > 0) {
    hipEvent_t* ev = &c->ring[drt_ctx::kEv * ((c->frames - 1) % drt_ctx::kRing)];
    DRT_HIP(c, hipSetDevice(c->device));
    DRT_HIP(c, hipEventSynchronize(ev[2]));
    float ms_k = 0, ms_all = 0;
    DRT_HIP(c, hipEventElapsedTime(&ms_k, ev[0], ev[1]));
    DRT_HIP(c, hipEventElapsedTime(&ms_all, ev[0], ev[2]));
    c->last.kernel_ms = ms_k;
    c->last.render_ms = ms_all;
    if (c->stats_valid) {
      unsigned long long s[ST_COUNT];
      DRT_HIP(c, hipMemcpy(s, c->d_stats_s[c->stats_slot].p, sizeof(s), hipMemcpyDeviceToHost));
      c->last.closest_rays = s[ST_CLOSEST]; c->last.shadow_rays = s[ST_SHADOW];
      c->last.closest_inner = s[ST_C_INNER]; c->last.closest_leaf = s[ST_C_LEAF];
      c->last.shadow_inner = s[ST_S_INNER]; c->last.shadow_leaf = s[ST_S_LEAF];
      c->last.closest_prims = s[ST_C_PRIMS]; c->last.shadow_prims = s[ST_S_PRIMS];
      c->last.samples = s[ST_SAMPLES];
      c->last.wave_node_iters = s[ST_WAVE_NODE_ITERS];
      c->last.wave_path_iters = s[ST_WAVE_PATH_ITERS];
      c->last.lane_path_iters = s[ST_LANE_PATH_ITERS];
      c->last.cycles_refill = s[ST_CYC_REFILL];
      c->last.cycles_node = s[ST_CYC_NODE];
      c->last.cycles_shade = s[ST_CYC_PROC];
      c->last.stack_pushes = s[ST_PUSH];
      c->last.stack_spills = s[ST_PUSH_SPILL];
      c->last.wave_leaf_iters = s[ST_WAVE_LEAF_ITERS];
      c->last.cycles_leaf = s[ST_CYC_LEAF];
      c->last.wide_shadow_rays = s[ST_W_RAYS];
      c->last.wide_inner = s[ST_W_INNER];
      c->last.wide_leaf = s[ST_W_LEAF];
      c->last.wide_prims = s[ST_W_PRIMS];
      c->last.wide_verify = s[ST_W_VERIFY];
      c->last.wide_grid_walks = s[ST_W_GRIDFB];
    }
    c->last.seq_handover = c->slot_handover[c->stats_slot] ? 1 : 0;
    if (c->last.seq_handover) {  // push / pop counts of the frame's continuation slots
      uint32_t pp[2] = {0, 0};
      DRT_HIP(c, hipMemcpy(pp, c->d_counter_s[c->stats_slot].as<unsigned int>() + kSeqPush, sizeof(pp),
                           hipMemcpyDeviceToHost));
      c->last.seq_pushed = pp[0];
      c->last.seq_popped = pp[1];
    }
  }
  *out = c->last;
  return DRT_OK;
}

// Batched queries on device buffers, asynchronous on st.  BVH: prep -> streaming traversal
// (timed with the context's trace events) -> closest-hit epilogue; Grid / NONE: trace_kernel.
static int trace_device(drt_ctx* c, const float* d_rays, int32_t n, int shadow, float* dt, float* dn, int32_t* dobj,
                        uint8_t* docc, hipStream_t st) {
  SceneArgs S;
  if (!c->has_scene) DRT_FAIL(c, DRT_E_STATE, "no scene uploaded");
  int rc = scene_args(c, c->accel, S, (c->trace_flags & DRT_FRAME_REFERENCE_ORDER) != 0);
  if (rc) return rc;
  DRT_HIP(c, hipSetDevice(c->device));
  c->trace_timed = false;
  c->trace_stats_valid = false;
  if (c->accel != DRT_ACCEL_BVH) {
    launch_trace(S, c->accel, c->tri_only, d_rays, n, shadow, dt, dn, dobj, docc, st);
    DRT_HIP(c, hipGetLastError());
    return DRT_OK;
  }
  if (c->trace_issued) {  // serialise with the previous batched query of this context
    if (c->d_tq.bytes < 2 * sizeof(float4) * (size_t)n || c->d_tprim.bytes < sizeof(uint32_t) * (size_t)n)
      DRT_HIP(c, hipEventSynchronize(c->tev[2]));  // about to regrow buffers it may still read
    DRT_HIP(c, hipStreamWaitEvent(st, c->tev[2], 0));
  }
  DRT_HIP(c, c->d_tq.ensure(2 * sizeof(float4) * (size_t)n));
  DRT_HIP(c, c->d_tprim.ensure(sizeof(uint32_t) * (size_t)n));
  DRT_HIP(c, c->d_counter.ensure(1024));
  DRT_HIP(c, c->d_tstats.ensure(sizeof(unsigned long long) * ST_COUNT));
  const bool stats = (c->trace_flags & DRT_FRAME_STATS) != 0;
  float4* q = c->d_tq.as<float4>();
  launch_trace_prep(d_rays, n, shadow, q, st);
  DRT_HIP(c, hipMemsetAsync(c->d_counter.p, 0, 256, st));
  if (stats) DRT_HIP(c, hipMemsetAsync(c->d_tstats.p, 0, sizeof(unsigned long long) * ST_COUNT, st));
  TraceArgs A{};
  A.rays = q;
  A.rays_b = q + 1;
  A.stride = 2;
  A.n = (uint32_t)n;
  A.counter = c->d_counter.as<unsigned int>();
  A.t_out = dt;
  A.prim_out = c->d_tprim.as<uint32_t>();
  A.occ_out = docc;
  A.stats = c->d_tstats.as<unsigned long long>();
  A.refill_min = env_int("DRT_TRACE_REFILL_MIN", 24);
  A.parts = 1;
  A.part_len = (uint32_t)n;
  DRT_HIP(c, hipEventRecord(c->tev[0], st));
  launch_trace_stream(S, A, shadow != 0, c->tri_only, stats, env_int("DRT_TRACE_WAVES", 6), st);
  DRT_HIP(c, hipGetLastError());
  DRT_HIP(c, hipEventRecord(c->tev[1], st));
  if (!shadow) launch_trace_finish(S, q, n, dt, A.prim_out, dn, dobj, st);
  DRT_HIP(c, hipGetLastError());
  DRT_HIP(c, hipEventRecord(c->tev[2], st));
  c->trace_issued = true;
  c->trace_timed = true;
  c->trace_stats_valid = stats;
  return DRT_OK;
}

static int trace_common(drt_ctx* c, const float* rays, int32_t n, int shadow, float* t, float* nrm, int32_t* obj,
                        uint8_t* occ) {
  if (!c || n < 0 || (n > 0 && !rays)) return DRT_E_INVALID;
  if (n == 0) return DRT_OK;
  if (!c->has_scene) DRT_FAIL(c, DRT_E_STATE, "no scene uploaded");
  DRT_HIP(c, hipSetDevice(c->device));
  const size_t rb = sizeof(float) * 6 * (size_t)n;
  const size_t ob = shadow ? (size_t)n : (sizeof(float) * 4 + sizeof(int32_t)) * (size_t)n;
  DRT_HIP(c, c->d_rays.ensure(rb));
  DRT_HIP(c, c->d_out.ensure(ob));
  DRT_HIP(c, hipMemcpyAsync(c->d_rays.p, rays, rb, hipMemcpyHostToDevice, c->stream));
  float* dt = c->d_out.as<float>();
  float* dn = dt + n;
  int32_t* dobj = (int32_t*)(dn + 3 * (size_t)n);
  uint8_t* docc = c->d_out.as<uint8_t>();
  int rc = trace_device(c, c->d_rays.as<float>(), n, shadow, dt, dn, dobj, docc, c->stream);
  if (rc) return rc;
  if (shadow) {
    DRT_HIP(c, hipMemcpyAsync(occ, docc, (size_t)n, hipMemcpyDeviceToHost, c->stream));
  } else {
    DRT_HIP(c, hipMemcpyAsync(t, dt, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    DRT_HIP(c, hipMemcpyAsync(nrm, dn, sizeof(float) * 3 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    DRT_HIP(c, hipMemcpyAsync(obj, dobj, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  }
  DRT_HIP(c, hipStreamSynchronize(c->stream));
  return DRT_OK;
}

int drt_trace_device(drt_ctx* c, int shadow, const float* d_rays, int32_t n, float* d_t, float* d_normal,
                     int32_t* d_object, uint8_t* d_occluded, void* hip_stream) {
  if (!c || n < 0 || (n > 0 && !d_rays)) return DRT_E_INVALID;
  if (shadow ? !d_occluded : (!d_t || !d_normal || !d_object)) return DRT_E_INVALID;
  if (n == 0) return DRT_OK;
  return trace_device(c, d_rays, n, shadow, d_t, d_normal, d_object, d_occluded,
                      hip_stream ? (hipStream_t)hip_stream : c->stream);
}

int drt_set_trace_flags(drt_ctx* c, int flags) {
  if (!c) return DRT_E_INVALID;
  c->trace_flags = flags;
  return DRT_OK;
}

int drt_trace_stats(drt_ctx* c, drt_frame_stats* out) {
  if (!c || !out) return DRT_E_INVALID;
  drt_frame_stats r{};
  if (c->trace_timed) {
    DRT_HIP(c, hipSetDevice(c->device));
    DRT_HIP(c, hipEventSynchronize(c->tev[1]));
    float ms = 0;
    DRT_HIP(c, hipEventElapsedTime(&ms, c->tev[0], c->tev[1]));
    r.kernel_ms = ms;
    r.render_ms = ms;
    if (c->trace_stats_valid) {
      unsigned long long s[ST_COUNT];
      DRT_HIP(c, hipMemcpy(s, c->d_tstats.p, sizeof(s), hipMemcpyDeviceToHost));
      r.closest_rays = s[ST_CLOSEST]; r.shadow_rays = s[ST_SHADOW];
      r.closest_inner = s[ST_C_INNER]; r.closest_leaf = s[ST_C_LEAF];
      r.shadow_inner = s[ST_S_INNER]; r.shadow_leaf = s[ST_S_LEAF];
      r.closest_prims = s[ST_C_PRIMS]; r.shadow_prims = s[ST_S_PRIMS];
      r.wave_node_iters = s[ST_WAVE_NODE_ITERS];
      r.stack_pushes = s[ST_PUSH];
      r.stack_spills = s[ST_PUSH_SPILL];
      r.wave_leaf_iters = s[ST_WAVE_LEAF_ITERS];
      r.wide_shadow_rays = s[ST_W_RAYS];
      r.wide_inner = s[ST_W_INNER];
      r.wide_leaf = s[ST_W_LEAF];
      r.wide_prims = s[ST_W_PRIMS];
      r.wide_verify = s[ST_W_VERIFY];
    }
  }
  *out = r;
  return DRT_OK;
}

int drt_trace_closest(drt_ctx* c, const float* rays, int32_t n, float* t, float* nrm, int32_t* obj) {
  if (!t || !nrm || !obj) return DRT_E_INVALID;
  return trace_common(c, rays, n, 0, t, nrm, obj, nullptr);
}

int drt_trace_shadow(drt_ctx* c, const float* rays, int32_t n, uint8_t* occ) {
  if (!occ) return DRT_E_INVALID;
  return trace_common(c, rays, n, 1, nullptr, nullptr, nullptr, occ);
}

}  // extern "C"
