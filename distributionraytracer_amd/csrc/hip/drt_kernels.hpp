// drt_kernels.hpp — kernel argument blocks shared by drt_kernels.hip and drt_capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/drt.h"

namespace drt {

enum Accel : int { ACC_NONE = 0, ACC_GRID = 1, ACC_BVH = 2 };

enum FrameMode : int {
  MODE_AA = 0,            // one thread per (pixel, sample): main.cpp:618-671 without DoF/roughness
  MODE_SEQ = 1,           // one thread per pixel, samples in order with the keyed RNG stream
  MODE_WHITTED_QUAD = 2,  // one thread per (pixel, regular light sample): main.cpp:683-697
  MODE_WHITTED_POINT = 3,  // one thread per pixel: main.cpp:698-701
  MODE_PROG = 4,           // progressive zone A: one jittered sample per pixel, main.cpp:540-586
  // An in-order keyed-stream frame (MODE_SEQ) of a scene without refraction, in two passes:
  MODE_SKEL = 5,    // pass 1, one lane per pixel, samples in order: only the closest-hit chain of
                    // each sample (primary ray, mirror bounces) — which fixes every random draw's
                    // position — recording each sample's stream position and each bounce's hit
  MODE_REPLAY = 6,  // pass 2, one lane per (pixel, sample), any order: the whole rayTracing() of
                    // the sample from its recorded stream position, closest hits read back, shadow
                    // rays traced
  // An AA frame (MODE_AA) of a refraction-free BVH scene in two passes (round 4), so that the
  // shadow queries run in waves of shadow queries only, on the 4-ary shadow tree:
  MODE_CHAIN = 7,   // pass 1, one lane per (pixel, sample): the sample's closest-hit chain only,
                    // each bounce's hit recorded; pass 2 is MODE_REPLAY.  A Whitted frame (spp 0,
                    // round 5) in two passes: one lane per pixel, the chain its light samples share
  MODE_AREPLAY = 8,  // pass 2 of an AA / Whitted frame (round 5: its own instantiation; MODE_REPLAY
                    // stays the in-order frames'): no keyed-stream draw after the prologue reaches
                    // the frame, so no RNG, DoF or stream positions in its code
  // An AA / Whitted frame of a scene WITH a refracting material in two passes (round 5): a sample's
  // closest hits form a binary tree (refraction child first, then reflection, main.cpp:465-512):
  MODE_TCHAIN = 9,   // pass 1: the whole tree of closest-hit queries, no shadow rays, each hit recorded
                     // in the order rayTracing() makes the queries (<= 2^(max_depth+1) - 1 per sample)
  MODE_TREPLAY = 10,  // pass 2: the whole rayTracing() with refraction, the closest hits read back in
                      // that order, shadow queries on the shadow tree / the Grid
  // The Grid's wavefront replay (round 5, WfArgs): one Grid::Traverse(Ray&) shadow query per work item
  // from FrameArgs::q_rays (thr < 0: no query), its answer to q_occ
  MODE_QSTREAM = 11
};

enum StatSlot : int {
  ST_CLOSEST = 0, ST_SHADOW, ST_C_INNER, ST_C_LEAF, ST_S_INNER, ST_S_LEAF, ST_C_PRIMS, ST_S_PRIMS, ST_SAMPLES,
  // SIMD efficiency: wave-level iterations of the node loop / of the path loop (one count per
  // wave per iteration, by its lowest active lane)
  ST_WAVE_NODE_ITERS, ST_WAVE_PATH_ITERS, ST_LANE_PATH_ITERS,
  // stats builds of the persistent kernel: s_memtime cycles per wave in each loop section
  ST_CYC_REFILL, ST_CYC_NODE, ST_CYC_PROC,
  // traversal-stack pushes, and those that went past the LDS part of the stack
  ST_PUSH, ST_PUSH_SPILL,
  // node loop: wave iterations that ran the leaf block, and s_memtime cycles spent in it
  ST_WAVE_LEAF_ITERS, ST_CYC_LEAF,
  // shadow queries on the 4-ary shadow tree (drt_layout.hpp): queries, inner-node visits, leaf
  // visits, primitive tests and exact leaf-box checks of in-range hits (the ST_S_* slots then
  // count only the shadow queries that walked the reference's binary tree)
  ST_W_RAYS, ST_W_INNER, ST_W_LEAF, ST_W_PRIMS, ST_W_VERIFY, ST_W_GRIDFB,
  ST_COUNT
};

constexpr int kMaxFrames = 16;     // max_depth <= 15
constexpr int kMaxBvhDepth = 96;   // traversal stack entries (host rejects deeper trees)
// A shadow-tree lane keeps its stack in the LDS rows of both the descriptor and the t part (it has
// no entry distances) and spills past them: 2 * CAP + (kMaxBvhDepth - CAP) >= kMaxBvhDepth + 9
// entries at every occupancy the kernels use (CAP >= 9).  A 4-ary node pushes at most 3, so the
// host collapses a tree only when 3 * its depth fits.
constexpr int kWideMaxStack = kMaxBvhDepth + 8;
constexpr int kLdsStack = 16;      // traversal stack entries kept in LDS per thread
constexpr int kBlock = 256;        // path-kernel block size
#ifndef DRT_PBLOCK
#define DRT_PBLOCK 256
#endif
// Block size of the BVH persistent and streaming kernels.  Their LDS traversal stack is laid out
// [entry][thread] with one kRowBytes row per entry, and the stack pointer is the LDS byte address
// depth * kRowBytes + threadIdx.x * 4 (so depth = spa >> kRowShift).
constexpr int kPBlock = DRT_PBLOCK;
constexpr uint32_t kRowBytes = (uint32_t)kPBlock * 4u;
constexpr int kRowShift = kPBlock == 256 ? 10 : (kPBlock == 128 ? 9 : 8);
static_assert(kPBlock == 256 || kPBlock == 128 || kPBlock == 64, "persistent block: 64, 128 or 256 threads");
constexpr size_t kMacroBits = 131072;  // Grid macro-cell bitmap budget: 16 KB of LDS per block
constexpr size_t kPrimPadBytes = 64;  // zeroed tail of the primitive buffer (node_step's slot reads)
// persistent kernels: 32-bit work-item counters; bigger frames run the 64-bit path_kernel
constexpr uint64_t kPersistentMaxItems = 0xF0000000ull;
// two-pass in-order frames: the closest-hit record (8 B per sample and bounce) stays below this
constexpr uint64_t kTwoPassMaxBytes = 32ull << 30;

struct SceneArgs {
  // Camera (camera.h:32-61), precomputed on the host
  float eye[3], u[3], v[3], n[3];
  float w, h, plane_dist, focal_ratio, aperture;
  int res_x, res_y;
  const drt_light* lights;
  int n_lights;
  const drt_material* mats;
  int n_mats;
  const float4* prims;
  int n_prims;
  float bg[3];
  int has_sky;
  const uint8_t* sky[6];
  int sky_w[6], sky_h[6], sky_bpp[6];
  // BVH
  const float4* nodes;
  float root_box[6];
  uint32_t root_desc;
  // Grid
  int gdim[3];
  float gmin[3], gmax[3];
  // the Grid shadow tree's cell certificate (grid_certificate): cells per unit length per axis, n / width,
  // and the margin to a cell face, in cells
  float gscale[3], gmargin;
  const uint32_t* cell_start;
  const uint32_t* cell_objs;
  // macro-cell occupancy bitmap: bit (x>>shift) + mx*((y>>shift) + my*(z>>shift)) set if any
  // cell of that macro-cell holds an object
  const uint32_t* gmacro;
  const float4* cell_recs;  // per reference, in cell order: the primitive record, q2.w = its index
  // triangle scenes: per reference in cell order a 40-B (v0, e1, e2, scene index) record, two per
  // 80-B pair; cell i's records [tpos[i] & 0x7fffffff, (tpos[i+1] & 0x7fffffff) - (tpos[i+1] >> 31))
  const float4* cell_tris;
  const uint32_t* cell_tpos;
  const float4* gprims;     // (experiment DRT_GRID_INDEXED) each record once, Morton cell order, q2.w = index
  const uint32_t* cell_pos; // (experiment DRT_GRID_INDEXED) per reference: its record in gprims
  int gmacro_shift, gmacro_dim[3], gmacro_words;
  const uint2* big_leaves;
  // 4-ary shadow tree (drt_layout.hpp): null = every shadow query walks the reference's binary
  // tree in its visit order (DRT_FRAME_REFERENCE_ORDER, or a tree the host could not collapse)
  const float4* wnodes;
  const float4* wleaf;  // exact reference leaf box per primitive (BVH object order)
  uint32_t wroot;       // the root's wide record
};

// Wavefront replay of an AA / Whitted two-pass BVH frame without refraction (round 5): the closest hits
// are all known after MODE_CHAIN, so every shading decision except occlusion is a function of them.
// wf_gen (one thread per sample slot) walks each sample's recorded chain and writes every shadow query
// of every level ([level][visited light pair][slot]: 32-B trace_stream records, thr < 0 = no query) with its
// NdotL / NdotH, and one 16-B record per level; trace_stream answers the shadow queries; wf_combine
// walks the levels back, adding the unshadowed light terms in the reference's order, and writes the
// sample.
struct WfArgs {
  float4* rays;    // per query slot: (o, thr); thr < 0: no query in this slot
  float4* rays_b;  // per query slot: (d, 0) — a second array, so that each store / load is one contiguous run
  float2* nl;     // per query slot: (NdotL, NdotH)
  uint8_t* occ;   // per query slot: 1 = occluded (trace_stream)
  float4* lvl;    // per (level, slot): (background colour of a miss, material | flags << 24)
  uint32_t n_slots;  // sample slots of this chunk of the frame (the buffers' slot dimension)
  uint32_t slot0;    // the chunk's first sample slot
  uint32_t band;     // sample slots per band (wf_q); bands * band >= n_slots
  int bands;
  int levels;        // max_depth + 1
  int inorder;       // an in-order (DoF / glossy) frame: keyed-stream draws from FrameArgs::skel_rk (MODE_REPLAY)
  int grid;       // Grid scene: queries as Grid::Traverse(Ray&) takes them (unit L, range |L|)
  int pairs;      // query slots per level: the (light, k) pairs the light loop visits (a point light: k = 0 only)
  // compact (round 6, BVH): each 64-slot group's queries of a (level, pair) packed to the group's first
  // slots, in lane order, with the query's own slot index in rays_b.w, and per (band, level, group) their
  // count in cnt[(band * levels + level) * (band_slots / 64) + group] (band a multiple of 256), so that
  // trace_stream hands out queries without reading empty slots (TraceArgs::sparse 2).  0: thr = -1 markers.
  int compact;
  uint8_t* cnt;
};

struct FrameArgs {
  uint32_t seed;
  int max_depth;
  float roughness;
  int mode;
  int dof;
  uint32_t spp;
  int n_sqrt;         // (int)sqrt(spp)        (main.cpp:619)
  int nsub;           // work items per pixel
  uint32_t grid_res;  // light 0 gridRes       (main.cpp:684)
  int grid_size;      // (int)sqrt(gridRes)    (main.cpp:689)
  // light_spp extension: shadow samples per quad light per hit
  int light_spp;      // m >= 1 (1 = the reference)
  int light_grid;     // floor(sqrt(m))
  float light_inv;    // 1.0f / m
  int tile, tiles_x, shard, n_shards, n_my_tiles;
  uint64_t n_items;
  float4* samples;
  unsigned long long* stats;
  unsigned int* work_counter;  // persistent kernel: next unclaimed work item (zeroed per frame)
  int refill_min;              // persistent kernel: refill a wave once this many lanes are idle
  int process_min;             // persistent kernel: shade once this many lanes have a result
  int waves;                   // persistent kernel: register budget (waves per SIMD: BVH 6 or 7, Grid 5 or 6)
  int grid_walk;               // Grid persistent kernel: empty-macro-cell steps per call
  int grid_pairs;              // Grid persistent kernel: object-pair round trips per call
  uint32_t part_items;         // persistent kernel: items per XCD work partition (ceil(n_items / 8))
  const uint8_t* perm;         // persistent kernel, AA / in-order frames: shuffle_kernel's slot -> sample map
  // Persistent kernel, MODE_SEQ frame tail: once every pixel is claimed, waves past the number
  // the unfinished pixels need hand each pixel's remaining samples over at a sample boundary
  // (item, next sample, keyed-stream position packed in 64 bits; 0 = slot not yet written) and
  // exit, so that the next frame's blocks take their CUs.  Null: off.
  unsigned long long* seq_cont;
  uint32_t seq_cap;            // continuation slots (one per resident lane bounds the pushes)
  int seq_slack;               // waves kept = ceil(unfinished pixels * seq_slack / 100 / 64)
  int seq_pop_min;             // a kept wave takes handed-over pixels once this many lanes are idle
  uint32_t seq_backlog;        // a lane keeps its pixel while this many wait in the slots (0: no bound)
  // MODE_SKEL / MODE_REPLAY: per sample slot (pixel * nsub + sample) its keyed-stream position at
  // the sample's start, and per slot and depth (max_depth + 1 entries) the closest hit of that
  // bounce: (t bits, primitive record), primitive 0xFFFFFFFF = miss
  uint32_t* skel_rk;
  uint2* skel_hits;
  // MODE_REPLAY of an AA frame (pass 2 after MODE_CHAIN): no keyed-stream positions (skel_rk null);
  // reflections use MODE_AA's direction (the draws after the prologue never reach the frame, Q16)
  int aa_chain;
  // Two-pass Whitted frames (round 5): the grid_res light samples of a pixel share its pixel-centre
  // primary ray and every mirror bounce (main.cpp:683-696), so MODE_CHAIN traces one chain per pixel
  // and MODE_REPLAY's sample slot i reads record i / chain_div (chain_div = grid_res; 1 for AA
  // frames).  MODE_CHAIN counts chain_div samples per item.
  int chain_div;
  // replay passes: frame heads, max_depth + 1 float4 per resident lane (blockIdx * blockDim +
  // threadIdx), each lane's run contiguous
  float4* heads;
  // MODE_TCHAIN / MODE_TREPLAY: records per sample (2^(max_depth+1) - 1); a lane's rk holds its next
  // record index
  int tree_recs;
  // MODE_QSTREAM: 2 float4 per query ((o, range), (d, 0)), 1 byte per answer (1 = shadowed)
  const float4* q_rays;    // per query: (o, range); thr < 0: no query
  const float4* q_rays_b;  // per query: (d, 0)
  uint8_t* q_occ;
  // stats launches (STATS build of path_persistent), when set: per resident wave of this launch its
  // (start, end) s_memrealtime stamps (100 MHz), indexed by global thread id / 64 (drt_frame_wave_times)
  unsigned long long* wave_times;
};

// Control words of the MODE_SEQ tail in the per-frame work-counter block (1 KiB, zeroed per
// frame, after the 8 partition counters): pushes and pops of the continuation slots as one
// 64-bit pair, and the pixels finished, on a 128-B line of its own (every pixel adds to it).
constexpr uint32_t kSeqPush = 128, kSeqPop = 129, kSeqDone = 192;


// Streaming BVH traversal (trace_stream): one query per lane, refilled from a query array.
struct TraceArgs {
  const float4* rays;          // 2 per query: (o.xyz, range threshold), (d.xyz, 0); shadow d is unit
  const float4* rays_b;        // query i: (o, range) at rays[i * stride], (d, 0) at rays_b[i * stride]
  int stride;                  // 2: interleaved records (rays_b = rays + 1); 1: two arrays
  uint32_t n;
  unsigned int* counter;       // next unclaimed query (zeroed per launch)
  float* t_out;                // closest: best t (FLT_MAX on a miss)
  uint32_t* prim_out;          // closest: primitive record index (0xFFFFFFFF on a miss)
  uint8_t* occ_out;            // shadow: 1 if occluded
  unsigned long long* stats;   // ST_* counters (stats launches only)
  int refill_min;
  int sparse;                  // 1: shadow queries with thr < 0 are empty slots: skipped, occ_out not written;
                               // 2: WfArgs::compact queries — per 256-query chunk four 64-slot group counts
                               // (cnt), the answer written to the query's own slot (rays_b.w)
  const uint8_t* cnt;          // sparse 2: WfArgs::cnt
  int levels, pairs;           // sparse 2: the query array's shape [band][level][pair][band_slots]
  uint32_t band;
  // work partitions: `parts` ranges of part_len queries, one claim counter each (64 B apart); a wave
  // starts on the range of its XCD and moves on when that one is claimed (parts 1: one counter)
  int parts;
  uint32_t part_len;
  // the Grid scene's shadow tree (trace_stream GV): queries it leaves to the Grid walk, by their position
  // in the query array, and their count (grid_fallback)
  float4* fb_rays;  // two per query: (o, range), (d, its slot)
  unsigned int* fb_count;
};

struct ReduceArgs {
  const float4* samples;
  int nsub;
  float scale;  // (float)(1.0/spp) for AA (main.cpp:666), 1.0f/gridRes (main.cpp:696), 1 otherwise
  int tile, tiles_x, shard, n_shards, n_my_tiles;
  int res_x, res_y;
  int full_frame;  // write the (x, y) frame, else the shard-compact buffer
  int prog_frame;  // > 0: progressive FrameCount, out = lerp(out, sample, 1/n) (main.cpp:574-586)
  float* out;
};

}  // namespace drt
