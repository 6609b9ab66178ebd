/*
 * drt.h — C ABI of the MI355X distribution ray tracer (libdrt.so).
 *
 * This is the drop-in boundary for the reference's hot path (rita-mota/DistributionRayTracer,
 * paths relative to DistributionRayTracer/).  The reference has no FFI: its hot path is the
 * C++ class API called from main.cpp.  Each entry point below names the reference interface
 * it replaces:
 *
 *   drt_upload_scene   <- Scene / Camera / Light / Material / Object state read by
 *                         rayTracing() (scene.h:24-231, camera.h:12-101)
 *   drt_set_camera     <- Camera::SetEye (camera.h:63-72), called by renderScene() every frame
 *                         in draw mode (main.cpp:530-533): the camera alone, scene resident
 *   drt_upload_bvh     <- BVH::Build result (rayAccelerator.h:87-94, bvh.cpp:27-227)
 *   drt_upload_grid    <- Grid::Build result (rayAccelerator.h:12-37, grid.cpp:30-97)
 *   drt_trace_closest  <- BVH::Traverse(Ray&, Object**, HitRecord&)  (bvh.cpp:231-314)
 *                         Grid::Traverse(Ray&, Object**, HitRecord&) (grid.cpp:247-306)
 *                         the NONE linear scan                       (main.cpp:310-336)
 *   drt_trace_shadow   <- BVH::Traverse(Ray&) (bvh.cpp:316-391), Grid::Traverse(Ray&)
 *                         (grid.cpp:309-358)
 *   drt_render         <- renderScene() zone B (main.cpp:525-738) incl. rayTracing()
 *                         (main.cpp:294-521): jittered AA, light-sample shuffle, thin-lens
 *                         DoF, Whitted area-light grid, Phong + shadows, refraction/reflection
 *
 * Conventions: plain C types only; caller owns all host memory; the context owns all device
 * memory.  Every function returns 0 (DRT_OK) or a negative drt_status and never exits the
 * process; drt_last_error() describes the last failure.  One host thread per context.
 * Calls are blocking except drt_render_device, which is asynchronous on the given stream.
 *
 * Frame buffer layout (main.cpp:705-714): float RGB, index 3*(x + RES_X*y), row y = 0 is the
 * BOTTOM row of the image (OpenGL / DevIL lower-left origin).
 *
 * RNG: the reference uses CRT rand() seeded with time()^2; parity is defined on the keyed
 * stream of SURVEY.md §8c — the k-th rand() call inside pixel P = y*RES_X + x returns
 * mix32(seed ^ mix32(P*0x9E3779B9 ^ mix32(k))) >> 17, RAND_MAX = 0x7FFF.
 */
#ifndef DRT_H
#define DRT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRT_ABI_VERSION 3
#define DRT_FRAME_SLOTS 4 /* drt_frame_params.slot: 0 .. DRT_FRAME_SLOTS-1 */

typedef enum {
  DRT_OK = 0,
  DRT_E_INVALID = -1,     /* bad argument / malformed scene                         */
  DRT_E_HIP = -2,         /* HIP runtime error                                        */
  DRT_E_NODEVICE = -3,    /* no usable gfx950 device                                  */
  DRT_E_OOM = -4,         /* device allocation failed                                 */
  DRT_E_STATE = -5,       /* call order (e.g. render before upload)                   */
  DRT_E_UNSUPPORTED = -6  /* feature outside this build                               */
} drt_status;

enum { DRT_ACCEL_NONE = 0, DRT_ACCEL_GRID = 1, DRT_ACCEL_BVH = 2 };               /* scene.h:22 */
enum { DRT_PRIM_TRIANGLE = 0, DRT_PRIM_SPHERE = 1, DRT_PRIM_PLANE = 2, DRT_PRIM_BOX = 3 };
enum { DRT_LIGHT_POINT = 0, DRT_LIGHT_QUAD = 1 };                                  /* scene.h:16 */

typedef struct drt_ctx drt_ctx;

typedef struct {
  int32_t device;       /* HIP device ordinal                                        */
  int32_t reserved[7];
} drt_options;

/* Camera frame exactly as the host Camera constructor computes it (camera.h:32-61). */
typedef struct {
  float eye[3], u[3], v[3], n[3];
  float w, h, plane_dist, focal_ratio, aperture;
  int32_t res_x, res_y;
} drt_camera;

/* Light (scene.h:68-107): quad lights span pos + e1*s + e2*t. */
typedef struct {
  int32_t type;
  float pos[3];
  float e1[3], e2[3];
  uint32_t grid_res;
} drt_light;

/* Material (scene.h:34-66); refl is m_Refl (= Ks for P3F materials, scene.h:42). */
typedef struct {
  float diff[3];
  float kd;
  float spec[3];
  float ks, shine, refl, trans, ior;
} drt_material;

/* Object (scene.h:109-180).  triangle: a,b,c = P0,P1,P2; sphere: a = centre, r = radius;
 * plane: a = PN, r = D; box: a = min, b = max.  material < 0 = none (reference UB). */
typedef struct {
  int32_t type;
  int32_t material;
  float a[3], b[3], c[3];
  float r;
} drt_prim;

typedef struct {
  drt_camera camera;
  const drt_material* materials;
  int32_t n_materials;
  const drt_prim* prims;
  int32_t n_prims;
  const drt_light* lights;
  int32_t n_lights;
  float background[3];          /* bclr (scene.cpp:680)                                  */
  int32_t accel;                /* DRT_ACCEL_*                                           */
  uint32_t spp;                 /* 0 = Whitted (main.cpp:1005-1010)                      */
  int32_t has_skybox;           /* env (scene.cpp:687)                                   */
  const uint8_t* skybox[6];     /* faces RIGHT..BACK, rows bottom-up (scene.cpp:345)     */
  int32_t sky_w[6], sky_h[6], sky_bpp[6];
} drt_scene_desc;

/* One BVHNode (rayAccelerator.h:50-67) in the reference's node numbering: inner nodes keep
 * their two children at index and index+1 (bvh.cpp:206-222); leaves cover
 * object_order[index .. index+n_objs). */
typedef struct {
  float bmin[3], bmax[3];
  uint32_t leaf;
  uint32_t index;
  uint32_t n_objs;
} drt_bvh_node;

/* drt_frame_params.flags: DRT_FRAME_STATS counts rays / node visits / primitive tests;
 * DRT_FRAME_SHARD_LAYOUT makes drt_render_device write the shard-compact tile buffer of
 * drt_shard_layout() even for n_shards == 1 (a one-device drt_group);
 * DRT_FRAME_REFERENCE_ORDER (also a drt_set_trace_flags flag) walks every shadow query
 * (BVH::Traverse(Ray&), bvh.cpp:316-391) on the reference's binary tree in its visit order, so
 * that the shadow node / leaf / primitive counts equal the reference's.  Without it, shadow
 * queries of finite rays walk a 4-ary tree collapsed from the same BVH: the occlusion answer,
 * hence every frame, is identical (an any-hit query does not depend on the visit order), and
 * drt_frame_stats counts that work in its wide_* fields. */
enum { DRT_FRAME_STATS = 1, DRT_FRAME_SHARD_LAYOUT = 2, DRT_FRAME_REFERENCE_ORDER = 4 };

typedef struct {
  uint32_t seed;       /* keyed-RNG seed                                                */
  int32_t max_depth;   /* MAX_DEPTH (main.cpp:34) = 4                                   */
  float roughness;     /* roughness_param (main.cpp:507) = 0                            */
  int32_t shard;       /* this rank's shard: the tiles at dealing positions p with
                          p % n_shards == shard (sharding.py: row ty rotated by ty tiles)  */
  int32_t n_shards;    /* 1 = whole frame                                               */
  int32_t tile;        /* tile edge in pixels (0 -> 16)                                 */
  int32_t flags;       /* DRT_FRAME_STATS: count rays / node visits / prim tests        */
  int32_t light_spp;   /* extension: shadow samples per quad light per
                          hit, 0 or 1 = the reference (main.cpp:391: one sample)          */
  int32_t progressive_frame; /* 0: renderScene zone B.  n >= 1: zone A (main.cpp:536-599) with
                          FrameCount n — one jittered sample per pixel, written (n = 1) or
                          lerped into the output with weight 1/n (n > 1: the output buffer is
                          read, so pass the previous frame back); n >= MAX_SAMPLES (10000)
                          leaves the output untouched (main.cpp:537)                     */
  int32_t slot;        /* frame scratch slot, 0 .. DRT_FRAME_SLOTS-1: frames on different
                          slots of one context may run concurrently on different streams
                          (pipelining); a frame on a slot whose previous frame ran on another
                          stream waits for that frame on the device; other values are
                          DRT_E_INVALID                                                    */
  int32_t reserved[2];
} drt_frame_params;

typedef struct {
  uint64_t closest_rays, shadow_rays;     /* Traverse() calls                            */
  uint64_t closest_inner, closest_leaf;   /* node-loop iterations (bvh.cpp:245)           */
  uint64_t shadow_inner, shadow_leaf;     /* (bvh.cpp:331)                                */
  uint64_t closest_prims, shadow_prims;   /* Object::hit calls                           */
  uint64_t samples;                       /* rayTracing(depth = 1) calls                 */
  double render_ms;                        /* device time of the last drt_render*        */
  double kernel_ms;                        /* device time of the path-tracing kernel     */
  uint64_t wave_node_iters;                /* node-loop iterations counted once per wave */
  uint64_t wave_path_iters, lane_path_iters; /* path-loop iterations per wave / per lane  */
  uint64_t cycles_refill, cycles_node, cycles_shade; /* persistent kernel: s_memtime cycles */
  uint64_t stack_pushes, stack_spills;   /* traversal-stack pushes / those beyond the LDS part */
  uint64_t wave_leaf_iters, cycles_leaf; /* node-loop iterations that ran the leaf block / its cycles */
  /* in-order keyed-stream frames (DoF / glossy): pixels handed between waves at the frame's tail
   * and taken up again (0 when the hand-over was off for the frame); filled for every frame */
  uint64_t seq_pushed, seq_popped;
  int32_t seq_handover;                   /* the hand-over was on for the frame                  */
  int32_t reserved;
  /* shadow queries that walked the 4-ary shadow tree (not DRT_FRAME_REFERENCE_ORDER): queries,
   * inner-node visits, leaf visits, primitive tests, exact leaf-box checks of in-range hits.
   * shadow_inner / shadow_leaf / shadow_prims then count only the queries (non-finite rays)
   * that walked the reference's binary tree. */
  uint64_t wide_shadow_rays, wide_inner, wide_leaf, wide_prims, wide_verify;
  /* a Grid scene's shadow tree (drt_upload_grid_shadow_bvh): its queries left to the Grid walk */
  uint64_t wide_grid_walks;
} drt_frame_stats;

int drt_create(drt_ctx** out, const drt_options* opt);
void drt_destroy(drt_ctx* ctx);
const char* drt_last_error(const drt_ctx* ctx);
int drt_abi_version(void);

int drt_upload_scene(drt_ctx* ctx, const drt_scene_desc* scene);
/* Replace the camera of the resident scene (Camera::SetEye, camera.h:63-72; the interactive
 * renderer calls it every frame, main.cpp:530-533).  Primitives, lights, materials, skybox and
 * the BVH / grid stay resident: nothing is re-packed or copied.  The next frame issued uses the
 * new camera; frames already issued keep theirs.  DRT_E_STATE without a scene. */
int drt_set_camera(drt_ctx* ctx, const drt_camera* camera);
int drt_upload_bvh(drt_ctx* ctx, const drt_bvh_node* nodes, uint32_t n_nodes, const uint32_t* object_order,
                   uint32_t n_objects);
int drt_upload_grid(drt_ctx* ctx, const int32_t dims[3], const float bmin[3], const float bmax[3],
                    const int64_t* cell_start /* nx*ny*nz+1 */, const int32_t* cell_objs, int64_t n_refs);
/* Optional, after drt_upload_grid of a triangle scene (round 6): a BVH of the same objects (the
 * BVH::Build result, as drt_upload_bvh takes it).  The Grid frame's wavefront shadow queries then walk a
 * 4-ary tree collapsed from it with widened boxes, and a hit counts only with a Grid cell certificate
 * (the ray's point at the hit lies well inside a cell the object is listed in, so Grid::Traverse(Ray&),
 * grid.cpp:309-358, finds it too); queries without one are walked on the Grid.  The answers are
 * Grid::Traverse(Ray&)'s.  Any drt_upload_scene / drt_upload_grid / drt_upload_bvh drops it.
 * DRT_GRID_SHADOW_TREE=0 keeps the Grid walk for every query. */
int drt_upload_grid_shadow_bvh(drt_ctx* ctx, const drt_bvh_node* nodes, uint32_t n_nodes,
                               const uint32_t* object_order, uint32_t n_objects);

/* How a frame would run (no device work): work items (a (pixel, sample) pair, or a pixel whose
 * samples run in order), float4 sample slots, the frame mode (0 AA, 1 in-order keyed stream,
 * 2 Whitted quad grid, 3 Whitted point, 4 progressive) and whether the persistent kernel takes it
 * (frames of >= 0xF0000000 work items run the 64-bit one-item-per-thread kernel instead). */
typedef struct {
  uint64_t work_items;
  uint64_t sample_slots;
  int32_t mode;
  int32_t persistent;
  int32_t tiles_in_shard;
  int32_t passes;      /* 2: a pass over the samples' closest hits and a pass over every sample with
                          its closest hits read back; 1 otherwise.  Two passes for:
                          - in-order frames (DoF / glossy) of scenes without refraction (a pixel's
                            samples in order);
                          - AA frames of BVH (shadow tree uploaded) / Grid scenes of >= 1024 objects
                            whose whole frame has >= 2^23 samples or whose scene has >= 2^19 objects,
                            and at any size when the scene has non-triangle primitives and no
                            refracting material;
                          - Whitted frames of such scenes: quad light 0 at any size (one closest-hit
                            chain per pixel shared by its gridRes light samples); point light by the
                            AA size rule, and at any size on a Grid scene of mixed primitives without
                            a refracting material.
                          With a refracting material the AA / Whitted passes record each sample's
                          whole closest-hit tree (<= 2^(max_depth+1) - 1 hits) if it fits 32 GB.  The
                          plan depends on the params and the uploaded scene only, and drt_render
                          follows it.  Both plans render the same frame; the stats differ only in
                          where shadow work is counted (shadow_* on the reference tree, wide_* on
                          the shadow tree) and, for quad-light Whitted frames, in closest_* (gridRes
                          times fewer traversals). */
  int32_t wavefront;   /* 1: pass 2 of this two-pass frame runs as a wavefront — every shadow query of
                          the frame generated from the recorded closest hits, answered by a streaming
                          kernel (BVH: trace_stream on the shadow tree; Grid: its stepper's query
                          stream), then combined per sample with the frame's reduce folded in.  Every
                          two-pass frame without refraction: AA, Whitted and in-order (DoF / glossy)
                          frames, BVH and Grid (< 2^32 query slots; the query buffers in chunks of at
                          most DRT_WAVEFRONT_CHUNK_BYTES, default 24 GB, per frame slot).
                          DRT_WAVEFRONT=0 (DRT_WAVEFRONT_GRID=0, DRT_WAVEFRONT_INORDER=0 per kind):
                          the persistent replay.  A frame whose query buffers cannot be allocated runs
                          the persistent replay, which renders the same frame. */
  int32_t reserved[3];
} drt_frame_plan;
int drt_plan_frame(const drt_ctx* ctx, const drt_frame_params* params, drt_frame_plan* out);

/* RES_X, RES_Y of the uploaded scene's camera (DRT_E_STATE without a scene). */
int drt_frame_resolution(const drt_ctx* ctx, int32_t res_xy[2]);

/* Whole frame into host memory (RES_Y*RES_X*3 floats). */
int drt_render(drt_ctx* ctx, const drt_frame_params* params, float* rgb_out);

/* Tile-sharded frame into DEVICE memory, asynchronous on `hip_stream` (a hipStream_t, NULL =
 * the context's stream).  With n_shards == 1 the output is the full frame; otherwise it is
 * the shard-compact tile buffer of drt_shard_layout(). */
int drt_shard_layout(const drt_ctx* ctx, const drt_frame_params* params, int64_t* tiles_in_shard,
                     int64_t* floats_per_shard);
int drt_render_device(drt_ctx* ctx, const drt_frame_params* params, float* d_out, void* hip_stream);
/* Reassemble n_shards shard-compact buffers (laid end to end, floats_per_shard apart) into a
 * full device frame. */
int drt_unshard_device(drt_ctx* ctx, const drt_frame_params* params, const float* d_shards, float* d_frame,
                       void* hip_stream);

/* Batched ray queries against the uploaded scene (rays: n x {ox,oy,oz,dx,dy,dz}).
 * closest: t (FLT_MAX on miss), the HitRecord normal, object index (-1 on miss).
 * shadow: 1 if occluded, with the accelerator's own range rule. */
int drt_trace_closest(drt_ctx* ctx, const float* rays, int32_t n, float* t, float* normal, int32_t* object);
int drt_trace_shadow(drt_ctx* ctx, const float* rays, int32_t n, uint8_t* occluded);

/* The same queries on DEVICE buffers, asynchronous on `hip_stream` (NULL = the context's
 * stream): d_rays n x 6 floats; closest fills d_t / d_normal / d_object, shadow d_occluded.
 * BVH scenes run the streaming traversal kernel (one query per lane, lanes refilled as they
 * finish).  Replaces the same BVH/Grid Traverse calls as drt_trace_closest / drt_trace_shadow.
 * Batched queries of one context are serialised: a query issued on another stream waits (on
 * the device) for the previous one, whose scratch records and claim counter it reuses. */
int drt_trace_device(drt_ctx* ctx, int shadow, const float* d_rays, int32_t n, float* d_t, float* d_normal,
                     int32_t* d_object, uint8_t* d_occluded, void* hip_stream);
/* flags for later batched queries: DRT_FRAME_STATS counts their traversal work */
int drt_set_trace_flags(drt_ctx* ctx, int flags);
/* Device time of the streaming traversal kernel of the most recent BVH batched query
 * (kernel_ms) and, with DRT_FRAME_STATS set, its ray / node / leaf / primitive counters;
 * zeroes for Grid / NONE queries.  Waits for that query. */
int drt_trace_stats(drt_ctx* ctx, drt_frame_stats* out);

/* Counters (frames rendered with DRT_FRAME_STATS) and device times of the most recent frame;
 * waits for that frame. */
int drt_get_stats(drt_ctx* ctx, drt_frame_stats* out);

/* Device durations of the most recent min(max_frames, 512) frames, oldest first: the
 * path-tracing kernel (path_ms) and kernel + reduce (total_ms), from HIP events recorded on the
 * stream each frame ran on.  Waits for those frames.  Returns the count written (>= 0). */
int drt_frame_times(drt_ctx* ctx, int max_frames, double* path_ms, double* total_ms);
/* The same frames as absolute spans on one device clock, in ms from the path-kernel start of the
 * oldest frame returned: path-kernel start / end and frame end.  Frames on different streams
 * overlap; the union of their path-kernel spans is the device time the path kernel held. */
int drt_frame_spans(drt_ctx* ctx, int max_frames, double* path_start, double* path_end, double* frame_end);

/* Diagnostics of the last stats frame (DRT_FRAME_STATS) rendered by the persistent kernel: per resident
 * wave of its pass-1 (pass = 0) or pass-2 (pass = 1, the persistent replay or the Grid's query stream)
 * launch, the (start, end) s_memrealtime stamps (100 MHz) in start_end[2 * w], [2 * w + 1]; 0 = no such
 * wave.  Returns the number of wave slots written (<= max_waves).  No reference counterpart: it measures
 * the tail of a launch. */
int drt_frame_wave_times(drt_ctx* ctx, int pass, uint64_t* start_end, int64_t max_waves);

/* Device time of each launch of the last wavefront frame's pass 2 (the frame issued last whose plan
 * has `wavefront`): out_ms = {wf_gen, shadow-query stream (trace_stream / the Grid's MODE_QSTREAM),
 * wf_combine}, summed over its chunks (HIP events between the launches on the frame's stream; the first
 * 64 chunks).  Waits for that frame.  Returns the chunks counted; DRT_E_STATE before any wavefront
 * frame.  Read it before the next frame is issued. */
int drt_frame_stage_times(drt_ctx* ctx, double out_ms[3]);
/* The same frames' passes: a two-pass frame (drt_frame_plan.passes == 2) is the closest-chain pass
 * then the replay pass, timed from the path-kernel start to the end of the first launch and from
 * there to the path-kernel end (HIP events on the frame's stream; pass1 + pass2 = path_ms of
 * drt_frame_times).  A one-pass frame reports its path kernel as pass 1 and ~0 for pass 2 (two
 * events recorded back to back: a few microseconds).  For a
 * frame rendered alone these are the launches' device times; with frames in flight a pass's span
 * also holds its waits for CU room.  Waits for those frames.  Returns the count written (>= 0). */
int drt_frame_pass_times(drt_ctx* ctx, int max_frames, double* pass1_ms, double* pass2_ms);

/* ---- several GPUs behind one handle (main.cpp:603 is the loop being split) ----
 * One drt_ctx per device, one HIP stream per device and an RCCL clique over them
 * (ncclCommInitAll, librccl loaded at run time).  A frame: every device renders its interleaved
 * 16x16 tiles (shard r of n, the drt_frame_params.shard dealing) into a shard buffer, one
 * ncclAllGather moves the shards over xGMI, device 0 reassembles the frame.  Upload the scene
 * to every device's context (drt_group_ctx + drt_upload_*, or drt_group_scene_upload in
 * drt_host.h).  Progressive frames need a one-device group. */
typedef struct drt_group drt_group;
/* devices: n_devices distinct ordinals, or NULL for 0 .. n_devices-1 */
int drt_group_create(drt_group** out, int n_devices, const int32_t* devices);
void drt_group_destroy(drt_group* g);
const char* drt_group_last_error(const drt_group* g);
int drt_group_size(const drt_group* g);
drt_ctx* drt_group_ctx(drt_group* g, int rank);
/* Whole frame into host memory (RES_Y*RES_X*3 floats, row 0 = bottom); blocking.  params:
 * n_shards 0 or 1 (the group deals the tiles). */
int drt_group_render(drt_group* g, const drt_frame_params* params, float* rgb_out);
/* Whole frame into DEVICE memory on device 0 (d_frame: RES_Y*RES_X*3 floats), asynchronous:
 * device 0's work on `stream0` (NULL = the group's), the other devices' on the group's streams.
 * Shard and gather buffers belong to params->slot: frames on different slots do not share them,
 * and a frame on a slot whose last frame ran on another stream0 waits for that frame's reassembly
 * (on the device). */
int drt_group_render_device(drt_group* g, const drt_frame_params* params, float* d_frame, void* stream0);
/* drt_set_camera on every device of the group. */
int drt_group_set_camera(drt_group* g, const drt_camera* camera);
/* Wait for every device's stream. */
int drt_group_synchronize(drt_group* g);

#ifdef __cplusplus
}
#endif
#endif
