// drt_kernels.hip — gfx950 kernels of the distribution ray tracer hot path.
//
//  * path_kernel<ACCEL, TRI_ONLY, STATS>: renderScene zone B (main.cpp:603-721) + the whole
//    rayTracing() recursion (main.cpp:294-521) for one work item (a pixel sample, a Whitted
//    light sample, or a whole pixel in keyed-sequential mode).  The recursion is an explicit
//    DFS over frames so per-level clamping (main.cpp:489, 512, 520) is kept exactly; every
//    closest-hit AND every shadow query of the path goes through ONE traversal call site, so
//    lanes of a wave doing different kinds of queries stay converged in the node loop.
//  * reduce_kernel: ordered per-pixel sum (Color +=, main.cpp:664) and scale (main.cpp:666).
//  * trace_kernel: batched BVH/Grid/NONE closest and shadow queries (the Traverse() API).
//  * unshard_kernel: tile-compact shard buffers -> full frame.
#include <algorithm>
#include <cstdlib>

#include "drt_device.hpp"
#include "drt_kernels.hpp"

namespace drt {

struct Counters {
  uint32_t v[ST_COUNT];
};

// ------------------------------------------------------------------------------------------
// BVH traversal (bvh.cpp:231-314 closest, bvh.cpp:316-391 shadow), one loop for both.
// closest: ties -> right child first, pops skip entries with t >= best;  shadow: ties -> left
// first, any hit with t <= range (double len + EPSILON, pre-rounded to a float threshold)
// ends the query, pops are unconditional.
// ------------------------------------------------------------------------------------------
// Traversal stack: the top kLdsStack entries of each thread live in LDS (lane-interleaved:
// entry k of thread t at [k][t], so a wave's pushes/pops hit 64 consecutive banks); deeper
// entries spill to a private (scratch) array.  The 1M-triangle SAH tree is 25 levels deep and
// its stacks rarely exceed ~12 live entries, so the spill path is cold.
// LDS-typed pointers: with plain (generic) pointers the compiler merges the LDS and the scratch
// arms of a pop into one flat_load, which waits on both memory paths.
typedef __attribute__((address_space(3))) uint8_t LdsByte;
typedef __attribute__((address_space(3))) uint32_t LdsU32;
typedef __attribute__((address_space(3))) float LdsF32;

struct TravStack {
  LdsU32* desc;  // stride kBlock
  LdsF32* t;     // stride kBlock
};

__device__ __forceinline__ bool wave_leader() {
  return (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__ballot(1));
}

template <bool TRI_ONLY, bool STATS>
__device__ __forceinline__ bool bvh_traverse(const SceneArgs& S, const RayP& r, bool shadow, float shadow_thr,
                                             float& best_t, uint32_t& best_prim, Counters& C, TravStack ls) {
  float tmp;
  if (!box_hit(S.root_box[0], S.root_box[1], S.root_box[2], S.root_box[3], S.root_box[4], S.root_box[5], r, tmp))
    return false;
  uint32_t ov_desc[kMaxBvhDepth - kLdsStack];
  float ov_t[kMaxBvhDepth - kLdsStack];
  int sp = 0;
  uint32_t cur = S.root_desc;
  best_t = 3.402823466e+38f;  // HitRecord t = FLT_MAX
  bool hit = false;
  const float4* __restrict__ nodes = S.nodes;
  while (true) {
    if (STATS && wave_leader()) C.v[ST_WAVE_NODE_ITERS]++;
    if (!desc_is_leaf(cur)) {
      if (STATS) C.v[shadow ? ST_S_INNER : ST_C_INNER]++;
      const float4* nd = nodes + 4 * (size_t)cur;
      const float4 a = nd[0], b = nd[1], c = nd[2];
      const uint4 d = *reinterpret_cast<const uint4*>(nd + 3);
      float tL, tR;
      bool hL = box_hit(a.x, a.y, a.z, a.w, b.x, b.y, r, tL);
      bool hR = box_hit(b.z, b.w, c.x, c.y, c.z, c.w, r, tR);
      if (box_inside(a.x, a.y, a.z, a.w, b.x, b.y, r.o)) tL = 0.0f;
      if (box_inside(b.z, b.w, c.x, c.y, c.z, c.w, r.o)) tR = 0.0f;
      if (hL && hR) {
        const bool left_first = shadow ? (tL <= tR) : (tL < tR);
        cur = left_first ? d.x : d.y;
        const uint32_t pd = left_first ? d.y : d.x;
        const float pt = left_first ? tR : tL;
        if (sp < kLdsStack) {
          ls.desc[sp * kBlock] = pd;
          ls.t[sp * kBlock] = pt;
        } else {
          ov_desc[sp - kLdsStack] = pd;
          ov_t[sp - kLdsStack] = pt;
        }
        sp++;
        continue;
      }
      if (hL) { cur = d.x; continue; }
      if (hR) { cur = d.y; continue; }
    } else {
      if (STATS) C.v[shadow ? ST_S_LEAF : ST_C_LEAF]++;
      uint32_t first = desc_first(cur), cnt = desc_count(cur);
      if (cnt == kBigLeaf) {
        uint2 bl = S.big_leaves[first];
        first = bl.x;
        cnt = bl.y;
      }
      for (uint32_t i = 0; i < cnt; i++) {
        if (STATS) C.v[shadow ? ST_S_PRIMS : ST_C_PRIMS]++;
        float t;
        if (hit_prim<TRI_ONLY>(S.prims, first + i, r, t)) {
          if (shadow) {
            if (t <= shadow_thr) { best_prim = first + i; return true; }
          } else if (t < best_t) {
            best_t = t;
            best_prim = first + i;
            hit = true;
          }
        }
      }
    }
    bool found = false;
    while (sp > 0) {
      sp--;
      uint32_t pd;
      float pt;
      if (sp < kLdsStack) {
        pd = ls.desc[sp * kBlock];
        pt = ls.t[sp * kBlock];
      } else {
        pd = ov_desc[sp - kLdsStack];
        pt = ov_t[sp - kLdsStack];
      }
      if (shadow || pt < best_t) {
        cur = pd;
        found = true;
        break;
      }
    }
    if (!found) break;
  }
  return shadow ? false : hit;
}

// ------------------------------------------------------------------------------------------
// Uniform grid (grid.cpp:100-358): Amanatides-Woo with the reference's double stepping.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int dclampi(float x, int hi) {  // (int)clamp((double)x, 0, hi) (maths.h:65)
  double v = (double)x;
  double r = v < 0.0 ? 0.0 : (v > (double)hi ? (double)hi : v);
  return (int)r;
}

template <bool TRI_ONLY, bool STATS>
__device__ bool grid_traverse(const SceneArgs& S, const RayP& r, bool shadow, float shadow_len, float& best_t,
                              uint32_t& best_prim, Counters& C) {
  const int nx = S.gdim[0], ny = S.gdim[1], nz = S.gdim[2];
  const float x0 = S.gmin[0], y0 = S.gmin[1], z0 = S.gmin[2], x1 = S.gmax[0], y1 = S.gmax[1], z1 = S.gmax[2];
  const float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
  float txmin, tymin, tzmin, txmax, tymax, tzmax;
  if (r.sx()) { txmin = (x0 - ox) * r.ix; txmax = (x1 - ox) * r.ix; } else { txmin = (x1 - ox) * r.ix; txmax = (x0 - ox) * r.ix; }
  if (r.sy()) { tymin = (y0 - oy) * r.iy; tymax = (y1 - oy) * r.iy; } else { tymin = (y1 - oy) * r.iy; tymax = (y0 - oy) * r.iy; }
  if (r.sz()) { tzmin = (z0 - oz) * r.iz; tzmax = (z1 - oz) * r.iz; } else { tzmin = (z1 - oz) * r.iz; tzmax = (z0 - oz) * r.iz; }
  float t0 = (txmin > tymin) ? txmin : tymin;
  if (tzmin > t0) t0 = tzmin;
  float t1 = (txmax < tymax) ? txmax : tymax;
  if (tzmax < t1) t1 = tzmax;
  best_t = 3.402823466e+38f;
  if (t0 > t1 || t1 < 0.0f) return shadow;  // grid.cpp:170; shadow rays missing the box count as shadowed (:323)
  int ix, iy, iz;
  if (box_inside(x0, y0, z0, x1, y1, z1, r.o)) {
    ix = dclampi((ox - x0) * nx / (x1 - x0), nx - 1);
    iy = dclampi((oy - y0) * ny / (y1 - y0), ny - 1);
    iz = dclampi((oz - z0) * nz / (z1 - z0), nz - 1);
  } else {
    V3 p = add(r.o, mul(r.d, t0));
    ix = dclampi((p.x - x0) * nx / (x1 - x0), nx - 1);
    iy = dclampi((p.y - y0) * ny / (y1 - y0), ny - 1);
    iz = dclampi((p.z - z0) * nz / (z1 - z0), nz - 1);
  }
  const double dtx = (double)((txmax - txmin) / (float)nx);
  const double dty = (double)((tymax - tymin) / (float)ny);
  const double dtz = (double)((tzmax - tzmin) / (float)nz);
  double txn, tyn, tzn;
  int ixs, iys, izs, ixe, iye, ize;
  if (dx > 0.0f) { txn = (double)txmin + (ix + 1) * dtx; ixs = 1; ixe = nx; } else { txn = (double)txmin + (nx - ix) * dtx; ixs = -1; ixe = -1; }
  if (dx == 0.0f) txn = 3.4028234663852886e38;
  if (dy > 0.0f) { tyn = (double)tymin + (iy + 1) * dty; iys = 1; iye = ny; } else { tyn = (double)tymin + (ny - iy) * dty; iys = -1; iye = -1; }
  if (dy == 0.0f) tyn = 3.4028234663852886e38;
  if (dz > 0.0f) { tzn = (double)tzmin + (iz + 1) * dtz; izs = 1; ize = nz; } else { tzn = (double)tzmin + (nz - iz) * dtz; izs = -1; ize = -1; }
  if (dz == 0.0f) tzn = 3.4028234663852886e38;
  uint32_t closest = 0xFFFFFFFFu;
  while (true) {
    if (STATS) C.v[shadow ? ST_S_LEAF : ST_C_LEAF]++;
    const size_t cidx = (size_t)ix + (size_t)nx * iy + (size_t)nx * ny * iz;
    const uint32_t b = S.cell_start[cidx], e = S.cell_start[cidx + 1];
    for (uint32_t q = b; q < e; q++) {
      if (STATS) C.v[shadow ? ST_S_PRIMS : ST_C_PRIMS]++;
      uint32_t obj = S.cell_objs[q];
      float t;
      if (hit_prim<TRI_ONLY>(S.prims, obj, r, t)) {
        if (shadow) {
          if (t < shadow_len) { best_prim = obj; return true; }
        } else if (t < best_t) {
          best_t = t;
          closest = obj;
        }
      }
    }
    if (txn < tyn && txn < tzn) {
      if (!shadow && (double)best_t < txn) { best_prim = closest; return closest != 0xFFFFFFFFu; }
      txn += dtx; ix += ixs;
      if (ix == ixe) return false;
    } else if (tyn < tzn) {
      if (!shadow && (double)best_t < tyn) { best_prim = closest; return closest != 0xFFFFFFFFu; }
      tyn += dty; iy += iys;
      if (iy == iye) return false;
    } else {
      if (!shadow && (double)best_t < tzn) { best_prim = closest; return closest != 0xFFFFFFFFu; }
      tzn += dtz; iz += izs;
      if (iz == ize) return false;
    }
  }
}

// ------------------------------------------------------------------------------------------
// NONE: linear scan (main.cpp:315-326 closest; main.cpp:432-439 shadow, skipping the hit
// object and accepting 1e-4 < t < |L|).
// ------------------------------------------------------------------------------------------
template <bool TRI_ONLY, bool STATS>
__device__ __forceinline__ bool none_traverse(const SceneArgs& S, const RayP& r, bool shadow, float shadow_len,
                                              uint32_t skip, float& best_t, uint32_t& best_prim, Counters& C) {
  best_t = 3.402823466e+38f;
  bool hit = false;
  for (int i = 0; i < S.n_prims; i++) {
    if (shadow && (uint32_t)i == skip) continue;
    if (STATS) C.v[shadow ? ST_S_PRIMS : ST_C_PRIMS]++;
    float t;
    if (hit_prim<TRI_ONLY>(S.prims, (uint32_t)i, r, t)) {
      if (shadow) {
        if (t > 1e-4f && t < shadow_len) { best_prim = (uint32_t)i; return true; }
      } else if (t < best_t) {
        best_t = t;
        best_prim = (uint32_t)i;
        hit = true;
      }
    }
  }
  return shadow ? false : hit;
}

template <int ACCEL, bool TRI_ONLY, bool STATS>
__device__ __forceinline__ bool traverse(const SceneArgs& S, const RayP& r, bool shadow, float thr, uint32_t skip,
                                         float& t, uint32_t& prim, Counters& C, TravStack ls) {
  if (STATS) C.v[shadow ? ST_SHADOW : ST_CLOSEST]++;
  if (ACCEL == ACC_BVH) return bvh_traverse<TRI_ONLY, STATS>(S, r, shadow, thr, t, prim, C, ls);
  if (ACCEL == ACC_GRID) return grid_traverse<TRI_ONLY, STATS>(S, r, shadow, thr, t, prim, C);
  return none_traverse<TRI_ONLY, STATS>(S, r, shadow, thr, skip, t, prim, C);
}

// Largest float <= (double)len + EPSILON: `rec.t <= length + EPSILON` (bvh.cpp:376) in float.
__device__ __forceinline__ float shadow_threshold(float len) {
  double thr = (double)len + 0.001;
  float f = (float)thr;
  if ((double)f > thr) f = nextafterf(f, -INFINITY);
  return f;
}

// Scene::GetSkyboxColor (scene.cpp:380-458)
__device__ V3 skybox_color(const SceneArgs& S, V3 c) {
  float ma;
  int side;  // RIGHT, LEFT, TOP, BOTTOM, FRONT, BACK
  if (fabsf(c.x) > fabsf(c.y)) { ma = fabsf(c.x); side = c.x >= 0.0f ? 1 : 0; }
  else { ma = fabsf(c.y); side = c.y >= 0.0f ? 2 : 3; }
  if (fabsf(c.z) > ma) { ma = fabsf(c.z); side = c.z >= 0.0f ? 4 : 5; }
  float sc, tc;
  switch (side) {
    case 0: sc = -c.z; tc = c.y; break;
    case 1: sc = c.z; tc = c.y; break;
    case 2: sc = -c.x; tc = -c.z; break;
    case 3: sc = -c.x; tc = c.z; break;
    case 4: sc = -c.x; tc = c.y; break;
    default: sc = c.x; tc = c.y; break;
  }
  double invMa = (double)(1.0f / ma);
  float s = (float)(((double)sc * invMa + 1.0) / 2.0);
  float t = (float)(((double)tc * invMa + 1.0) / 2.0);
  const unsigned w = (unsigned)S.sky_w[side], h = (unsigned)S.sky_h[side], bpp = (unsigned)S.sky_bpp[side];
  unsigned xp = (unsigned)(int)((float)(w - 1u) * s);
  unsigned yp = (unsigned)(int)((float)(h - 1u) * t);
  const uint8_t* px = S.sky[side] + ((size_t)yp * w + xp) * bpp;
  return mk((float)px[0] / 255.99f, (float)px[1] / 255.99f, (float)px[2] / 255.99f);
}

__device__ __forceinline__ V3 background(const SceneArgs& S, V3 dir) {
  return S.has_sky ? skybox_color(S, dir) : mk(S.bg[0], S.bg[1], S.bg[2]);
}

// Camera::PrimaryRay (camera.h:74-83) and the thin-lens overload (camera.h:86-101).
__device__ __forceinline__ RayP primary_ray(const SceneArgs& S, float px, float py) {
  float a = px / (float)S.res_x - 0.5f;
  float b = py / (float)S.res_y - 0.5f;
  V3 dir = normalize(sub(add(mul(mul(ld3(S.u), S.w), a), mul(mul(ld3(S.v), S.h), b)), mul(ld3(S.n), S.plane_dist)));
  return make_ray(ld3(S.eye), dir);
}
__device__ __forceinline__ RayP primary_ray_lens(const SceneArgs& S, V3 lens, float px, float py) {
  V3 eo = add(add(ld3(S.eye), mul(ld3(S.u), lens.x)), mul(ld3(S.v), lens.y));
  float ppx = (px / (float)S.res_x - 0.5f) * S.w * S.focal_ratio;
  float ppy = (py / (float)S.res_y - 0.5f) * S.h * S.focal_ratio;
  float f = S.plane_dist * S.focal_ratio;
  V3 dir = normalize(sub(add(mul(ld3(S.u), ppx - lens.x), mul(ld3(S.v), ppy - lens.y)), mul(ld3(S.n), f)));
  return make_ray(eo, dir);
}

// ------------------------------------------------------------------------------------------
// Light loop (main.cpp:383-451) with the light_spp extension: the loop runs over (light, k)
// pairs j = light * m + k.  A quad light takes m points ((k % g + s.x) / g, (k / g + s.y) / g),
// g = floor(sqrt(m)), of the pixel's light sample s and each unshadowed Phong term is added
// scaled by 1/m; a point light takes only k = 0.  With m = 1 this is the reference's loop
// exactly (point = area_point(s), term scaled by nothing).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ V3 light_point(const drt_light& Lt, V3 ls, int k, const FrameArgs& F) {
  if (Lt.type != DRT_LIGHT_QUAD) return ld3(Lt.pos);
  if (F.light_spp > 1) {
    const int g = F.light_grid;
    ls = mk(((float)(k % g) + ls.x) / (float)g, ((float)(k / g) + ls.y) / (float)g, 0.0f);
  }
  return add(add(ld3(Lt.pos), mul(ld3(Lt.e1), ls.x)), mul(ld3(Lt.e2), ls.y));
}
// Phong term of an unshadowed light sample (main.cpp:444-450).
__device__ __forceinline__ V3 light_term(const drt_material& m, float NdotL, float NdotH, const drt_light& Lt,
                                         const FrameArgs& F) {
  const V3 diff = mul(mul(ld3(m.diff), m.kd), NdotL);
  const V3 spec = mul(mul(ld3(m.spec), m.ks), powf(NdotH, m.shine));
  V3 c = add(diff, spec);
  if (F.light_spp > 1 && Lt.type == DRT_LIGHT_QUAD) c = mul(c, F.light_inv);
  return c;
}
// Material / light table reads of the persistent kernels' shading (round 5).  In the BVH kernels, when
// the active lanes of the wave read at most two distinct entries (one material and the two lights of
// the benchmark scenes), the entries come through scalar loads (SMEM, the scalar cache) and a per-lane
// select instead of per-lane vector loads on the vector-memory path the kernel is bound by: replay
// vector-memory read instructions 843 -> 822 M per headline frame (scalar 377 -> 468 M), headline
// +0.3 %, C3 +0.2 %, C4 +1.9 %; the Grid stepper measured 2.8 % slower with it (register allocation)
// and keeps per-lane loads (profiles/r05_ab_uniform_tables_chain_leaf.jsonl).  -DDRT_NO_UNIFORM_TABLES
// turns it off (A/B).
template <bool UNI, class T>
__device__ __forceinline__ T tab_uni(const T* base, uint32_t i) {
  typedef const __attribute__((address_space(4))) uint32_t CU;
  constexpr int N = (int)(sizeof(T) / 4);
  static_assert(sizeof(T) % 4 == 0, "dword table entries");
  const uint32_t i0 = __builtin_amdgcn_readfirstlane(i);
  const uint64_t other = __ballot(i != i0);
  T r;
  if (other == 0) {
    CU* p = (CU*)(const void*)(base + i0);
    uint32_t w[N];
#pragma unroll
    for (int k = 0; k < N; k++) w[k] = p[k];
    __builtin_memcpy(&r, w, sizeof(T));
  } else {
    const uint32_t i1 = __builtin_amdgcn_readlane(i, (int)__builtin_ctzll(other));
    if (__ballot(i != i0 && i != i1) == 0) {
      CU* p0 = (CU*)(const void*)(base + i0);
      CU* p1 = (CU*)(const void*)(base + i1);
      const bool second = i == i1;
      uint32_t w[N];
#pragma unroll
      for (int k = 0; k < N; k++) w[k] = second ? p1[k] : p0[k];
      __builtin_memcpy(&r, w, sizeof(T));
    } else {
      r = base[i];
    }
  }
  return r;
}
template <int ACC, class T>
__device__ __forceinline__ T tab(const T* base, uint32_t i) {
#ifndef DRT_NO_UNIFORM_TABLES
  if constexpr (ACC == ACC_BVH) return tab_uni<true>(base, i);
#endif
  return base[i];
}

// Light index of pair j (no integer division in the reference case m = 1).
__device__ __forceinline__ int light_of_pair(int j, const FrameArgs& F) {
  return F.light_spp == 1 ? j : j / F.light_spp;
}
// The pair after j (point lights skip k > 0).
__device__ __forceinline__ int next_light_pair(const SceneArgs& S, const FrameArgs& F, int j) {
  j++;
  const int m = F.light_spp;
  if (m > 1) {
    const int li = j / m;
    if (j - li * m > 0 && li < S.n_lights && S.lights[li].type != DRT_LIGHT_QUAD) j = (li + 1) * m;
  }
  return j;
}

// One pending reflection/refraction parent (the C++ call frame of rayTracing, main.cpp:294).
struct Frame {
  V3 acc, hitP, N, V, lightPos, beer;
  float ior1, kr;
  uint32_t mat;
  uint32_t flags;  // bit0: in reflection child, bit1: outside, bit2: has reflection, bit3: reflectDir.N > 0
};

// ------------------------------------------------------------------------------------------
// rayTracing(ray, 1, 1.0, lightSample) — main.cpp:294-521 — as an explicit DFS.
// ------------------------------------------------------------------------------------------
template <int ACCEL, bool TRI_ONLY, bool STATS, bool RNG>
__device__ V3 trace_path(const SceneArgs& S, const FrameArgs& F, RayP q, V3 ls, KRng& rng, Counters& C,
                         TravStack tst) {
  Frame fr[kMaxFrames];
  int sp = 0;
  int depth = 1;
  float ior1 = 1.0f;
  // shading state of the node whose shadow rays are in flight
  V3 hitP = mk(0, 0, 0), N = mk(0, 0, 0), V = mk(0, 0, 0), acc = mk(0, 0, 0), lightPos = mk(0, 0, 0);
  float NdotL = 0.f, NdotH = 0.f, thr = 0.f, hitT = 0.f;
  uint32_t hitPrim = 0, mat = 0;
  bool outside = true;
  int j = 0;
  bool shadow = false;
  const float offset = 1e-4f;
  V3 result = mk(0, 0, 0);

  while (true) {
    if (STATS) {
      C.v[ST_LANE_PATH_ITERS]++;
      if (wave_leader()) C.v[ST_WAVE_PATH_ITERS]++;
    }
    float t = 0.f;
    uint32_t prim = 0;
    const bool hit = traverse<ACCEL, TRI_ONLY, STATS>(S, q, shadow, thr, hitPrim, t, prim, C, tst);

    bool ret = false;  // the current node produced its return value `c`
    V3 c = mk(0, 0, 0);
    bool after_lights = false;
    if (!shadow) {
      if (!hit) {  // main.cpp:351-357
        c = cclamp(background(S, q.d));
        ret = true;
      } else {
        hitT = t;
        hitPrim = prim;
        hitP = add(q.o, mul(q.d, hitT));  // main.cpp:361
        N = normalize(prim_normal(S.prims, prim, q, hitT));
        outside = dot(q.d, N) < 0.0f;
        if (!outside) N = neg(N);
        mat = prim_material(S.prims[3 * prim]);
        V = neg(normalize(q.d));
        acc = mk(0, 0, 0);
        lightPos = mk(0, 0, 0);
        j = 0;
        after_lights = (S.n_lights == 0);
      }
    } else {  // result of the shadow query of light pair j (main.cpp:444-450)
      const drt_light& Lt = S.lights[light_of_pair(j, F)];
      if (!hit) acc = add(acc, light_term(S.mats[mat], NdotL, NdotH, Lt, F));
      j = next_light_pair(S, F, j);
      after_lights = (j >= S.n_lights * F.light_spp);
    }

    if (!ret && !after_lights) {  // set up the shadow ray of light pair j (main.cpp:386-422)
      const int li = light_of_pair(j, F);
      lightPos = light_point(S.lights[li], ls, j - li * F.light_spp, F);
      V3 L = sub(lightPos, hitP);
      V3 Ls = L;
      L = normalize(L);
      V3 H = normalize(add(L, V));
      NdotL = smax(dot(N, L), 0.0f);
      NdotH = smax(dot(N, H), 0.0f);
      V3 so = add(hitP, mul(N, offset));
      if (ACCEL == ACC_BVH) {  // BVH::Traverse(Ray&) normalises Ls and tests t <= |Ls| + EPSILON
        thr = shadow_threshold(length(Ls));
        q = make_ray(so, normalize(Ls));
      } else if (ACCEL == ACC_GRID) {  // Grid::Traverse(Ray&): range |L|, direction re-normalised
        thr = length(L);
        q = make_ray(so, normalize(L));
      } else {  // NONE: t < L.length()
        thr = length(L);
        q = make_ray(so, L);
      }
      shadow = true;
      continue;
    }

    if (!ret) {  // after the light loop: recursion (main.cpp:453-520)
      const drt_material& m = S.mats[mat];
      if (depth > F.max_depth) {
        c = acc;  // unclamped (main.cpp:454)
        ret = true;
      } else {
        float kr = m.refl;
        float ior2 = m.ior;
        if (!outside) ior2 = 1.0f;
        float eta = ior1 / ior2;
        V3 Vt = sub(mul(N, dot(V, N)), V);
        float sin_i = length(Vt);
        V3 tv = dvf(Vt, length(Vt));
        float sin_t = eta * sin_i;
        const bool has_refr = (m.trans == 1.0f && sin_t < 1.0f);
        const bool has_refl = m.ks > 0.0f;
        RayP child = q;
        float child_ior = ior1;
        V3 beer = mk(1.f, 1.f, 1.f);
        if (has_refr) {
          float sin_t2 = (float)((double)sin_t * (double)sin_t);
          float cos_t = sqrtf(1.0f - sin_t2);
          V3 r_t = normalize(add(mul(tv, sin_t), mul(neg(N), cos_t)));
          float cos_i = dot(N, V);
          float cosTheta = (ior1 > ior2) ? cos_t : cos_i;
          float r0 = (ior1 - ior2) / (ior1 + ior2);
          r0 = (float)((double)r0 * (double)r0);
          kr = (float)((double)r0 + (double)(1.0f - r0) * pow((double)(1.0f - cosTheta), 5.0));
          if (!outside) {
            V3 e = mul(sub(mk(1.f, 1.f, 1.f), ld3(m.diff)), -hitT);
            beer = mk(expf(e.x), expf(e.y), expf(e.z));
          }
          child = make_ray(sub(hitP, mul(N, offset)), r_t);
          child_ior = ior2;
        } else if (m.trans > 0.0f && sin_t >= 1.0f) {
          kr = 1.0f;
        }
        if (has_refr || has_refl) {
          Frame& f = fr[sp++];
          f.acc = acc; f.hitP = hitP; f.N = N; f.V = V; f.lightPos = lightPos; f.beer = beer;
          f.ior1 = ior1; f.kr = kr; f.mat = mat;
          f.flags = (has_refr ? 0u : 1u) | (outside ? 2u : 0u) | (has_refl ? 4u : 0u);
          if (!has_refr) {  // straight to the reflection child (main.cpp:504-512)
            V3 R = sub(mul(mul(N, dot(V, N)), 2.0f), V);
            if (RNG) R = normalize(add(R, mul(rnd_unit_sphere(rng), F.roughness)));
            else R = normalize(R);
            if (dot(R, N) > 0.0f) f.flags |= 8u;  // reflectDir*N > 0 (main.cpp:515)
            child = make_ray(add(hitP, mul(N, offset)), R);
            child_ior = ior1;
          }
          q = child;
          ior1 = child_ior;
          ls = lightPos;  // secondary rays receive the light position as their sample (main.cpp:489, 512)
          depth++;
          shadow = false;
          continue;
        }
        c = cclamp(acc);
        ret = true;
      }
    }

    // return value c of the current node: unwind finished frames (main.cpp:489-520)
    bool resumed = false;
    while (sp > 0) {
      Frame& f = fr[sp - 1];
      if ((f.flags & 1u) == 0u) {  // refraction child returned
        V3 rc = cclamp(c);
        if ((f.flags & 2u) == 0u) rc = cmulc(rc, f.beer);
        f.acc = add(f.acc, mul(rc, 1.0f - f.kr));
        if (f.flags & 4u) {  // now the reflection child
          f.flags |= 1u;
          V3 R = sub(mul(mul(f.N, dot(f.V, f.N)), 2.0f), f.V);
          if (RNG) R = normalize(add(R, mul(rnd_unit_sphere(rng), F.roughness)));
          else R = normalize(R);
          if (dot(R, f.N) > 0.0f) f.flags |= 8u;  // reflectDir*N > 0 (main.cpp:515)
          q = make_ray(add(f.hitP, mul(f.N, offset)), R);
          ior1 = f.ior1;
          ls = f.lightPos;
          depth = sp + 1;
          shadow = false;
          resumed = true;
          break;
        }
        c = cclamp(f.acc);
        sp--;
      } else {  // reflection child returned
        V3 rc = cclamp(c);
        if (f.flags & 8u) {
          const drt_material& m = S.mats[f.mat];
          f.acc = add(f.acc, cmulc(mul(rc, f.kr), ld3(m.spec)));
        }
        c = cclamp(f.acc);
        sp--;
      }
    }
    if (resumed) continue;
    result = c;
    break;
  }
  return result;
}

// ------------------------------------------------------------------------------------------
// Work item decode + per-sample prologue (main.cpp:618-648).
// ------------------------------------------------------------------------------------------
// Tile dealing (sharding.py TileLayout): shard s renders the tiles at positions
// p = s, s + N, s + 2N, ... of a dealing order in which row ty is rotated by ty tiles, i.e. tile
// (tx, ty) sits at p = ty * tiles_x + (tx + ty) % tiles_x.  Shards then take diagonal stripes and
// every shard sees every column of the image (plain row-major dealing with tiles_x % N == 0
// gave each shard the same columns in every row: shard times 13.9-15.3 ms at N = 8).
__host__ __device__ __forceinline__ void tile_of_position(uint32_t p, uint32_t tiles_x, uint32_t& tx, uint32_t& ty) {
  ty = p / tiles_x;
  const uint32_t r = p - ty * tiles_x;
  tx = (r + tiles_x - ty % tiles_x) % tiles_x;
}
__host__ __device__ __forceinline__ uint32_t position_of_tile(uint32_t tx, uint32_t ty, uint32_t tiles_x) {
  return ty * tiles_x + (tx + ty) % tiles_x;
}

struct Item {
  int x, y, sub;
  bool valid;
};
__device__ __forceinline__ Item decode_item(const FrameArgs& F, int res_x, int res_y, uint64_t item, int per_pixel) {
  const uint64_t per_tile = (uint64_t)F.tile * F.tile * per_pixel;
  const uint32_t k = (uint32_t)(item / per_tile);
  const uint32_t rem = (uint32_t)(item - (uint64_t)k * per_tile);
  const uint32_t pix = rem / per_pixel;
  Item it;
  it.sub = (int)(rem - pix * per_pixel);
  uint32_t tx, ty;
  tile_of_position(F.shard + k * F.n_shards, F.tiles_x, tx, ty);
  it.x = (int)(tx * F.tile + pix % F.tile);
  it.y = (int)(ty * F.tile + pix / F.tile);
  it.valid = it.x < res_x && it.y < res_y;
  return it;
}

// Pixel jitter r[p] and the shuffled light sample s[p] of sample p, straight from the keyed
// stream: r uses calls 4p, 4p+1; s uses 4q+2, 4q+3 of the sample q that the Fisher-Yates pass
// (calls 4spp .. 5spp-2) moved to slot p.  Tracking slot p backwards through the swaps gives q.
__device__ __forceinline__ int shuffle_source(const FrameArgs& F, uint32_t pmix, int p) {
  const int spp = (int)F.spp;
  int pos = p;
  for (int i = 1; i < spp; i++) {
    int jj = keyed_rand(F.seed, pmix, 4u * spp + (uint32_t)(spp - 1 - i)) % (i + 1);
    if (pos == i) pos = jj;
    else if (pos == jj) pos = i;
  }
  return pos;
}
__device__ __forceinline__ void sample_prologue_at(const FrameArgs& F, uint32_t pmix, int p, int pos, float& rx,
                                                   float& ry, float& sx, float& sy) {
  const int n = F.n_sqrt;
  float ex = (float)keyed_rand(F.seed, pmix, 4u * p) / 32767.0f;
  float ey = (float)keyed_rand(F.seed, pmix, 4u * p + 1u) / 32767.0f;
  rx = ((float)(p % n) + ex) / (float)n;
  ry = ((float)(p / n) + ey) / (float)n;
  sx = (float)keyed_rand(F.seed, pmix, 4u * pos + 2u) / 32767.0f;
  sy = (float)keyed_rand(F.seed, pmix, 4u * pos + 3u) / 32767.0f;
}
__device__ __forceinline__ void sample_prologue(const FrameArgs& F, uint32_t pmix, int p, float& rx, float& ry,
                                                float& sx, float& sy) {
  sample_prologue_at(F, pmix, p, shuffle_source(F, pmix, p), rx, ry, sx, sy);
}

// The whole Fisher-Yates pass of main.cpp:642-648 once per pixel, forward, on an LDS copy of
// the slot array: perm[pixel * spp + p] = the sample whose light sample ends in slot p — what
// shuffle_source finds for one slot by walking the spp - 1 swaps backwards.  The path kernel
// then reads one byte per sample instead of hashing spp - 1 keyed draws.
constexpr int kShuffleBlock = 64;
__global__ void __launch_bounds__(kShuffleBlock) shuffle_kernel(FrameArgs F, int res_x, int res_y, uint8_t* perm) {
  __shared__ uint8_t a[256 * kShuffleBlock];  // a[k * kShuffleBlock + thread]
  const uint32_t px = blockIdx.x * kShuffleBlock + threadIdx.x;
  const uint32_t n_px = (uint32_t)F.n_my_tiles * F.tile * F.tile;
  if (px >= n_px) return;
  const Item it = decode_item(F, res_x, res_y, px, 1);
  const int spp = (int)F.spp;
  uint8_t* o = perm + (size_t)px * spp;
  if (!it.valid) return;  // padding of a partial tile: never read
  const uint32_t pmix = (uint32_t)(it.y * res_x + it.x) * 0x9E3779B9u;
  for (int k = 0; k < spp; k++) a[k * kShuffleBlock + threadIdx.x] = (uint8_t)k;
  for (int i = spp - 1; i >= 1; i--) {  // j = rand() % (i + 1); swap(s[i], s[j])
    const int j = keyed_rand(F.seed, pmix, 4u * spp + (uint32_t)(spp - 1 - i)) % (i + 1);
    const uint8_t t = a[i * kShuffleBlock + threadIdx.x];
    a[i * kShuffleBlock + threadIdx.x] = a[j * kShuffleBlock + threadIdx.x];
    a[j * kShuffleBlock + threadIdx.x] = t;
  }
  for (int k = 0; k < spp; k++) o[k] = a[k * kShuffleBlock + threadIdx.x];
}

template <bool STATS>
__device__ __forceinline__ void flush_stats(const FrameArgs& F, const Counters& C) {
  if (!STATS) return;
  for (int s = 0; s < ST_COUNT; s++) {
    unsigned long long v = C.v[s];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&F.stats[s], v);
  }
}

// Progressive zone A primary ray and light sample (main.cpp:556-571): pixel_sample = (x +
// rand_double(), y + rand_double()) — the double sum of an int and r/32768 rounded to float is
// the float sum of the same exact operands — then the lens (DoF), then Vector(rand_float(),
// rand_float(), 0) whose first draw (right-to-left evaluation) is the y component.
__device__ __forceinline__ void prog_primary(const SceneArgs& S, const FrameArgs& F, const Item& it, KRng& rng,
                                             RayP& r, V3& ls) {
  const float px = (float)it.x + rng.rand_float();
  const float py = (float)it.y + rng.rand_float();
  if (F.dof) r = primary_ray_lens(S, dvf(mul(rnd_unit_disk(rng), S.aperture), 2.0f), px, py);
  else r = primary_ray(S, px, py);
  const float ly = rng.rand_float();
  const float lx = rng.rand_float();
  ls = mk(lx, ly, 0.0f);
}

template <int ACCEL, bool TRI_ONLY, bool STATS, int MODE>
__global__ void __launch_bounds__(kBlock) path_kernel(SceneArgs S, FrameArgs F) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_stack[];
  TravStack tst{(LdsU32*)lds_stack + threadIdx.x, (LdsF32*)(lds_stack + kLdsStack * kBlock) + threadIdx.x};
  const uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Counters C;
  for (int s = 0; s < ST_COUNT; s++) C.v[s] = 0;
  if (item < F.n_items) {
    const int per_pixel = (MODE == MODE_SEQ) ? 1 : F.nsub;
    Item it = decode_item(F, S.res_x, S.res_y, item, per_pixel);
    V3 color = mk(0, 0, 0);
    if (it.valid) {
      const uint32_t P = (uint32_t)(it.y * S.res_x + it.x);
      const uint32_t pmix = P * 0x9E3779B9u;
      KRng rng{F.seed, pmix, 0};
      if (MODE == MODE_AA) {
        float rx, ry, sx, sy;
        sample_prologue(F, pmix, it.sub, rx, ry, sx, sy);
        RayP r = primary_ray(S, (float)it.x + rx, (float)it.y + ry);
        if (STATS) C.v[ST_SAMPLES]++;
        color = trace_path<ACCEL, TRI_ONLY, STATS, false>(S, F, r, mk(sx, sy, 0.0f), rng, C, tst);
      } else if (MODE == MODE_SEQ) {
        if (F.spp > 0) {  // AA with DoF and/or glossy reflection: the keyed stream in call order
          rng.k = 5u * F.spp - 1u;
          for (int p = 0; p < (int)F.spp; p++) {
            float rx, ry, sx, sy;
            sample_prologue(F, pmix, p, rx, ry, sx, sy);
            const float px = (float)it.x + rx, py = (float)it.y + ry;
            RayP r;
            if (F.dof) r = primary_ray_lens(S, dvf(mul(rnd_unit_disk(rng), S.aperture), 2.0f), px, py);
            else r = primary_ray(S, px, py);
            if (STATS) C.v[ST_SAMPLES]++;
            color = add(color, trace_path<ACCEL, TRI_ONLY, STATS, true>(S, F, r, mk(sx, sy, 0.0f), rng, C, tst));
          }
        } else {  // Whitted with glossy reflection: each light sample in order on one stream
          RayP r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
          const int ns = F.grid_res ? (int)F.grid_res : 1;
          for (int s = 0; s < ns; s++) {
            V3 ls = F.grid_res ? mk(((float)(s % F.grid_size) + 0.5f) / (float)F.grid_size,
                                    ((float)(s / F.grid_size) + 0.5f) / (float)F.grid_size, 0.0f)
                               : mk(0.5f, 0.5f, 0.0f);
            if (STATS) C.v[ST_SAMPLES]++;
            color = add(color, trace_path<ACCEL, TRI_ONLY, STATS, true>(S, F, r, ls, rng, C, tst));
          }
        }
      } else if (MODE == MODE_PROG) {
        RayP r;
        V3 ls;
        prog_primary(S, F, it, rng, r, ls);
        if (STATS) C.v[ST_SAMPLES]++;
        color = trace_path<ACCEL, TRI_ONLY, STATS, true>(S, F, r, ls, rng, C, tst);
      } else if (MODE == MODE_WHITTED_QUAD) {
        const int s = it.sub;
        V3 ls = mk(((float)(s % F.grid_size) + 0.5f) / (float)F.grid_size,
                   ((float)(s / F.grid_size) + 0.5f) / (float)F.grid_size, 0.0f);
        RayP r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
        if (STATS) C.v[ST_SAMPLES]++;
        color = trace_path<ACCEL, TRI_ONLY, STATS, false>(S, F, r, ls, rng, C, tst);
      } else {
        RayP r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
        if (STATS) C.v[ST_SAMPLES]++;
        color = trace_path<ACCEL, TRI_ONLY, STATS, false>(S, F, r, mk(0.5f, 0.5f, 0.0f), rng, C, tst);
      }
    }
    F.samples[item] = make_float4(color.x, color.y, color.z, 0.0f);
  }
  flush_stats<STATS>(F, C);
}

// ------------------------------------------------------------------------------------------
// Persistent BVH path kernel (all frame modes; MODE_SEQ runs a pixel's samples in order on one
// lane because its keyed stream is consumed in call order).
//
// Each lane runs rayTracing()'s DFS as an explicit state machine and every loop iteration
// does ONE unit of work per lane: a BVH node step (inner node, or leaf + stack pops) for lanes
// with a query in flight, or a shading step (consume a query result, set up the next shadow /
// secondary query or unwind a finished frame) for lanes whose query has completed.  Shading is
// batched: it runs only when `process_min` lanes are waiting (or nobody is traversing), so the
// long shading code is not re-entered for a single lane.  Lanes whose sample is finished are
// refilled from a global work counter, `refill_min` at a time, so waves never drain while any
// work is left.  Results are per work item (sample) exactly as in path_kernel; the ordered
// per-pixel reduce is unchanged, so frames are bit-identical.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kNoItem = 0xFFFFFFFFu;
constexpr uint32_t kPartYield = 0xFFFFFFFFu;  // MODE_SEQ tail: the wave hands its pixels over

// LDS traversal-stack entries per thread for a given occupancy target (5 blocks of 256 threads
// fit 16 entries in 160 KiB; 6-8 blocks need a shorter LDS stack, the rest spills to scratch).
__host__ __device__ constexpr int lds_cap(int waves) {
  // per thread: 160 KiB over waves * 4 SIMDs * 64 lanes, 8 B per entry, whatever the block size
  return (160 * 1024 / (waves * 256 * 8) - 1) < 16 ? (160 * 1024 / (waves * 256 * 8) - 1) : 16;
}

// Per-lane state flags, packed into one VGPR: divergent bools kept as separate variables
// become 64-bit SGPR lane masks that the loop has to carry (and spill) across iterations.
enum LaneFlag : uint32_t {
  LF_SHADOW = 1u,   // query in flight is a shadow (any-hit) query
  LF_TRAV = 2u,     // query still traversing
  LF_HIT = 4u,      // query found a hit
  LF_POP = 8u,      // next node step starts with a pop attempt
  LF_FINITE = 16u,  // ray origin and (float)(1.0/d) are all finite
  LF_OUTSIDE = 32u, // shading state: the hit was on the outside of the surface (main.cpp:364)
  LF_EMPTY = 64u,   // Grid: the current cell lies in an empty macro-cell (no range load needed)
  LF_INCELL = 128u, // Grid: objects of the current cell left, from record L.spa on
  LF_YIELD = 256u,  // MODE_SEQ tail: the lane's wave is handing its pixels over (set per shading pass)
  LF_RESUME = 512u, // MODE_SEQ tail: the lane took over a pixel; its next sample starts in finish_sample
  LF_LEAFCONT = 1024u, // BVH: `cur` is the rest of a leaf whose first primitives were tested (not a new visit)
  LF_WIDE = 2048u,     // BVH shadow query on the 4-ary shadow tree (drt_layout.hpp)
  LF_VERIFY = 4096u,   // shadow tree: primitive `cur` was hit within range; check its leaf's exact box
  LF_GVFB = 8192u      // Grid scene's shadow tree (trace_stream GV): no cell certificate, the Grid walk answers
};

struct Lane {
  uint32_t item;
  uint32_t fl;  // LaneFlag bits
  // query in flight
  RayP q;
  uint32_t cur, best_prim;
  // traversal-stack pointer as an LDS byte address: spa = depth * kRowBytes + threadIdx.x * 4
  // (the [entry][thread] layout of a kPBlock-thread block), so depth = spa >> kRowShift and the
  // lane's own column survives in the low bits — no base address has to stay live across the loop
  uint32_t spa;
  float best_t, thr;
  // path (rayTracing call chain)
  int depth, fsp;
  float ior1;
  V3 ls;
  // node being shaded
  V3 hitP, N, V, acc, lightPos;
  float NdotL, NdotH, hitT;
  uint32_t hitPrim, mat;
  int j;
  // MODE_SEQ / MODE_PROG only (dead otherwise): the lane owns a pixel and runs its samples in
  // order on the pixel's keyed stream — sample index, next rand() call index, pixel key
  uint32_t smp, rk, pmix;
  // ACC_GRID only (dead otherwise): the 3D-DDA of Grid::Traverse in double (grid.cpp:200-245);
  // the cell is packed in `cur` (ix | iy << 10 | iz << 20)
  // t_next per axis in double; dt per axis is a float widened to double (grid.cpp: dtx =
  // (txmax - txmin) / nx in float), so it is kept as the float (3 VGPRs instead of 6)
  double gtx, gty, gtz;
  float gdx, gdy, gdz;
};
// (Measured alternative, kept out: the shading state in a private per-activation frame array
// instead of registers — the extra scratch stores sit in vmcnt ahead of the next node fetch,
// 9 % slower.)

// AABB::hit + isInside (boundingBox.cpp:41-44, :64-124; bvh.cpp:256-257) for a ray whose origin
// and slab constants are finite.  Every slab product is then finite and, because a child box has
// min <= max, the product from the near plane is the smaller one on every axis: min/max pick
// exactly the values the reference's sign-selected MAX3/MIN3 pick (a zero may differ in sign,
// which no later comparison can observe).  `p > mn` equals `mn - p < 0` for finite floats (a
// difference of distinct floats never rounds to zero), so the inside test reuses the slab
// differences.
__device__ __forceinline__ bool box_test_finite(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                                const RayP& r, float& t) {
  const float dnx = mnx - r.o.x, dny = mny - r.o.y, dnz = mnz - r.o.z;
  const float dxx = mxx - r.o.x, dxy = mxy - r.o.y, dxz = mxz - r.o.z;
  const float ax = dnx * r.ix, bx = dxx * r.ix;
  const float ay = dny * r.iy, by = dxy * r.iy;
  const float az = dnz * r.iz, bz = dxz * r.iz;
  const float t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
  const float t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
  // inside <=> max(mn - o) < 0 && min(mx - o) > 0 <=> max(max(mn - o), -min(mx - o)) < 0, and
  // hit <=> t0 < t1 && t1 > 0 <=> max(t0, 0) < t1 — both exact without NaNs, and branch-free
  const float in = fmaxf(fmaxf(fmaxf(dnx, dny), dnz), -fminf(fminf(dxx, dxy), dxz));
  const float te = (t0 < 0.0f) ? t1 : t0;
  t = (in < 0.0f) ? 0.0f : te;
  return fmaxf(t0, 0.0f) < t1;
}
__device__ __forceinline__ bool ray_finite(const RayP& r) {
  return inv_finite(r) && fabsf(r.o.x) < __builtin_inff() && fabsf(r.o.y) < __builtin_inff() &&
         fabsf(r.o.z) < __builtin_inff();
}
// Shadow-tree lanes: finite rays; with the one-fma child test (DRT_WIDE_FMA1, node_step) also |inv| <=
// 2^40 (no direction component below ~1e-12 of the ray's length) and |o| <= 2^60.
__device__ __forceinline__ bool wide_ray_ok(const RayP& r) {
#ifndef DRT_WIDE_FMA1
  return ray_finite(r);
#else
  const float mi = fmaxf(fmaxf(fabsf(r.ix), fabsf(r.iy)), fabsf(r.iz));
  const float mo = fmaxf(fmaxf(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z));
  return mi <= 0x1p40f && mo <= 0x1p60f;  // false for NaN
#endif
}

// Grid::Traverse(Ray&)'s first step (grid.cpp:318-324): a shadow ray whose slab test misses the grid box
// counts as shadowed.  The same float arithmetic as grid_traverse / grid_init.
__device__ __forceinline__ bool grid_box_missed(const SceneArgs& S, const RayP& r) {
  const float x0 = S.gmin[0], y0 = S.gmin[1], z0 = S.gmin[2], x1 = S.gmax[0], y1 = S.gmax[1], z1 = S.gmax[2];
  float txmin, tymin, tzmin, txmax, tymax, tzmax;
  if (r.sx()) { txmin = (x0 - r.o.x) * r.ix; txmax = (x1 - r.o.x) * r.ix; } else { txmin = (x1 - r.o.x) * r.ix; txmax = (x0 - r.o.x) * r.ix; }
  if (r.sy()) { tymin = (y0 - r.o.y) * r.iy; tymax = (y1 - r.o.y) * r.iy; } else { tymin = (y1 - r.o.y) * r.iy; tymax = (y0 - r.o.y) * r.iy; }
  if (r.sz()) { tzmin = (z0 - r.o.z) * r.iz; tzmax = (z1 - r.o.z) * r.iz; } else { tzmin = (z1 - r.o.z) * r.iz; tzmax = (z0 - r.o.z) * r.iz; }
  float t0 = (txmin > tymin) ? txmin : tymin;
  if (tzmin > t0) t0 = tzmin;
  float t1 = (txmax < tymax) ? txmax : tymax;
  if (tzmax < t1) t1 = tzmax;
  return t0 > t1 || t1 < 0.0f;  // grid.cpp:170 (NaN compares false: not missed, as there)
}

// The Grid cell certificate of a shadow-tree hit (trace_stream GV).  Primitive P was hit at t < range.
// Grid::Traverse(Ray&) (grid.cpp:309-358) tests P as soon as its DDA enters any cell of P's cell range
// (Grid::Build registers P in every cell of [min, max] of its box, grid.cpp:78-92), and the walk
// covers the ray from its start to the grid's exit.  The ray's point at t, p = o + t d, lies in the
// grid; if it lies in a cell c of P's range, more than S.gmargin of a cell from each of c's faces, the
// DDA visits c — its face crossing times are the float-rounded Init_Traverse values stepped in double,
// off by less than 16 eps K n cells after n steps (|t_min|, |dt| and the products each carry a few float
// roundings of values up to K grid widths, K = 1 + max_a (|min_a| + |max_a|) / width_a), and the walk's
// start cell is off only within that distance of a face — so the walk tests P there and answers
// occluded (or finds another occluder first).  The cell coordinate u = (o + t d - min) * n / width is
// computed here in float, within 5 eps K n cells of the real one; S.gmargin = 128 eps K n_max (scene_args)
// is 6x the two bounds together.  rng0 = (ix_min, iy_min, iz_min, ix_max), rng1 = (iy_max, iz_max, ., .).
__device__ __forceinline__ bool grid_certificate(const SceneArgs& S, const RayP& r, float t, const float4& rng0,
                                                 const float4& rng1) {
  const float m = S.gmargin;
  const float ux = (r.o.x + t * r.d.x - S.gmin[0]) * S.gscale[0];
  const float uy = (r.o.y + t * r.d.y - S.gmin[1]) * S.gscale[1];
  const float uz = (r.o.z + t * r.d.z - S.gmin[2]) * S.gscale[2];
  const float cx = floorf(ux), cy = floorf(uy), cz = floorf(uz);
  const float fx = ux - cx, fy = uy - cy, fz = uz - cz;
  return fx > m && fx < 1.0f - m && fy > m && fy < 1.0f - m && fz > m && fz < 1.0f - m &&  // (false for NaN)
         cx >= rng0.x && cx <= rng0.w && cy >= rng0.y && cy <= rng1.x && cz >= rng0.z && cz <= rng1.y;
}

// Grid::Init_Traverse (grid.cpp:160-245) for the lane's query: grid-box entry, first cell and
// the double-precision DDA state, exactly as grid_traverse computes them.  False: box missed.
__device__ __forceinline__ bool grid_init(const SceneArgs& S, Lane& L) {
  const RayP& r = L.q;
  const int nx = S.gdim[0], ny = S.gdim[1], nz = S.gdim[2];
  const float x0 = S.gmin[0], y0 = S.gmin[1], z0 = S.gmin[2], x1 = S.gmax[0], y1 = S.gmax[1], z1 = S.gmax[2];
  const float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
  float txmin, tymin, tzmin, txmax, tymax, tzmax;
  if (r.sx()) { txmin = (x0 - ox) * r.ix; txmax = (x1 - ox) * r.ix; } else { txmin = (x1 - ox) * r.ix; txmax = (x0 - ox) * r.ix; }
  if (r.sy()) { tymin = (y0 - oy) * r.iy; tymax = (y1 - oy) * r.iy; } else { tymin = (y1 - oy) * r.iy; tymax = (y0 - oy) * r.iy; }
  if (r.sz()) { tzmin = (z0 - oz) * r.iz; tzmax = (z1 - oz) * r.iz; } else { tzmin = (z1 - oz) * r.iz; tzmax = (z0 - oz) * r.iz; }
  float t0 = (txmin > tymin) ? txmin : tymin;
  if (tzmin > t0) t0 = tzmin;
  float t1 = (txmax < tymax) ? txmax : tymax;
  if (tzmax < t1) t1 = tzmax;
  if (t0 > t1 || t1 < 0.0f) return false;  // grid.cpp:170
  int ix, iy, iz;
  if (box_inside(x0, y0, z0, x1, y1, z1, r.o)) {
    ix = dclampi((ox - x0) * nx / (x1 - x0), nx - 1);
    iy = dclampi((oy - y0) * ny / (y1 - y0), ny - 1);
    iz = dclampi((oz - z0) * nz / (z1 - z0), nz - 1);
  } else {
    V3 p = add(r.o, mul(r.d, t0));
    ix = dclampi((p.x - x0) * nx / (x1 - x0), nx - 1);
    iy = dclampi((p.y - y0) * ny / (y1 - y0), ny - 1);
    iz = dclampi((p.z - z0) * nz / (z1 - z0), nz - 1);
  }
  L.gdx = (txmax - txmin) / (float)nx;
  L.gdy = (tymax - tymin) / (float)ny;
  L.gdz = (tzmax - tzmin) / (float)nz;
  L.gtx = (dx > 0.0f) ? (double)txmin + (ix + 1) * (double)L.gdx : (double)txmin + (nx - ix) * (double)L.gdx;
  if (dx == 0.0f) L.gtx = 3.4028234663852886e38;
  L.gty = (dy > 0.0f) ? (double)tymin + (iy + 1) * (double)L.gdy : (double)tymin + (ny - iy) * (double)L.gdy;
  if (dy == 0.0f) L.gty = 3.4028234663852886e38;
  L.gtz = (dz > 0.0f) ? (double)tzmin + (iz + 1) * (double)L.gdz : (double)tzmin + (nz - iz) * (double)L.gdz;
  if (dz == 0.0f) L.gtz = 3.4028234663852886e38;
  L.cur = (uint32_t)ix | ((uint32_t)iy << 10) | ((uint32_t)iz << 20);
  return true;
}

// The DDA step of grid.cpp:268-303 / :337-355 as selects, not a three-way branch: the axis whose
// t_next is smallest (the reference's if / else-if order; NaN falls to z), the closest-hit exit
// (best.t < that t_next) and one double add on the selected axis — the value the reference's
// `tx_next += dtx` gives.  A lane with `act` false keeps its state, so the empty-macro-cell walk
// is a wave-uniform loop (one ballot per iteration) instead of divergent exec-mask bookkeeping:
// the branchy form spent ~60 SALU per step (SALU 144.5 G vs VALU 97.8 G per frame).  Plain
// values in and out: selects between lvalues became selects between addresses and put the lane
// state in scratch.
struct DdaState {
  double tx, ty, tz;
  int ix, iy, iz;
  bool end, exited;
};
struct DdaAxes {
  double dx, dy, dz;  // dtx, dty, dtz
  int sx, sy, sz;     // ix_step ...
  int ex, ey, ez;     // ix_stop ...
};
__device__ __forceinline__ double sel3(bool cx, bool cy, double a, double b, double c) {
  const double r = cy ? b : c;
  return cx ? a : r;
}
__device__ __forceinline__ DdaState dda_step(DdaState d, const DdaAxes& a, bool act, bool shadow, double bt) {
  const bool cx = d.tx < d.ty && d.tx < d.tz;
  const bool cy = !cx && d.ty < d.tz;
  const bool cz = !cx && !cy;
  const double tsel = sel3(cx, cy, d.tx, d.ty, d.tz);
  const bool e = act && !shadow && bt < tsel;
  const bool adv = act && !e;
  const double tn = tsel + sel3(cx, cy, a.dx, a.dy, a.dz);
  d.tx = (adv && cx) ? tn : d.tx;
  d.ty = (adv && cy) ? tn : d.ty;
  d.tz = (adv && cz) ? tn : d.tz;
  d.ix += (adv && cx) ? a.sx : 0;
  d.iy += (adv && cy) ? a.sy : 0;
  d.iz += (adv && cz) ? a.sz : 0;
  d.exited = d.exited || (adv && ((cx && d.ix == a.ex) || (cy && d.iy == a.ey) || (cz && d.iz == a.ez)));
  d.end = d.end || e;
  return d;
}

// One cell of Grid::Traverse (grid.cpp:247-306 closest, :309-358 shadow): the cell's objects in
// insertion order (shadow: any t < |d| ends the query), then the DDA step — closest hits end
// when best.t < t_next of the stepped axis, leaving the grid is a miss (even with a farther hit).
// (Measured alternative, kept out: one memory round trip per iteration — the cell range, or two
// objects with the next cell's range prefetched speculatively — 6-17 % slower than a whole cell
// per iteration.  Round 3: the same stream inside one call — up to R rounds, each giving every
// lane one unit of memory work in shared load instructions (its next two objects, or its new
// cell's range through the first object slot), with the DDA step and a capped walk per round:
// 1.1-1.2 G vector-memory instructions fewer and a third less waiting, but SALU 41 -> 57-67 G and
// LDS 0.25 -> 0.69 G (the walk and its macro-cell lookups once per round): 1 010-1 090 against
// 1 292 Mrays/s at every (R, walk) tried, branch-free loads included
// (profiles/r03_grid_stream_ab.jsonl).  Cells and records in macro-cell-bricked order: neutral.
// A 64-bit occupancy mask per macro-cell, read beside a cell's range once per macro-cell and held
// in two VGPRs, so that the walk also steps through the empty cells of non-empty macro-cells
// (36-48 % of their cells) without loading their ranges: bit-identical, but VGPR spills 102 ->
// 115 and 1 047 against 1 300 Mrays/s; 3-11 % slower on the shipped Grid scenes too.)
// triangle scenes read the 40-B pair layout (drt_upload_grid); -DDRT_GRID_RECS48 keeps the 48-B
// records for every scene (A/B)
template <bool TRI_ONLY>
constexpr bool kGridPacked =
#if defined(DRT_GRID_RECS48) || defined(DRT_GRID_INDEXED)  // (the indexed A/B layout uses the 48-B records)
    false;
#else
    TRI_ONLY;
#endif
template <bool TRI_ONLY, bool STATS>
__device__ __forceinline__ void grid_step(const SceneArgs& S, Lane& L, Counters& C, const LdsU32* macro, int walk,
                                          int pairs) {
  uint32_t fl = L.fl;
  const bool shadow = (fl & LF_SHADOW) != 0u;
  const int nx = S.gdim[0], ny = S.gdim[1], nz = S.gdim[2];
  int ix = (int)(L.cur & 1023u), iy = (int)((L.cur >> 10) & 1023u), iz = (int)(L.cur >> 20);
  const bool resume = (fl & LF_INCELL) != 0u;  // the cell's objects from the cursor on
  if (STATS && !resume) C.v[shadow ? ST_S_LEAF : ST_C_LEAF]++;
  const size_t cidx = (size_t)ix + (size_t)nx * iy + (size_t)nx * ny * iz;
  uint32_t b = 0, e = 0;  // LF_EMPTY: the cell lies in an empty macro-cell (the last call's walk)
  if (!(fl & LF_EMPTY)) {  // the cell's range [start, next start) in one 8-B load (4-B aligned)
    uint2 r;
    __builtin_memcpy(&r, (kGridPacked<TRI_ONLY> ? S.cell_tpos : S.cell_start) + cidx, sizeof(r));
    if (kGridPacked<TRI_ONLY>) {  // pair-aligned starts; bit 31 of the next start: this list ends on a padding slot
      r.x &= 0x7fffffffu;
      r.y = (r.y & 0x7fffffffu) - (r.y >> 31);
    }
    b = resume ? L.spa : r.x;
    e = r.y;
  }
  // the cell's objects in insertion order, two inline records (drt_upload_grid) per round trip
  // (Measured alternative, kept out (round 3): 16-B per-cell records (start, end, first two object
  // indices) over the scene-order primitives, so that an object's one record serves every cell it
  // overlaps instead of 3.3 inline copies; later indices read two at a time beside the pair before.
  // Same dependent round trips and bit-identical frames, but one more load per pair and 32 more VGPR
  // spills: 916 against 1 298 Mrays/s on the 1M-triangle grid.)
  bool done = false;
  // triangle scenes: the test and the hit update as selects, no exec-mask branches per object
  // (+1.3 % Mrays/s on the Grid; the same test in the BVH leaf block measured -1.7 %)
  auto test = [&](const float4& p0, const float4& p1, const float4& p2) {
    if (STATS) C.v[shadow ? ST_S_PRIMS : ST_C_PRIMS]++;
    float t;
    bool h;
    if (TRI_ONLY) h = hit_triangle_sel(p0, p1, p2, L.q, t);
    else h = hit_prim_rec<TRI_ONLY>(p0, p1, p2, L.q, t);
    const bool nearer = h & !shadow & (t < L.best_t);
    done = done | (h & shadow & (t < L.thr));
    L.best_t = nearer ? t : L.best_t;
    L.best_prim = nearer ? __float_as_uint(p2.w) : L.best_prim;
  };
#ifdef DRT_GRID_DIAG
  if (STATS) C.v[ST_CYC_LEAF]++;  // lane cell visits (grid_step calls)
#endif
  // At most `pairs` round trips per call, for the same reason as the walk's cap below: a lane in
  // a crowded cell would keep the wave in this loop while the others wait.  It stays in the cell
  // (LF_INCELL, the next record in L.spa, which the Grid stepper does not otherwise use) and goes
  // on in the next call.
  bool stay = false;
  for (uint32_t q = b, k = 0; q < e; q += 2, k++) {
    if (k == (uint32_t)pairs) {
      stay = true;
      L.spa = q;
      break;
    }
#ifdef DRT_GRID_DIAG
    if (STATS && wave_leader()) C.v[ST_WAVE_LEAF_ITERS]++;  // pair-loop wave iterations
#endif
    const bool two = q + 1 < e;
#ifdef DRT_GRID_INDEXED
    uint2 ix;  // the pair's record positions (one 8-B load, 4-B aligned)
    __builtin_memcpy(&ix, S.cell_pos + q, sizeof(ix));
    const float4* r = S.gprims + 3 * (size_t)ix.x;
    const float4* r2 = S.gprims + 3 * (size_t)ix.y;
    const float4 a0 = r[0], a1 = r[1], a2 = r[2];
    float4 c0, c1, c2;
    if (two) {
      c0 = r2[0];
      c1 = r2[1];
      c2 = r2[2];
    }
#else
    float4 a0, a1, a2, c0, c1, c2;
    if (kGridPacked<TRI_ONLY>) {  // a pair of 40-B triangle records (q is even): five 16-B loads, three for one
      const float4* r = S.cell_tris + 5 * (size_t)(q >> 1);
      const float4 x0 = r[0], x1 = r[1], x2 = r[2];
      float4 x3, x4;
      if (two) {
        x3 = r[3];
        x4 = r[4];
      }
      a0 = make_float4(x0.x, x0.y, x0.z, 0.0f);      // v0
      a1 = make_float4(x0.w, x1.x, x1.y, 0.0f);      // e1
      a2 = make_float4(x1.z, x1.w, x2.x, x2.y);      // e2, scene index
      c0 = make_float4(x2.z, x2.w, x3.x, 0.0f);
      c1 = make_float4(x3.y, x3.z, x3.w, 0.0f);
      c2 = make_float4(x4.x, x4.y, x4.z, x4.w);
    } else {
      const float4* r = S.cell_recs + 3 * (size_t)q;
      a0 = r[0];
      a1 = r[1];
      a2 = r[2];
      if (two) {
        c0 = r[3];
        c1 = r[4];
        c2 = r[5];
      }
    }
#endif
    test(a0, a1, a2);
    if (!done && two) test(c0, c1, c2);
    if (done) {
      L.fl = (fl | LF_HIT) & ~LF_TRAV;
      return;
    }
  }
  // the DDA step as selects (dda_step) and the empty-macro-cell walk as a wave-uniform loop
  const float dx = L.q.d.x, dy = L.q.d.y, dz = L.q.d.z;
  const int sx = dx > 0.0f ? 1 : -1, sy = dy > 0.0f ? 1 : -1, sz = dz > 0.0f ? 1 : -1;
  const int ex = dx > 0.0f ? nx : -1, ey = dy > 0.0f ? ny : -1, ez = dz > 0.0f ? nz : -1;
  const double bt = (double)L.best_t;
  DdaState d{L.gtx, L.gty, L.gtz, ix, iy, iz, false, false};
  const DdaAxes ax{(double)L.gdx, (double)L.gdy, (double)L.gdz, sx, sy, sz, ex, ey, ez};
  d = dda_step(d, ax, !stay, shadow, bt);
  // Cells of an empty macro-cell hold no object: walk through them here (the same steps and
  // end tests, no memory access) instead of spending a loop iteration and a load on each.  At most
  // `walk` steps per call: the loop is wave-uniform, and the lanes of a long empty run (a ray
  // through the empty space around the objects) would otherwise keep the whole wave stepping for a
  // few lanes (measured: 38 walk iterations per call at 2 active lanes).  A lane still in an empty
  // macro-cell after them goes on in the next call, with LF_EMPTY telling it to skip that cell's
  // range load (the cell is empty).
  const int ms = S.gmacro_shift, mx = S.gmacro_dim[0], my = S.gmacro_dim[1];
  bool pending = false;  // stopped by the cap inside an empty macro-cell
  for (int w = 0;; w++) {
    bool act = !stay && !d.end && !d.exited;
    const uint32_t mi = act ? (uint32_t)(d.ix >> ms) + (uint32_t)mx * ((uint32_t)(d.iy >> ms) + (uint32_t)my * (uint32_t)(d.iz >> ms))
                            : 0u;
    act = act && !((macro[mi >> 5] >> (mi & 31u)) & 1u);
    if (w == walk) {
      pending = act;
      break;
    }
    if (__ballot(act) == 0) break;
    if (STATS && act) C.v[shadow ? ST_S_LEAF : ST_C_LEAF]++;
#ifdef DRT_GRID_DIAG
    if (STATS && act) C.v[ST_PUSH]++;                     // walk lane steps
    if (STATS && wave_leader()) C.v[ST_PUSH_SPILL]++;     // walk wave iterations
#endif
    d = dda_step(d, ax, act, shadow, bt);
  }
  L.gtx = d.tx;
  L.gty = d.ty;
  L.gtz = d.tz;
  ix = d.ix;
  iy = d.iy;
  iz = d.iz;
  const bool end = d.end, exited = d.exited;
  fl = pending ? (fl | LF_EMPTY) : (fl & ~LF_EMPTY);
  fl = stay ? (fl | LF_INCELL) : (fl & ~LF_INCELL);
  if (end) fl = (fl & ~LF_TRAV) | (L.best_prim != 0xFFFFFFFFu ? LF_HIT : 0u);
  else if (exited) fl &= ~LF_TRAV;
  else L.cur = (uint32_t)ix | ((uint32_t)iy << 10) | ((uint32_t)iz << 20);
  L.fl = fl;
}

template <bool STATS, int ACC, bool WIDE = false>
__device__ __forceinline__ void start_query(const SceneArgs& S, Lane& L, const RayP& q, bool shadow, float thr,
                                            Counters& C) {
  if (STATS) C.v[shadow ? ST_SHADOW : ST_CLOSEST]++;
  L.q = q;
  L.thr = thr;
  L.best_t = 3.402823466e+38f;
  if (ACC == ACC_GRID) {
    L.best_prim = 0xFFFFFFFFu;
    const bool in = grid_init(S, L);
    // a shadow ray that misses the grid box counts as shadowed (grid.cpp:323-324, Q8)
    L.fl = (L.fl & LF_OUTSIDE) | (shadow ? LF_SHADOW : 0u) | (in ? LF_TRAV : (shadow ? LF_HIT : 0u));
    return;
  }
  L.spa &= kRowBytes - 1u;
  L.cur = S.root_desc;
  float tmp;
  const bool root = box_hit(S.root_box[0], S.root_box[1], S.root_box[2], S.root_box[3], S.root_box[4],
                            S.root_box[5], q, tmp);  // bvh.cpp:242 / :328: a root miss is an empty result
  const bool fin = ray_finite(q);
  L.fl = (L.fl & LF_OUTSIDE) | (shadow ? LF_SHADOW : 0u) | (root ? LF_TRAV : 0u) | (fin ? LF_FINITE : 0u);
  // finite shadow rays walk the 4-ary shadow tree; the others keep the reference's slab NaN rules
  // on its binary tree
  if (WIDE && shadow && fin && S.wnodes != nullptr && wide_ray_ok(q)) {
    if (STATS) C.v[ST_W_RAYS]++;
    L.fl |= LF_WIDE;
    L.cur = S.wroot;
  }
}

__device__ __forceinline__ uint64_t stamp_cycles() {
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// One iteration of the node loop of bvh.cpp:245-312 / :331-388: visit node `cur` (both child
// boxes of an inner node, or every primitive of a leaf), then — if the visit produced no next
// node — make ONE pop attempt.  A closest-hit pop that is pruned (t >= best, bvh.cpp:303) leaves
// LF_POP set, so the next iteration tries the next entry; the visit order is exactly the
// reference's, only spread over iterations with uniform, short control flow.
//
// Memory: a lane visits either an inner node or a leaf, so one fetch serves both kinds of lanes.
// Every visiting lane loads four 16-B slots of its record (the 64-B node record, or the leaf's
// first 48-B primitive record plus the first slot of the second) and leaves of two or more
// primitives two more slots; then the wave waits ONCE and each lane computes on the same
// registers.  Without this a wave with lanes of both kinds paid two dependent round trips per
// iteration.  Primitives past the second (SAH leaves, bvh.cpp:193) are fetched in pairs after.
// LEAF1 (round 3; the path kernels' AA, Whitted, progressive and closest-chain modes, and the
// streaming kernel): a leaf's primitives one per step instead, through the same four shared loads,
// so that no load is issued for the few lanes holding a two-primitive leaf — the memory path
// pays a per-instruction floor (tools/td_lanes.hip): +1.4 % on the headline, +0.4 % on C3, though
// a leaf takes cnt steps.  (Round 1 measured one primitive per step 3 % slower, before the shared
// node / leaf fetch.)
// KIND: 0 = the query kind is the lane's LF_SHADOW flag (path kernels), 1 = closest-hit only,
// 2 = shadow only (the streaming traversal kernel's specialisations).
// WIDE (path kernels with shadow queries, the streaming shadow kernel): lanes flagged LF_WIDE walk
// the 4-ary shadow tree (drt_layout.hpp) — a wide record in the same four shared slot loads, its
// four child boxes tested at once, the nearest hit child next and the others pushed — and an
// in-range primitive hit becomes LF_VERIFY: the next step loads that primitive's exact reference
// leaf box through the same shared loads and accepts the hit only if the box is hit
// (boundingBox.cpp:64-124), else the leaf is dropped and the walk goes on.
// UNI (the streaming kernel's shadow queries): when the visiting lanes' record is the first visiting
// lane's — a wave's queries come from consecutive samples of one pixel toward one light point, so their
// walks coincide for long stretches — those lanes read it through one scalar load (the scalar cache)
// instead of per-lane vector loads on the vector-memory path the kernel is bound by.
// GV (round 6, the Grid scene's shadow queries on a shadow tree; trace_stream GV): the tree is
// collapsed from a BVH of the Grid scene's objects with every child box widened (drt_upload_grid_shadow_bvh),
// a primitive hit counts when t < range (grid.cpp:340), and instead of the leaf's box the hit is checked
// against the Grid: the ray's point at that t must lie inside a cell of the primitive's cell range,
// away from every cell face by more than the DDA's rounding (grid_certificate).  A certified hit is
// one Grid::Traverse(Ray&) would find; an uncertified one leaves the query to the Grid walk (LF_GVFB).
template <bool TRI_ONLY, bool STATS, int CAP, int KIND = 0, int LEAF1 = 1, bool WIDE = false, bool UNI = false,
          bool GV = false, class LaneT>
__device__ __forceinline__ void node_step(const SceneArgs& S, LaneT& L, LdsByte* lds, uint32_t* ov_desc,
                                          float* ov_t, bool wave_finite, Counters& C, uint64_t& cyc_leaf) {
  constexpr uint32_t kLdsBytes = (uint32_t)CAP * kRowBytes;  // desc part; the t part follows
  uint32_t fl = L.fl;
  const bool shadow = KIND == 0 ? (fl & LF_SHADOW) != 0u : KIND == 2;
  const bool wide = WIDE && (fl & LF_WIDE) != 0u;
  const uint32_t cur = L.cur;
  const bool visit = !(fl & LF_POP);
  const bool verify = WIDE && visit && (fl & LF_VERIFY) != 0u;
  const bool inner = visit && !verify && !desc_is_leaf(cur);
  const bool leaf = visit && !verify && desc_is_leaf(cur);
  uint32_t first = desc_first(cur), cnt = desc_count(cur);
  const bool big = leaf && cnt == kBigLeaf;
  // LEAF1 1 / 2: one primitive of a leaf per step (below), 2 also leaving the last slot unread for
  // such a step; 0: the whole leaf in the step
  const bool whole = LEAF1 == 0 || big;
  if (big) {  // oversized leaf: (first, count) from the side table
    const uint2 bl = S.big_leaves[first];
    first = bl.x;
    cnt = bl.y;
  }
  // (a shadow-tree node record is 4 slots, 8 for the 8-ary tree of -DDRT_WIDE8)
  const float4* rec = leaf ? S.prims + 3 * (size_t)first
                           : (verify ? S.wleaf + 2 * (size_t)cur
                                     : (wide ? S.wnodes + (size_t)(kWideK == 8 ? 8 : 4) * cur : S.nodes + 4 * (size_t)cur));
  float4 s0, s1, s2, s3, s4, s5;
  bool uni_done = false;
  if (UNI && visit) {
    const uint64_t ra = (uint64_t)(uintptr_t)rec;
    const uint64_t r0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(ra >> 32)) << 32) |
                        (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)ra);
    if (ra == r0) {  // the first visiting lane's record: one scalar 64-B load serves these lanes
      typedef const __attribute__((address_space(4))) uint32_t CU;
      CU* p = (CU*)(const void*)(uintptr_t)r0;
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; k++) w[k] = p[k];
      __builtin_memcpy(&s0, w, 16);
      __builtin_memcpy(&s1, w + 4, 16);
      __builtin_memcpy(&s2, w + 8, 16);
      __builtin_memcpy(&s3, w + 12, 16);
      uni_done = true;
    }
  }
  if (visit && !uni_done) {
    s0 = rec[0];
    s1 = rec[1];
    s2 = rec[2];
    // (Measured alternative, kept out: an 8-B load of the last slot for inner nodes, which use
    // only its two child descriptors: the split into two masked loads cost 8.6 %.)
    // The last slot serves inner nodes (child descriptors) and whole-leaf steps (the second
    // primitive's first slot); a one-primitive leaf step does not read it (LEAF1 2: +1.3 % on the
    // headline; the closest-chain pass of in-order frames lost 1.5 % with it and keeps 1).
    if (LEAF1 != 2 || inner || whole) s3 = rec[3];
  }
  if ((leaf && whole && cnt > 1) || (kWideK == 8 && WIDE && inner && wide)) {  // (8-ary node: its descriptors)
    s4 = rec[4];
    s5 = rec[5];
  }
  // (Measured alternative, kept out (round 3): the quad-cooperative fetch — the 4 lanes of a quad
  // load each other's records one 64-B segment per load instruction and transpose them with DPP
  // quad_perm; tools/gather_ceiling.hip variant `quad_coop`.  1.37x the per-lane gather rate from
  // an L1-resident table in isolation, but the path kernel ran 1 068 against 1 736 Mrays/s and the
  // streaming traversal kernel 0.65-0.78x: the transpose's ~50 VALU and DPP hazards sit on each
  // step's load -> test -> next-address chain, and the step must run with the whole wave active.)
  if (WIDE && inner && wide) {
    if (STATS) C.v[ST_W_INNER]++;
    // Child boxes decoded exactly (p + q * 2^E is a float, drt_layout.hpp) and tested with the
    // reference's sign-selected slabs (boundingBox.cpp:69-101; the ray is finite): each decoded box
    // contains the child's reference box, and the slab values are monotone in the planes, so a ray
    // that hits a reference box hits its decoded box.  The near / far plane bytes of all four
    // children are selected per axis at once.
    const uint32_t eb = __float_as_uint(s0.w);
    const float scx = __uint_as_float((eb & 0xffu) << 23), scy = __uint_as_float(((eb >> 8) & 0xffu) << 23),
                scz = __uint_as_float(((eb >> 16) & 0xffu) << 23);
    const bool px = L.q.sx(), py = L.q.sy(), pz = L.q.sz();
    // per axis the near / far plane bytes of every child (byte k & 3 of word k >> 2 is child k)
    uint32_t nx[kWideW], fx[kWideW], ny[kWideW], fy[kWideW], nz[kWideW], fz[kWideW];
    uint32_t d[kWideK];
    if constexpr (kWideK == 4) {
      const uint32_t lx = __float_as_uint(s1.x), hx = __float_as_uint(s1.y), ly = __float_as_uint(s1.z),
                     hy = __float_as_uint(s1.w), lz = __float_as_uint(s2.x), hz = __float_as_uint(s2.y);
      nx[0] = px ? lx : hx; fx[0] = px ? hx : lx;
      ny[0] = py ? ly : hy; fy[0] = py ? hy : ly;
      nz[0] = pz ? lz : hz; fz[0] = pz ? hz : lz;
      d[0] = __float_as_uint(s3.x); d[1] = __float_as_uint(s3.y); d[2] = __float_as_uint(s3.z); d[3] = __float_as_uint(s3.w);
    } else {  // 8-ary record: s1 / s2 / s3 = (lo w0, lo w1, hi w0, hi w1) of x / y / z, s4 / s5 the descriptors
      const float4 q3[3] = {s1, s2, s3};
      const bool pp[3] = {px, py, pz};
      uint32_t* nn[3] = {nx, ny, nz};
      uint32_t* ff[3] = {fx, fy, fz};
#pragma unroll
      for (int a = 0; a < 3; a++) {
        const uint32_t l0 = __float_as_uint(q3[a].x), l1 = __float_as_uint(q3[a].y), h0 = __float_as_uint(q3[a].z),
                       h1 = __float_as_uint(q3[a].w);
        nn[a][0] = pp[a] ? l0 : h0; nn[a][1] = pp[a] ? l1 : h1;
        ff[a][0] = pp[a] ? h0 : l0; ff[a][1] = pp[a] ? h1 : l1;
      }
      d[0] = __float_as_uint(s4.x); d[1] = __float_as_uint(s4.y); d[2] = __float_as_uint(s4.z); d[3] = __float_as_uint(s4.w);
      d[4] = __float_as_uint(s5.x); d[5] = __float_as_uint(s5.y); d[6] = __float_as_uint(s5.z); d[7] = __float_as_uint(s5.w);
    }
    float tn[kWideK];
    bool hk[kWideK];
#ifdef DRT_WIDE_PK
    static_assert(kWideK == 4, "packed decode: 4-ary records");
    // two children per packed-f32 instruction (v_pk_fma / v_pk_add / v_pk_mul): the same roundings
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v ox2 = {L.q.o.x, L.q.o.x}, oy2 = {L.q.o.y, L.q.o.y}, oz2 = {L.q.o.z, L.q.o.z};
    const f2v ix2 = {L.q.ix, L.q.ix}, iy2 = {L.q.iy, L.q.iy}, iz2 = {L.q.iz, L.q.iz};
    const f2v sx2 = {scx, scx}, sy2 = {scy, scy}, sz2 = {scz, scz};
    const f2v px2 = {s0.x, s0.x}, py2 = {s0.y, s0.y}, pz2 = {s0.z, s0.z};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int a = 16 * h, b = 16 * h + 8;
      auto dq = [&](uint32_t w) { return f2v{(float)((w >> a) & 0xffu), (float)((w >> b) & 0xffu)}; };
      const f2v tnx = (__builtin_elementwise_fma(dq(nx[0]), sx2, px2) - ox2) * ix2;
      const f2v tfx = (__builtin_elementwise_fma(dq(fx[0]), sx2, px2) - ox2) * ix2;
      const f2v tny = (__builtin_elementwise_fma(dq(ny[0]), sy2, py2) - oy2) * iy2;
      const f2v tfy = (__builtin_elementwise_fma(dq(fy[0]), sy2, py2) - oy2) * iy2;
      const f2v tnz = (__builtin_elementwise_fma(dq(nz[0]), sz2, pz2) - oz2) * iz2;
      const f2v tfz = (__builtin_elementwise_fma(dq(fz[0]), sz2, pz2) - oz2) * iz2;
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const float t0 = fmaxf(fmaxf(tnx[j], tny[j]), tnz[j]), t1 = fminf(fminf(tfx[j], tfy[j]), tfz[j]);
        hk[2 * h + j] = fmaxf(t0, 0.0f) < t1;
        tn[2 * h + j] = t0;
      }
    }
#elif defined(DRT_WIDE_FMA1)
    // (A/B, round 5; kept out) each plane as ONE fma, t = q * S + B with B = (p - o) * inv and S = 2^E * inv per axis
    // and node, instead of (fma(q, 2^E, p) - o) * inv (two more VALU per plane, 48 per node).  The
    // value is not the reference arithmetic's on the decoded plane, so the test is widened by a
    // bound on the difference: with M = max over axes of |B| + 255 |S| >= every |t| of
    // the node, both computations are within 5.0003 eps M of the exact real (P - o) * inv (eps =
    // 2^-24: B rounds twice, the fma once; the reference arithmetic twice), so testing
    // max(t0, 0) < t1 + 2D with 2D = 2^-20 M (+ 2^-99 for results near underflow, where |S| may have
    // lost bits) accepts every child the reference arithmetic accepts on the decoded box, hence
    // every child whose reference box the ray hits.  The extra children it may accept are ones the
    // exact decode rejected by < 1e-6 of their distance; the leaf-box check (LF_VERIFY) keeps the
    // answer exact.  Only lanes with |inv| <= 2^40 and |o| <= 2^60 walk the shadow tree
    // (wide_ray_ok), and build_wide keeps |p| <= 2^60 and 2^E <= 2^50, so nothing here overflows.
    const float Bx = (s0.x - L.q.o.x) * L.q.ix, By = (s0.y - L.q.o.y) * L.q.iy, Bz = (s0.z - L.q.o.z) * L.q.iz;
    const float Sx = scx * L.q.ix, Sy = scy * L.q.iy, Sz = scz * L.q.iz;
    const float M = fmaxf(fmaxf(__builtin_fmaf(255.0f, fabsf(Sx), fabsf(Bx)), __builtin_fmaf(255.0f, fabsf(Sy), fabsf(By))),
                          __builtin_fmaf(255.0f, fabsf(Sz), fabsf(Bz)));
    const float D2 = __builtin_fmaf(M, 0x1p-20f, 0x1p-99f);
#pragma unroll
    for (int k = 0; k < kWideK; k++) {
      const int w = k >> 2, sh = 8 * (k & 3);
      const float tnx = __builtin_fmaf((float)((nx[w] >> sh) & 0xffu), Sx, Bx);
      const float tfx = __builtin_fmaf((float)((fx[w] >> sh) & 0xffu), Sx, Bx);
      const float tny = __builtin_fmaf((float)((ny[w] >> sh) & 0xffu), Sy, By);
      const float tfy = __builtin_fmaf((float)((fy[w] >> sh) & 0xffu), Sy, By);
      const float tnz = __builtin_fmaf((float)((nz[w] >> sh) & 0xffu), Sz, Bz);
      const float tfz = __builtin_fmaf((float)((fz[w] >> sh) & 0xffu), Sz, Bz);
      const float t0 = fmaxf(fmaxf(tnx, tny), tnz), t1 = fminf(fminf(tfx, tfy), tfz);
      hk[k] = fmaxf(t0, 0.0f) < t1 + D2;
      tn[k] = t0;
    }
#else  // the reference arithmetic on the decoded planes
#pragma unroll
    for (int k = 0; k < kWideK; k++) {
      const int w = k >> 2, sh = 8 * (k & 3);
      const float tnx = (__builtin_fmaf((float)((nx[w] >> sh) & 0xffu), scx, s0.x) - L.q.o.x) * L.q.ix;
      const float tfx = (__builtin_fmaf((float)((fx[w] >> sh) & 0xffu), scx, s0.x) - L.q.o.x) * L.q.ix;
      const float tny = (__builtin_fmaf((float)((ny[w] >> sh) & 0xffu), scy, s0.y) - L.q.o.y) * L.q.iy;
      const float tfy = (__builtin_fmaf((float)((fy[w] >> sh) & 0xffu), scy, s0.y) - L.q.o.y) * L.q.iy;
      const float tnz = (__builtin_fmaf((float)((nz[w] >> sh) & 0xffu), scz, s0.z) - L.q.o.z) * L.q.iz;
      const float tfz = (__builtin_fmaf((float)((fz[w] >> sh) & 0xffu), scz, s0.z) - L.q.o.z) * L.q.iz;
      const float t0 = fmaxf(fmaxf(tnx, tny), tnz), t1 = fminf(fminf(tfx, tfy), tfz);
      hk[k] = fmaxf(t0, 0.0f) < t1;  // t0 < t1 && t1 > 0
      tn[k] = t0;
    }
#endif
    // go on with the first hit child (any order gives the same answer); push the others.  Nearest-
    // first order (the reference's rule for its two children) measured 1.6 % / 3.1 % slower on the
    // headline / C3 replay pass than this first-hit order (profiles/r04_replay_tuning_ab.jsonl).
    int ci = -1;
    float best = 0.0f;
#pragma unroll
    for (int k = 0; k < kWideK; k++) {
#ifdef DRT_WIDE_NEAREST  // (A/B) the hit child entered first
      const bool take = hk[k] && (ci < 0 || tn[k] < best);
#else
      const bool take = hk[k] && ci < 0;
#endif
      ci = take ? k : ci;
      best = take ? tn[k] : best;
    }
    constexpr uint32_t kWideLds = 2u * kLdsBytes;  // a shadow-tree stack uses the t rows too
    uint32_t spa = L.spa;
    // pushed in reverse, so that the pops go on in slot order: with the slots in ascending box
    // surface (build_wide, DRT_WIDE_ORDER 2) a lane enters its hit children smallest first.  Measured
    // on the headline: 1 956 against 1 929-1 931 Mrays/s for the build order with pushes in slot
    // order; 1 947 with ascending slots pushed in slot order, 1 951-1 953 descending and reversed
    // (profiles/r04_wide_order_push_ab.jsonl).
#pragma unroll
    for (int k = kWideK - 1; k >= 0; k--) {
      if (hk[k] && k != ci) {
        if (spa < kWideLds) *(LdsU32*)(lds + spa) = d[k];
        else ov_desc[(spa - kWideLds) >> kRowShift] = d[k];
        if (STATS) {
          C.v[ST_PUSH]++;
          if (spa >= kWideLds) C.v[ST_PUSH_SPILL]++;
        }
        spa += kRowBytes;
      }
    }
    L.spa = spa;
    uint32_t nxt = d[0];
#pragma unroll
    for (int k = 1; k < kWideK; k++) nxt = ci == k ? d[k] : nxt;
    L.cur = nxt;
    fl |= ci < 0 ? LF_POP : 0u;
  }
  if (WIDE && verify) {  // the exact reference leaf box of primitive `cur`, hit within range
    if (STATS) C.v[ST_W_VERIFY]++;
    fl &= ~LF_VERIFY;
    if constexpr (GV) {  // s0, s1: the primitive's cell range (grid_certificate)
      const bool in = grid_certificate(S, L.q, L.best_t, s0, s1);
      fl = (fl | (in ? LF_HIT : LF_GVFB)) & ~LF_TRAV;
    } else {
      float tv;
      const bool in = box_test_finite(s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, L.q, tv);
      fl = in ? ((fl | LF_HIT) & ~LF_TRAV) : (fl | LF_POP);
    }
  }
  if (inner && !wide) {
    if (STATS) C.v[shadow ? ST_S_INNER : ST_C_INNER]++;
    const float4 a = s0, b = s1, c = s2;
    const uint4 d = make_uint4(__float_as_uint(s3.x), __float_as_uint(s3.y), 0u, 0u);
    float tL, tR;
    bool hL, hR;
    if (wave_finite) {
      hL = box_test_finite(a.x, a.y, a.z, a.w, b.x, b.y, L.q, tL);
      hR = box_test_finite(b.z, b.w, c.x, c.y, c.z, c.w, L.q, tR);
    } else {
      hL = box_hit(a.x, a.y, a.z, a.w, b.x, b.y, L.q, tL);
      hR = box_hit(b.z, b.w, c.x, c.y, c.z, c.w, L.q, tR);
      if (box_inside(a.x, a.y, a.z, a.w, b.x, b.y, L.q.o)) tL = 0.0f;
      if (box_inside(b.z, b.w, c.x, c.y, c.z, c.w, L.q.o)) tR = 0.0f;
    }
    const bool both = hL && hR;
    // shadow: tL <= tR, closest: tL < tR (bvh.cpp:262 / :344).  Only consulted when both boxes
    // are hit, and then tL, tR are non-NaN and >= 0 (or -0), so they order as sign-cleared
    // integers and `<=` is `< + 1`.
    const uint32_t uL = __float_as_uint(tL) & 0x7fffffffu, uR = __float_as_uint(tR) & 0x7fffffffu;
    const bool left_first = uL < uR + (KIND == 0 ? (fl & LF_SHADOW) : (KIND == 2 ? 1u : 0u));
    L.cur = (hL && (left_first || !hR)) ? d.x : d.y;
    fl |= (hL | hR) ? 0u : LF_POP;
    // push the far child (bvh.cpp:268-283); the LDS slot above the top is free, so the store
    // is unconditional and only the stack pointer depends on `both`
    const uint32_t pd = left_first ? d.y : d.x;
    const float pt = left_first ? tR : tL;
    const uint32_t spa = L.spa;
    if (spa < kLdsBytes) {
      *(LdsU32*)(lds + spa) = pd;
      *(LdsF32*)(lds + kLdsBytes + spa) = pt;
    } else if (both) {
      ov_desc[(spa >> kRowShift) - CAP] = pd;
      ov_t[(spa >> kRowShift) - CAP] = pt;
    }
    L.spa = spa + (both ? kRowBytes : 0u);
    if (STATS && both) {
      C.v[ST_PUSH]++;
      if (spa >= kLdsBytes) C.v[ST_PUSH_SPILL]++;
    }
  }
  uint64_t t0 = 0;
  if (STATS) {
    t0 = stamp_cycles();
    if (__ballot(leaf) != 0 && (threadIdx.x & 63u) == 0) C.v[ST_WAVE_LEAF_ITERS]++;
  }
  if (leaf) {
    if (STATS && !(fl & LF_LEAFCONT)) C.v[wide ? ST_W_LEAF : (shadow ? ST_S_LEAF : ST_C_LEAF)]++;
    bool done = false;  // shadow any-hit found (bvh.cpp:376-377)
    // leaf_test: one Object::hit of the leaf in order (bvh.cpp:287-295 / :370-378)
    auto leaf_test = [&](const float4& p0, const float4& p1, const float4& p2, uint32_t prim) {
      if (STATS) C.v[wide ? ST_W_PRIMS : (shadow ? ST_S_PRIMS : ST_C_PRIMS)]++;
      float t;
      if (hit_prim_rec<TRI_ONLY>(p0, p1, p2, L.q, t)) {
        if (shadow) {
          if (GV ? t < L.thr : t <= L.thr) {
            // shadow tree: the leaf was entered through a containing box; its exact box decides
            // (GV: the Grid cell certificate, at this t)
            if (wide) {
              fl |= LF_VERIFY;
              L.cur = prim;
              if (GV) L.best_t = t;
            } else {
              fl = (fl | LF_HIT) & ~LF_TRAV;
            }
            done = true;
          }
        } else if (t < L.best_t) {
          L.best_t = t;
          L.best_prim = prim;
          fl |= LF_HIT;
        }
      }
    };
    if (cnt > 0) leaf_test(s0, s1, s2, first);
    if (whole && !done && cnt > 1) leaf_test(s3, s4, s5, first + 1);
    const float4* pr = S.prims + 3 * (size_t)first;
    for (uint32_t i = 2; whole && !done && i < cnt; i += 2) {  // primitives in pairs, tested in order
      const bool two = i + 1 < cnt;
      const float4 p0 = pr[3 * i], p1 = pr[3 * i + 1], p2 = pr[3 * i + 2];
      float4 r0, r1, r2;
      if (two) {
        r0 = pr[3 * i + 3];
        r1 = pr[3 * i + 4];
        r2 = pr[3 * i + 5];
      }
      leaf_test(p0, p1, p2, first + i);
      if (!done && two) leaf_test(r0, r1, r2, first + i + 1);
    }
    // A leaf of up to 30 primitives goes on with its next primitive in the next step, whose shared
    // four loads fetch it with the other lanes' nodes: the rest of the leaf is itself a leaf
    // descriptor.  (The second primitive's two slots loaded beside the first, for the few lanes
    // with such a leaf, cost a load instruction each at a per-instruction floor: tools/td_lanes.hip.)
    const bool more = !whole && !done && cnt > 1;
    if (more) L.cur = leaf_desc(first + 1, cnt - 1);
    fl = more ? (fl | LF_LEAFCONT) : (fl & ~LF_LEAFCONT);
    if (!more && (fl & LF_TRAV) && !(WIDE && (fl & LF_VERIFY))) fl |= LF_POP;
  }
  if (STATS) cyc_leaf += stamp_cycles() - t0;
  if ((fl & (LF_POP | LF_TRAV)) == (LF_POP | LF_TRAV)) {  // bvh.cpp:299-311 / :381-387
    if (L.spa < kRowBytes) {
      fl &= ~LF_TRAV;
    } else {
      const uint32_t spa = L.spa - kRowBytes;
      L.spa = spa;
      uint32_t pd;
      float pt = 0.0f;
      // a shadow-tree lane's LDS stack spans the t rows too (it keeps no entry distances)
      if constexpr (!WIDE) {  // binary lanes only: the round-3 pop (measured 1 769 against 1 757 Mrays/s)
      if (spa < kLdsBytes) {
        pd = *(LdsU32*)(lds + spa);
        pt = *(LdsF32*)(lds + kLdsBytes + spa);
      } else {
        pd = ov_desc[(spa >> kRowShift) - CAP];
        pt = ov_t[(spa >> kRowShift) - CAP];
      }
      } else {
      const uint32_t lim = wide ? 2u * kLdsBytes : kLdsBytes;
      if (spa < lim) {
        pd = *(LdsU32*)(lds + spa);
        if (!shadow) pt = *(LdsF32*)(lds + kLdsBytes + spa);
      } else {
        pd = ov_desc[(spa - lim) >> kRowShift];
        pt = ov_t[(spa - lim) >> kRowShift];
      }
      }
      if (shadow || pt < L.best_t) {
        L.cur = pd;
        fl &= ~LF_POP;
      }
    }
  }
  L.fl = fl;
}

// Path-kernel modes whose shadow queries walk the 4-ary shadow tree (see the node loop).
// MODE_REPLAY: an in-order frame's replay (keyed-stream draws from recorded positions); MODE_AREPLAY:
// an AA / Whitted frame's replay (no draw after the prologue reaches the frame, so no RNG, DoF or
// stream positions in its code: L.rk holds the sample's closest-chain record instead)
template <int MODE>
constexpr bool kReplay = MODE == MODE_REPLAY || MODE == MODE_AREPLAY;
// passes that read their closest hits back (kReplay: refraction-free frames; MODE_TREPLAY: a hit tree)
template <int MODE>
constexpr bool kReadBack = kReplay<MODE> || MODE == MODE_TREPLAY;

template <int MODE>
constexpr bool kPathWide =
#ifdef DRT_PATH_WIDE
    MODE != MODE_SKEL;
#else
    kReadBack<MODE>;
#endif

template <bool STATS, int ACC, int MODE>
__device__ __forceinline__ void setup_shadow(const SceneArgs& S, const FrameArgs& F, Lane& L,
                                             Counters& C) {  // main.cpp:386-422
  const int li = light_of_pair(L.j, F);
  L.lightPos = light_point(tab<ACC>(S.lights, (uint32_t)li), L.ls, L.j - li * F.light_spp, F);
  V3 Lv = sub(L.lightPos, L.hitP);
  const V3 Ls = Lv;
  Lv = normalize(Lv);
  const V3 H = normalize(add(Lv, L.V));
  L.NdotL = smax(dot(L.N, Lv), 0.0f);
  L.NdotH = smax(dot(L.N, H), 0.0f);
  const V3 so = add(L.hitP, mul(L.N, 1e-4f));
  if (ACC == ACC_GRID)  // Grid::Traverse(Ray&) gets the unit L: range |L|, direction re-normalised (Q1)
    start_query<STATS, ACC>(S, L, make_ray(so, normalize(Lv)), true, length(Lv), C);
  else  // BVH::Traverse(Ray&) normalises Ls and accepts t <= |Ls| + EPSILON (bvh.cpp:321-322, :376)
    start_query<STATS, ACC, kPathWide<MODE>>(S, L, make_ray(so, normalize(Ls)), true, shadow_threshold(length(Ls)),
                                             C);
}

// reflectDir (main.cpp:504-508); MODE_SEQ draws rnd_unit_sphere on the lane's keyed stream
// exactly where the reference calls it, whatever the roughness (Q15)
template <int MODE>
__device__ __forceinline__ V3 reflect_dir(const FrameArgs& F, Lane& L, V3 N, V3 V) {
  V3 R = sub(mul(mul(N, dot(V, N)), 2.0f), V);
  if (MODE == MODE_SEQ || MODE == MODE_PROG || MODE == MODE_SKEL || MODE == MODE_REPLAY) {
    KRng rng{F.seed, L.pmix, L.rk};
    R = normalize(add(R, mul(rnd_unit_sphere(rng), F.roughness)));
    L.rk = rng.k;
    return R;
  }
  return normalize(R);
}

template <bool STATS, int MODE, int ACC>
__device__ void seq_start_sample(const SceneArgs& S, const FrameArgs& F, Lane& L, Counters& C);

// A closest-hit query of the path: traversed, or in MODE_REPLAY read back from pass 1's record of
// this sample and bounce (the lane is ready at once; pass 1 counted the traversal).
template <bool STATS, int MODE, int ACC>
__device__ __forceinline__ void closest_query(const SceneArgs& S, const FrameArgs& F, Lane& L, const RayP& q,
                                              Counters& C) {
  if (MODE == MODE_TREPLAY) {  // the sample's next closest hit, in the order pass 1 recorded them
    const uint2 h = F.skel_hits[L.rk++];
    L.q = q;
    L.best_t = __uint_as_float(h.x);
    L.best_prim = h.y;
    L.fl = (L.fl & LF_OUTSIDE) | (h.y != 0xFFFFFFFFu ? LF_HIT : 0u);
    return;
  }
  if (kReplay<MODE>) {
    // an AA / Whitted frame's replay keeps its record index in L.rk (lane_init; a Whitted frame's
    // light samples share their pixel's record, FrameArgs::chain_div), an in-order frame's is the item
    const uint32_t rec = MODE == MODE_AREPLAY ? L.rk : L.item;
    const uint2 h = F.skel_hits[(size_t)rec * (uint32_t)(F.max_depth + 1) + (uint32_t)(L.depth - 1)];
    L.q = q;
    L.best_t = __uint_as_float(h.x);
    L.best_prim = h.y;
    L.fl = (L.fl & LF_OUTSIDE) | (h.y != 0xFFFFFFFFu ? LF_HIT : 0u);
    return;
  }
  start_query<STATS, ACC>(S, L, q, false, 0.0f, C);
}

// The persistent kernel's rayTracing() call frames, split by what the unwind reads back
// (main.cpp:489-520).  Every parent needs the head: its accumulated colour, kr, material and
// flags — all a mirror-only parent (no refraction child) reads when its reflection child
// returns.  Only a parent with a refraction child keeps the tail: the hit point, normal and
// view vector for the reflection ray it traces after that child, its light position and ior,
// and the Beer factor.  Mirror bounces, the common case, so store 24 B instead of 88.
struct FrameHead {
  V3 acc;
  float kr;
  uint32_t mat;
  uint32_t flags;  // bit0: in reflection child, bit1: outside, bit2: has reflection, bit3: reflectDir.N > 0
};
struct FrameTail {
  V3 hitP, N, V, lightPos, beer;
  float ior1;
};
struct FrameStack {
  FrameHead h[kMaxFrames];
  FrameTail t[kMaxFrames];
};

// Round 5: the in-order frames' replay pass (no refraction: every parent is a mirror parent) keeps its
// frame heads in global memory, each lane's run of max_depth + 1 heads contiguous (FrameArgs::heads),
// one 16-B record per frame: (acc, material | flags << 24).  The private FrameStack is lane-interleaved
// scratch: a 24-B head store by a lane of a partly active shading wave wrote six partly filled sectors
// (C4: 76 GB of the replay pass's writes per frame).  -DDRT_HEADS_SCRATCH keeps the FrameStack (A/B).
template <int MODE, int ACC>
constexpr bool kReplayHeads =
#ifdef DRT_HEADS_SCRATCH
    false;
#else
    // the in-order frames' replay (C4: replay writes 70.0 -> 37.3 GB per frame, same speed); the AA /
    // Whitted replay measured 0.6 % faster with the scratch FrameStack on the headline (1 969-1 977
    // against 1 964-1 966 Mrays/s; its writes 10.7 against 5.5 GB), and the Grid's 7 % faster (28
    // against 50 VGPR spills; profiles/r05_ab_*)
    MODE == MODE_REPLAY && ACC == ACC_BVH;
#endif
__device__ __forceinline__ float4* replay_head(const FrameArgs& F, uint32_t fsp) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  return F.heads + (size_t)lane * (uint32_t)(F.max_depth + 1) + fsp;
}

// MODE_SEQ tail: hand the rest of the lane's pixel (next sample L.smp, keyed-stream position
// L.rk) to another wave through a continuation slot.  One 64-bit word per slot, written and read
// with agent-scope atomics, so no other store has to be ordered before it.  False (the lane goes
// on itself) when the state does not fit the word or the slots are used up.
__device__ __forceinline__ bool seq_donate(const FrameArgs& F, const Lane& L) {
  if (L.smp >= (1u << 12) || L.rk >= (1u << 20)) return false;
  if (F.seq_backlog) {  // keep the pixel while this many handed-over pixels still wait for a lane
    const unsigned long long pp = __hip_atomic_load((unsigned long long*)(F.work_counter + kSeqPush), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)pp - (uint32_t)(pp >> 32) >= F.seq_backlog) return false;
  }
  const uint32_t idx = atomicAdd(F.work_counter + kSeqPush, 1u);
  if (idx >= F.seq_cap) return false;
  const unsigned long long v = (unsigned long long)L.item | ((unsigned long long)(L.smp | (L.rk << 12)) << 32);
  __hip_atomic_store(F.seq_cont + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// rayTracing(depth = 1) returned c: store the sample; MODE_SEQ lanes go on with the pixel's next
// sample on the same stream (or, in a wave handing its pixels over, leave it to another lane).
template <bool STATS, int MODE, int ACC>
__device__ __forceinline__ void finish_sample(const SceneArgs& S, const FrameArgs& F, Lane& L, Counters& C, V3 c) {
  if (MODE == MODE_SEQ) {  // sample smp of the lane's pixel is done: next sample, same stream
    if (!(L.fl & LF_RESUME)) F.samples[(size_t)L.item * F.nsub + L.smp] = make_float4(c.x, c.y, c.z, 0.0f);
    if (++L.smp < (uint32_t)F.nsub) {
      if ((L.fl & LF_YIELD) && seq_donate(F, L)) {
        L.item = kNoItem;
        return;
      }
      seq_start_sample<STATS, MODE, ACC>(S, F, L, C);
      return;
    }
    if (F.seq_cont) atomicAdd(F.work_counter + kSeqDone, 1u);
    L.item = kNoItem;
    return;
  }
  if (MODE != MODE_TCHAIN) F.samples[L.item] = make_float4(c.x, c.y, c.z, 0.0f);  // (pass 2 writes it)
  L.item = kNoItem;
}

// Consume the completed query of lane L (main.cpp:294-521 between two traversals).
template <bool STATS, int MODE, int ACC>
__device__ void lane_process(const SceneArgs& S, const FrameArgs& F, Lane& L, FrameStack& fs, Counters& C) {
#ifdef DRT_REPLAY_CHAIN
again:  // (A/B) the replay pass shades a read-back closest hit at once instead of in the next pass:
        // VGPR spills 45 -> 57 and 2x slower frames (headline 992 against 1 929 Mrays/s)
#endif
  const float offset = 1e-4f;
  V3 c = mk(0, 0, 0);
  bool after_lights = false;
  const bool hit = (L.fl & LF_HIT) != 0u;
  if (MODE == MODE_TCHAIN && !(L.fl & LF_SHADOW))  // pass 1 of a refracting frame: record the hit
    F.skel_hits[L.rk++] = make_uint2(__float_as_uint(L.best_t), hit ? L.best_prim : 0xFFFFFFFFu);
  if (MODE == MODE_SEQ && (L.fl & LF_RESUME)) {
    // a handed-over pixel: no query result to consume, straight to finish_sample (fsp is 0)
  } else if (!(L.fl & LF_SHADOW)) {
    if (!hit) {  // main.cpp:351-357 (pass 1 of a refracting frame: its colours are pass 2's)
      c = MODE == MODE_TCHAIN ? mk(0.f, 0.f, 0.f) : cclamp(background(S, L.q.d));
    } else {
      L.hitT = L.best_t;
      L.hitPrim = L.best_prim;
      L.hitP = add(L.q.o, mul(L.q.d, L.hitT));
      L.N = normalize(prim_normal(S.prims, L.hitPrim, L.q, L.hitT));
      const bool outside = dot(L.q.d, L.N) < 0.0f;
      if (!outside) L.N = neg(L.N);
      L.fl = outside ? (L.fl | LF_OUTSIDE) : (L.fl & ~LF_OUTSIDE);
      L.mat = prim_material(S.prims[3 * L.hitPrim]);
      L.V = neg(normalize(L.q.d));
      L.acc = mk(0, 0, 0);
      L.lightPos = mk(0, 0, 0);
      L.j = 0;
      if (MODE != MODE_TCHAIN && S.n_lights > 0) {  // (pass 1 of a refracting frame: no shadow rays)
        setup_shadow<STATS, ACC, MODE>(S, F, L, C);
        return;
      }
      after_lights = true;
    }
  } else {  // main.cpp:444-450
    if (!hit)
      L.acc = add(L.acc, light_term(tab<ACC>(S.mats, L.mat), L.NdotL, L.NdotH, tab<ACC>(S.lights, (uint32_t)light_of_pair(L.j, F)), F));
    L.j = next_light_pair(S, F, L.j);
    if (L.j < S.n_lights * F.light_spp) {
      setup_shadow<STATS, ACC, MODE>(S, F, L, C);
      return;
    }
    after_lights = true;
  }
  if (after_lights) {  // main.cpp:453-520
    const drt_material& m = tab<ACC>(S.mats, L.mat);
    const bool outside = (L.fl & LF_OUTSIDE) != 0u;
    if (L.depth > F.max_depth) {
      c = L.acc;
    } else {
      float kr = m.refl;
      float ior2 = m.ior;
      if (!outside) ior2 = 1.0f;
      const float eta = L.ior1 / ior2;
      const V3 Vt = sub(mul(L.N, dot(L.V, L.N)), L.V);
      const float sin_i = length(Vt);
      const V3 tv = dvf(Vt, length(Vt));
      const float sin_t = eta * sin_i;
      // MODE_REPLAY frames have no refracting material (the two-pass plan's condition): no refraction
      // child, Fresnel or Beer code and no frame tails in that instantiation
      const bool has_refr = !kReplay<MODE> && (m.trans == 1.0f && sin_t < 1.0f);
      const bool has_refl = m.ks > 0.0f;
      V3 beer = mk(1.f, 1.f, 1.f);
      RayP child = L.q;
      float child_ior = L.ior1;
      if (has_refr) {
        const float sin_t2 = (float)((double)sin_t * (double)sin_t);
        const float cos_t = sqrtf(1.0f - sin_t2);
        const V3 r_t = normalize(add(mul(tv, sin_t), mul(neg(L.N), cos_t)));
        const float cos_i = dot(L.N, L.V);
        const float cosTheta = (L.ior1 > ior2) ? cos_t : cos_i;
        float r0 = (L.ior1 - ior2) / (L.ior1 + ior2);
        r0 = (float)((double)r0 * (double)r0);
        kr = (float)((double)r0 + (double)(1.0f - r0) * pow((double)(1.0f - cosTheta), 5.0));
        if (!outside) {
          const V3 e = mul(sub(mk(1.f, 1.f, 1.f), ld3(m.diff)), -L.hitT);
          beer = mk(expf(e.x), expf(e.y), expf(e.z));
        }
        child = make_ray(sub(L.hitP, mul(L.N, offset)), r_t);
        child_ior = ior2;
      } else if (m.trans > 0.0f && sin_t >= 1.0f) {
        kr = 1.0f;
      }
      if (kReplayHeads<MODE, ACC> && has_refl) {
        // a replay's frame head: one 16-B store to the lane's own run (replay_head), kr rebuilt from
        // the material and bit 4 at the unwind
        const V3 R = reflect_dir<MODE>(F, L, L.N, L.V);
        const uint32_t flags = 1u | (outside ? 2u : 0u) | 4u | (dot(R, L.N) > 0.0f ? 8u : 0u) | (kr == 1.0f && m.refl != 1.0f ? 16u : 0u);
        *replay_head(F, L.fsp) = make_float4(L.acc.x, L.acc.y, L.acc.z, __uint_as_float(L.mat | (flags << 24)));
        L.fsp++;
        L.ls = L.lightPos;
        L.depth++;
        closest_query<STATS, MODE, ACC>(S, F, L, make_ray(add(L.hitP, mul(L.N, offset)), R), C);
        return;
      }
      if (!kReplayHeads<MODE, ACC> && (has_refr || has_refl)) {
        FrameHead& f = fs.h[L.fsp];
        f.acc = L.acc; f.kr = kr; f.mat = L.mat;
        uint32_t flags = (has_refr ? 0u : 1u) | (outside ? 2u : 0u) | (has_refl ? 4u : 0u);
        if (has_refr) {  // the refraction child runs first; the tail serves the unwind after it
          FrameTail& ft = fs.t[L.fsp];
          ft.hitP = L.hitP; ft.N = L.N; ft.V = L.V; ft.lightPos = L.lightPos; ft.beer = beer; ft.ior1 = L.ior1;
        } else {
          const V3 R = reflect_dir<MODE>(F, L, L.N, L.V);
          if (dot(R, L.N) > 0.0f) flags |= 8u;
          child = make_ray(add(L.hitP, mul(L.N, offset)), R);
          child_ior = L.ior1;
        }
        f.flags = flags;
        L.fsp++;
        L.ior1 = child_ior;
        L.ls = L.lightPos;
        L.depth++;
        closest_query<STATS, MODE, ACC>(S, F, L, child, C);
#ifdef DRT_REPLAY_CHAIN
        if (kReplay<MODE>) goto again;
#endif
        return;
      }
      c = cclamp(L.acc);
    }
  }
  // unwind: c is the return value of the current rayTracing() call.  A frame that is popped is
  // only read (its sum lives in registers); the one store is the acc/flags of a parent that
  // continues with its reflection child.  The Grid stepper keeps the store-through form (each
  // frame updated in place): with the register-only form its allocation changed, 605 -> 510
  // Mrays/s, while the BVH kernel gained 1.5 %.
  if (kReplayHeads<MODE, ACC>) {  // a replay's frames: mirror parents only (main.cpp:513-518)
    while (L.fsp > 0) {
      const float4 h = *replay_head(F, L.fsp - 1);
      const uint32_t w = __float_as_uint(h.w), flags = w >> 24, mat = w & 0xffffffu;
      V3 acc = mk(h.x, h.y, h.z);
      if (flags & 8u) {
        const drt_material& mm = tab<ACC>(S.mats, mat);
        const float kr = (flags & 16u) ? 1.0f : mm.refl;
        acc = add(acc, cmulc(mul(cclamp(c), kr), ld3(mm.spec)));
      }
      c = cclamp(acc);
      L.fsp--;
    }
  }
  if (!kReplayHeads<MODE, ACC> && ACC == ACC_GRID) {
    while (L.fsp > 0) {
      FrameHead& f = fs.h[L.fsp - 1];
      if (!kReplay<MODE> && (f.flags & 1u) == 0u) {
        const FrameTail& ft = fs.t[L.fsp - 1];
        V3 rc = cclamp(c);
        if ((f.flags & 2u) == 0u) rc = cmulc(rc, ft.beer);
        f.acc = add(f.acc, mul(rc, 1.0f - f.kr));
        if (f.flags & 4u) {
          uint32_t flags = f.flags | 1u;
          const V3 R = reflect_dir<MODE>(F, L, ft.N, ft.V);
          if (dot(R, ft.N) > 0.0f) flags |= 8u;
          f.flags = flags;
          L.ior1 = ft.ior1;
          L.ls = ft.lightPos;
          L.depth = L.fsp + 1;
          closest_query<STATS, MODE, ACC>(S, F, L, make_ray(add(ft.hitP, mul(ft.N, offset)), R), C);
          return;
        }
        c = cclamp(f.acc);
        L.fsp--;
      } else {
        const V3 rc = cclamp(c);
        if (f.flags & 8u) f.acc = add(f.acc, cmulc(mul(rc, f.kr), ld3(tab<ACC>(S.mats, f.mat).spec)));
        c = cclamp(f.acc);
        L.fsp--;
      }
    }
  }
  while (!kReplayHeads<MODE, ACC> && ACC != ACC_GRID && L.fsp > 0) {
    FrameHead& f = fs.h[L.fsp - 1];
    const uint32_t flags = f.flags;
    V3 acc = f.acc;
    const float kr = f.kr;
    if (!kReplay<MODE> && (flags & 1u) == 0u) {  // refraction child returned (main.cpp:489-496)
      const FrameTail& ft = fs.t[L.fsp - 1];
      V3 rc = cclamp(c);
      if ((flags & 2u) == 0u) rc = cmulc(rc, ft.beer);
      acc = add(acc, mul(rc, 1.0f - kr));
      if (flags & 4u) {  // now the reflection child (main.cpp:503-512)
        const V3 R = reflect_dir<MODE>(F, L, ft.N, ft.V);
        f.acc = acc;
        f.flags = flags | 1u | (dot(R, ft.N) > 0.0f ? 8u : 0u);
        L.ior1 = ft.ior1;
        L.ls = ft.lightPos;
        L.depth = L.fsp + 1;
        closest_query<STATS, MODE, ACC>(S, F, L, make_ray(add(ft.hitP, mul(ft.N, offset)), R), C);
        return;
      }
    } else if (flags & 8u) {  // reflection child returned, reflectDir.N > 0 (main.cpp:513-518)
      acc = add(acc, cmulc(mul(cclamp(c), kr), ld3(tab<ACC>(S.mats, f.mat).spec)));
    }
    c = cclamp(acc);
    L.fsp--;
  }
  finish_sample<STATS, MODE, ACC>(S, F, L, C, c);
}

// ------------------------------------------------------------------------------------------
// Wavefront replay (round 5; drt_kernels.hpp WfArgs): pass 2 of a refraction-free two-pass frame as
// three launches — wf_gen, the shadow queries of the whole frame on the streaming kernel, wf_combine —
// instead of the persistent replay, whose waves interleave shading (a third of their lanes active) with
// the shadow traversal.  The arithmetic is lane_process's, in its order: setup_shadow's light point, ray
// and Phong factors per (level, light pair), the unshadowed terms added in pair order, the depth cut,
// and the mirror unwind.
// ------------------------------------------------------------------------------------------
enum : uint32_t { WF_MISS = 1u, WF_DEEP = 2u, WF_REFL = 4u, WF_RN = 8u, WF_KR1 = 16u };

__device__ __forceinline__ bool wf_pair_used(const SceneArgs& S, const FrameArgs& F, int j) {
  // the pairs next_light_pair visits: every quad-light pair, a point light's k = 0 only
  const int m = F.light_spp;
  return m == 1 || j % m == 0 || S.lights[j / m].type == DRT_LIGHT_QUAD;
}

// The wavefront's streaming buffers (query records, Phong factors, level records, answers) are written
// once and read once, between uses of the tree records.  -DDRT_WF_NT (A/B) moves them
// with non-temporal stores and loads, so that they do not displace tree records from the caches.
#ifdef DRT_WF_NT
typedef float wf_f4 __attribute__((ext_vector_type(4)));
typedef float wf_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void wf_st(float4* p, float4 v) { __builtin_nontemporal_store(wf_f4{v.x, v.y, v.z, v.w}, (wf_f4*)p); }
__device__ __forceinline__ void wf_st(float2* p, float2 v) { __builtin_nontemporal_store(wf_f2{v.x, v.y}, (wf_f2*)p); }
__device__ __forceinline__ void wf_st(uint8_t* p, uint8_t v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ float4 wf_ld(const float4* p) {
  const wf_f4 v = __builtin_nontemporal_load((const wf_f4*)p);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 wf_ld(const float2* p) {
  const wf_f2 v = __builtin_nontemporal_load((const wf_f2*)p);
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ uint8_t wf_ld(const uint8_t* p) { return __builtin_nontemporal_load(p); }
#else
template <class T>
__device__ __forceinline__ void wf_st(T* p, T v) { *p = v; }
template <class T>
__device__ __forceinline__ T wf_ld(const T* p) { return *p; }
#endif

// Query slot of (level l, pair u, chunk slot s): [band][level][pair][slot in band], a band being W.band
// consecutive sample slots, so that band b's queries are one contiguous range (the streaming kernels
// give XCD b that range first: its L2 then serves the rays of one screen band)
__device__ __forceinline__ size_t wf_q(const WfArgs& W, int l, int u, uint32_t s) {
  const uint32_t b = s / W.band, o = s - b * W.band;
  return (((size_t)b * (uint32_t)W.levels + (uint32_t)l) * (uint32_t)W.pairs + (uint32_t)u) * W.band + o;
}

// One level of a sample's recorded chain (wf_gen_kernel): a miss's background colour, or the hit's shadow queries — one per pair
// the light loop visits, with their Phong factors — and the level record (material, flags).  Returns
// whether the sample goes on with its mirror ray `next`; `ls` becomes the light sample it carries.
__device__ bool wf_level(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, uint32_t slot, int l, const RayP& q,
                         bool hit, float t, uint32_t prim, V3& ls, uint32_t pmix, uint32_t& rk, RayP& next) {
  const size_t li_ = (size_t)l * W.n_slots + slot;
  if (!hit) {  // main.cpp:351-357
    const V3 c = cclamp(background(S, q.d));
    wf_st(&W.lvl[li_], make_float4(c.x, c.y, c.z, __uint_as_float(WF_MISS << 24)));
    return false;
  }
  const V3 hitP = add(q.o, mul(q.d, t));
  V3 N = normalize(prim_normal(S.prims, prim, q, t));
  const bool outside = dot(q.d, N) < 0.0f;
  if (!outside) N = neg(N);
  const uint32_t mat = prim_material(S.prims[3 * prim]);
  const V3 V = neg(normalize(q.d));
  V3 lightPos = mk(0, 0, 0);
  for (int j = 0, u = 0; j < F.light_spp * S.n_lights; j++) {  // setup_shadow for every pair the light loop visits
    if (!wf_pair_used(S, F, j)) continue;
    const size_t qi = wf_q(W, l, u++, slot);
    const int li = light_of_pair(j, F);
    lightPos = light_point(S.lights[li], ls, j - li * F.light_spp, F);
    V3 Lv = sub(lightPos, hitP);
    const V3 Ls = Lv;
    Lv = normalize(Lv);
    const V3 H = normalize(add(Lv, V));
    const float NdotL = smax(dot(N, Lv), 0.0f), NdotH = smax(dot(N, H), 0.0f);
    const V3 so = add(hitP, mul(N, 1e-4f));
    // BVH::Traverse(Ray&) normalises Ls, range |Ls| + EPSILON; Grid::Traverse(Ray&) gets the unit L,
    // range |L|, direction re-normalised (Q1; setup_shadow)
    const V3 sd = W.grid ? normalize(Lv) : normalize(Ls);
    wf_st(&W.rays[qi], make_float4(so.x, so.y, so.z, W.grid ? length(Lv) : shadow_threshold(length(Ls))));
    wf_st(&W.rays_b[qi], make_float4(sd.x, sd.y, sd.z, 0.0f));
    wf_st(&W.nl[qi], make_float2(NdotL, NdotH));
  }
  uint32_t flags = 0u;
  bool more = false;
  if (l + 1 > F.max_depth) {  // depth > MAX_DEPTH: the accumulated colour, unclamped (main.cpp:454)
    flags = WF_DEEP;
  } else {
    const drt_material m = S.mats[mat];
    float kr = m.refl;
    float ior2 = m.ior;
    if (!outside) ior2 = 1.0f;
    const float eta = 1.0f / ior2;  // ior1: mirror children keep the camera's 1.0
    const V3 Vt = sub(mul(N, dot(V, N)), V);
    const float sin_t = eta * length(Vt);
    if (m.trans > 0.0f && sin_t >= 1.0f) kr = 1.0f;  // (trans == 1 never reaches a two-pass frame)
    if (m.ks > 0.0f) {  // reflectDir (reflect_dir)
      V3 R = sub(mul(mul(N, dot(V, N)), 2.0f), V);
      if (W.inorder) {
        KRng rng{F.seed, pmix, rk};
        R = normalize(add(R, mul(rnd_unit_sphere(rng), F.roughness)));
        rk = rng.k;
      } else {
        R = normalize(R);
      }
      flags = WF_REFL | (dot(R, N) > 0.0f ? WF_RN : 0u) | (kr == 1.0f && m.refl != 1.0f ? WF_KR1 : 0u);
      next = make_ray(add(hitP, mul(N, 1e-4f)), R);
      ls = lightPos;
      more = true;
    }
  }
  wf_st(&W.lvl[li_], make_float4(0.f, 0.f, 0.f, __uint_as_float(mat | (flags << 24))));
  return more;
}
#ifndef DRT_WF_PIECEWISE
// wf_level with every query store made by the whole wave (round 6; -DDRT_WF_PIECEWISE keeps the round-5
// wf_level + wf_mark_empty: wf_gen 3.09 against 2.57 ms, headline -0.9 %, C3 -1.9 %, C4 -2.5 %,
// profiles/r06_ab_wf_gen_fullwave.jsonl): a lane whose chain has ended
// (`live` false) or missed at this level stores the empty-slot marker (thr = -1) in the same store
// instruction as the lanes that store queries, so that each 128-B line of the query arrays is written
// whole by one instruction instead of in pieces by the level's stores and wf_mark_empty's; its
// direction and Phong factors are don't-care values.  The same queries, factors and level records.
__device__ bool wf_level_fw(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, uint32_t slot, int l,
                            const RayP& q, bool live, bool hit, float t, uint32_t prim, V3& ls, uint32_t pmix,
                            uint32_t& rk, RayP& next) {
  const size_t li_ = (size_t)l * W.n_slots + slot;
  if (live && !hit) {  // main.cpp:351-357
    const V3 c = cclamp(background(S, q.d));
    wf_st(&W.lvl[li_], make_float4(c.x, c.y, c.z, __uint_as_float(WF_MISS << 24)));
  }
  V3 hitP = mk(0, 0, 0), N = mk(0, 0, 1), V = mk(0, 0, 1);
  bool outside = true;
  uint32_t mat = 0;
  if (hit) {
    hitP = add(q.o, mul(q.d, t));
    N = normalize(prim_normal(S.prims, prim, q, t));
    outside = dot(q.d, N) < 0.0f;
    if (!outside) N = neg(N);
    mat = prim_material(S.prims[3 * prim]);
    V = neg(normalize(q.d));
  }
  V3 lightPos = mk(0, 0, 0);
  // compact queries (WfArgs::compact): this wave's 64 slots are one group; its lanes with a query at this
  // level take its first slots in lane order, and the group's count goes to W.cnt (by its lowest lane)
  uint32_t crank = 0;
  if (W.compact) {
    const uint64_t act = __ballot(true), hb = __ballot(hit);
    crank = __builtin_amdgcn_mbcnt_hi((uint32_t)(hb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hb, 0u));
    const uint32_t lo = (uint32_t)__builtin_ctzll(act), lane = threadIdx.x & 63u;
    if (lane == lo) {
      const uint32_t b = slot / W.band, g = (slot - b * W.band) >> 6;
      W.cnt[((size_t)b * (uint32_t)W.levels + (uint32_t)l) * (W.band >> 6) + g] = (uint8_t)__popcll(hb);
    }
  }
  for (int j = 0, u = 0; j < F.light_spp * S.n_lights; j++) {  // setup_shadow for every pair the light loop visits
    if (!wf_pair_used(S, F, j)) continue;
    const size_t qi = wf_q(W, l, u, slot);
    const size_t qc = wf_q(W, l, u, slot & ~63u) + crank;  // (compact) the query's packed slot
    u++;
    float4 ra = make_float4(0.f, 0.f, 0.f, -1.0f), rb = make_float4(0.f, 0.f, 0.f, 0.f);
    float2 nlv = make_float2(0.f, 0.f);
    if (hit) {
      const int li = light_of_pair(j, F);
      lightPos = light_point(S.lights[li], ls, j - li * F.light_spp, F);
      V3 Lv = sub(lightPos, hitP);
      const V3 Ls = Lv;
      Lv = normalize(Lv);
      const V3 H = normalize(add(Lv, V));
      const float NdotL = smax(dot(N, Lv), 0.0f), NdotH = smax(dot(N, H), 0.0f);
      const V3 so = add(hitP, mul(N, 1e-4f));
      const V3 sd = W.grid ? normalize(Lv) : normalize(Ls);
      ra = make_float4(so.x, so.y, so.z, W.grid ? length(Lv) : shadow_threshold(length(Ls)));
      rb = make_float4(sd.x, sd.y, sd.z, W.compact ? __uint_as_float((uint32_t)qi) : 0.0f);
      nlv = make_float2(NdotL, NdotH);
    }
    if (!W.compact) {
      wf_st(&W.rays[qi], ra);
      wf_st(&W.rays_b[qi], rb);
    } else if (hit) {
      wf_st(&W.rays[qc], ra);
      wf_st(&W.rays_b[qc], rb);
    }
    wf_st(&W.nl[qi], nlv);
  }
  if (!hit) return false;
  uint32_t flags = 0u;
  bool more = false;
  if (l + 1 > F.max_depth) {  // depth > MAX_DEPTH: the accumulated colour, unclamped (main.cpp:454)
    flags = WF_DEEP;
  } else {
    const drt_material m = S.mats[mat];
    float kr = m.refl;
    float ior2 = m.ior;
    if (!outside) ior2 = 1.0f;
    const float eta = 1.0f / ior2;
    const V3 Vt = sub(mul(N, dot(V, N)), V);
    const float sin_t = eta * length(Vt);
    if (m.trans > 0.0f && sin_t >= 1.0f) kr = 1.0f;
    if (m.ks > 0.0f) {
      V3 R = sub(mul(mul(N, dot(V, N)), 2.0f), V);
      if (W.inorder) {
        KRng rng{F.seed, pmix, rk};
        R = normalize(add(R, mul(rnd_unit_sphere(rng), F.roughness)));
        rk = rng.k;
      } else {
        R = normalize(R);
      }
      flags = WF_REFL | (dot(R, N) > 0.0f ? WF_RN : 0u) | (kr == 1.0f && m.refl != 1.0f ? WF_KR1 : 0u);
      next = make_ray(add(hitP, mul(N, 1e-4f)), R);
      ls = lightPos;
      more = true;
    }
  }
  wf_st(&W.lvl[li_], make_float4(0.f, 0.f, 0.f, __uint_as_float(mat | (flags << 24))));
  return more;
}
#endif
// No shadow query at levels from..max_depth of chunk slot `slot` (past its chain's end; a miss level
// has none either).
__device__ __forceinline__ void wf_mark_empty(const WfArgs& W, int from, uint32_t slot) {
  for (int k = from; k < W.levels; k++)
    for (int j = 0; j < W.pairs; j++) wf_st(&W.rays[wf_q(W, k, j, slot)], make_float4(0.f, 0.f, 0.f, -1.0f));
}

// MODE_SKEL: the closest query of bounce L.depth of sample L.smp returned: record it.  A hit that
// rayTracing() reflects from (depth <= MAX_DEPTH and Ks > 0, main.cpp:453-512; a two-pass scene has
// no refraction) starts the mirror child with the sample's reflectDir draw, computed exactly as
// lane_process does; otherwise the sample's closest-hit chain is complete and the pixel's next
// sample starts from the stream position it reached.  Shadow rays and colours are pass 2's.
template <bool STATS, int ACC>
__device__ void skel_process(const SceneArgs& S, const FrameArgs& F, Lane& L, Counters& C) {
  const bool hit = (L.fl & LF_HIT) != 0u;
  const size_t slot = (size_t)L.item * F.nsub + L.smp;
  F.skel_hits[slot * (uint32_t)(F.max_depth + 1) + (uint32_t)(L.depth - 1)] =
      make_uint2(__float_as_uint(L.best_t), hit ? L.best_prim : 0xFFFFFFFFu);
  if (hit && L.depth <= F.max_depth) {
    const uint32_t mat = prim_material(S.prims[3 * L.best_prim]);
    if (tab<ACC>(S.mats, mat).ks > 0.0f) {
      const V3 hitP = add(L.q.o, mul(L.q.d, L.best_t));  // main.cpp:361
      V3 N = normalize(prim_normal(S.prims, L.best_prim, L.q, L.best_t));
      if (!(dot(L.q.d, N) < 0.0f)) N = neg(N);
      const V3 V = neg(normalize(L.q.d));
      const V3 R = reflect_dir<MODE_SKEL>(F, L, N, V);
      L.depth++;
      start_query<STATS, ACC>(S, L, make_ray(add(hitP, mul(N, 1e-4f)), R), false, 0.0f, C);
      return;
    }
  }
  if (++L.smp < (uint32_t)F.nsub) {
    seq_start_sample<STATS, MODE_SKEL, ACC>(S, F, L, C);
    return;
  }
  L.item = kNoItem;
}

// MODE_CHAIN: the closest query of bounce L.depth of AA sample L.item returned: record it and go on
// with the mirror child exactly as lane_process would (main.cpp:453-512; a two-pass scene has no
// refraction), or end the item.  Shadow rays and colours are the replay pass's.
template <bool STATS, int ACC>
__device__ void chain_process(const SceneArgs& S, const FrameArgs& F, Lane& L, Counters& C) {
  const bool hit = (L.fl & LF_HIT) != 0u;
  F.skel_hits[(size_t)L.item * (uint32_t)(F.max_depth + 1) + (uint32_t)(L.depth - 1)] =
      make_uint2(__float_as_uint(L.best_t), hit ? L.best_prim : 0xFFFFFFFFu);
  if (hit && L.depth <= F.max_depth) {
    const uint32_t mat = prim_material(S.prims[3 * L.best_prim]);
    if (tab<ACC>(S.mats, mat).ks > 0.0f) {
      const V3 hitP = add(L.q.o, mul(L.q.d, L.best_t));  // main.cpp:361
      V3 N = normalize(prim_normal(S.prims, L.best_prim, L.q, L.best_t));
      if (!(dot(L.q.d, N) < 0.0f)) N = neg(N);
      const V3 V = neg(normalize(L.q.d));
      const V3 R = reflect_dir<MODE_AA>(F, L, N, V);
      L.depth++;
      start_query<STATS, ACC>(S, L, make_ray(add(hitP, mul(N, 1e-4f)), R), false, 0.0f, C);
      return;
    }
  }
  L.item = kNoItem;
}

// MODE_SEQ: start sample L.smp of pixel L.item (path_kernel's in-order loop, main.cpp:651-665,
// or the Whitted light-sample loop with glossy reflection, main.cpp:683-697).  The samples of
// a pixel go to samples[pixel * nsub + smp]; the ordered reduce sums them as the loop did.
template <bool STATS, int MODE, int ACC>
__device__ void seq_start_sample(const SceneArgs& S, const FrameArgs& F, Lane& L, Counters& C) {
  // MODE_REPLAY lanes hold a sample slot (pixel * nsub + sample), the others a pixel
  const uint32_t pixel = kReadBack<MODE> ? L.item / (uint32_t)F.nsub : L.item;
  const Item it = decode_item(F, S.res_x, S.res_y, pixel, 1);
  L.depth = 1;
  L.fsp = 0;
  L.ior1 = 1.0f;
  L.fl = 0u;
  if (STATS && !kReadBack<MODE>) C.v[ST_SAMPLES]++;  // pass 1 counts the two-pass frame's samples
  if (MODE == MODE_SKEL) F.skel_rk[(size_t)L.item * F.nsub + L.smp] = L.rk;
  RayP r;
  if (F.spp > 0) {
    float rx, ry, sx, sy;
    const int pos = F.perm ? (int)F.perm[(size_t)pixel * F.spp + L.smp] : shuffle_source(F, L.pmix, (int)L.smp);
    sample_prologue_at(F, L.pmix, (int)L.smp, pos, rx, ry, sx, sy);
    const float px = (float)it.x + rx, py = (float)it.y + ry;
    if (MODE != MODE_AREPLAY && MODE != MODE_TREPLAY && F.dof) {  // (an AA frame's replay has no DoF: those frames are in-order)
      KRng rng{F.seed, L.pmix, L.rk};
      r = primary_ray_lens(S, dvf(mul(rnd_unit_disk(rng), S.aperture), 2.0f), px, py);
      L.rk = rng.k;
    } else {
      r = primary_ray(S, px, py);
    }
    L.ls = mk(sx, sy, 0.0f);
  } else {
    const int s = (int)L.smp;
    r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
    L.ls = F.grid_res ? mk(((float)(s % F.grid_size) + 0.5f) / (float)F.grid_size,
                           ((float)(s / F.grid_size) + 0.5f) / (float)F.grid_size, 0.0f)
                      : mk(0.5f, 0.5f, 0.0f);
  }
  closest_query<STATS, MODE, ACC>(S, F, L, r, C);
}

// MODE_SEQ: start pixel `item` at sample smp with its keyed stream at call rk — a pixel just
// claimed (smp 0, rk past the prologue) or one another wave handed over (seq_donate).  One call
// site in the persistent loop for both, so the sample start is inlined there once.
template <bool STATS, int MODE, int ACC>
__device__ __forceinline__ void seq_begin(const SceneArgs& S, const FrameArgs& F, Lane& L, uint32_t item, uint32_t smp,
                                          uint32_t rk, Counters& C) {
  const Item it = decode_item(F, S.res_x, S.res_y, item, 1);
  if (!it.valid) {  // padding of a partial tile
    for (int k = 0; k < F.nsub; k++) F.samples[(size_t)item * F.nsub + k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (F.seq_cont) atomicAdd(F.work_counter + kSeqDone, 1u);
    L.item = kNoItem;
    return;
  }
  L.item = item;
  L.pmix = (uint32_t)(it.y * S.res_x + it.x) * 0x9E3779B9u;
  L.smp = smp;
  L.rk = rk;
  seq_start_sample<STATS, MODE, ACC>(S, F, L, C);
}
__device__ __forceinline__ uint32_t seq_first_rk(const FrameArgs& F) {
  return F.spp > 0 ? 5u * F.spp - 1u : 0u;  // after the prologue's 4 spp + spp - 1 calls
}

template <bool STATS, int MODE, int ACC>
__device__ __forceinline__ void lane_init(const SceneArgs& S, const FrameArgs& F, Lane& L, uint32_t item,
                                          Counters& C) {
  L.item = item;
  if (MODE == MODE_SEQ || MODE == MODE_SKEL) {  // work item = pixel
    seq_begin<STATS, MODE, ACC>(S, F, L, item, 0u, seq_first_rk(F), C);
    return;
  }
  if (kReadBack<MODE>) {  // work item = sample slot: the sample from its recorded stream position
    const Item it = decode_item(F, S.res_x, S.res_y, item, F.nsub);
    if (!it.valid) {  // padding of a partial tile
      F.samples[item] = make_float4(0.f, 0.f, 0.f, 0.f);
      L.item = kNoItem;
      return;
    }
    L.pmix = (uint32_t)(it.y * S.res_x + it.x) * 0x9E3779B9u;
    L.smp = (uint32_t)it.sub;
    // an AA / Whitted frame's replay has no stream positions (no draw after the prologue reaches the
    // frame, Q16): its rk holds the sample's closest-chain record instead (closest_query)
    const uint32_t rec = F.chain_div > 1 ? ((uint32_t)item - (uint32_t)it.sub) / (uint32_t)F.chain_div : item;
    L.rk = MODE == MODE_REPLAY ? F.skel_rk[item] : (MODE == MODE_TREPLAY ? rec * (uint32_t)F.tree_recs : rec);
    seq_start_sample<STATS, MODE, ACC>(S, F, L, C);
    return;
  }
  if (MODE == MODE_QSTREAM) {  // work item = one shadow query of a wavefront replay
    const float4 a = wf_ld(&F.q_rays[item]);
    if (a.w < 0.0f) {  // an empty slot: no query
      L.item = kNoItem;
      return;
    }
    const float4 b = wf_ld(&F.q_rays_b[item]);
    L.fl = 0u;
    start_query<STATS, ACC>(S, L, make_ray(mk(a.x, a.y, a.z), mk(b.x, b.y, b.z)), true, a.w, C);
    return;
  }
  if (MODE == MODE_PROG) {  // work item = pixel, one sample (main.cpp:540-572)
    const Item it = decode_item(F, S.res_x, S.res_y, item, 1);
    if (!it.valid) {
      F.samples[item] = make_float4(0.f, 0.f, 0.f, 0.f);
      L.item = kNoItem;
      return;
    }
    L.pmix = (uint32_t)(it.y * S.res_x + it.x) * 0x9E3779B9u;
    L.depth = 1;
    L.fsp = 0;
    L.ior1 = 1.0f;
    L.fl = 0u;
    if (STATS) C.v[ST_SAMPLES]++;
    KRng rng{F.seed, L.pmix, 0};
    RayP r;
    prog_primary(S, F, it, rng, r, L.ls);
    L.rk = rng.k;
    start_query<STATS, ACC>(S, L, r, false, 0.0f, C);
    return;
  }
  const int per_pixel = F.nsub;
  const Item it = decode_item(F, S.res_x, S.res_y, item, per_pixel);
  if (!it.valid) {  // padding of a partial tile
    F.samples[item] = make_float4(0.f, 0.f, 0.f, 0.f);
    L.item = kNoItem;
    return;
  }
  L.depth = 1;
  L.fsp = 0;
  L.ior1 = 1.0f;
  L.fl = 0u;
  if (STATS) C.v[ST_SAMPLES] += (MODE == MODE_CHAIN || MODE == MODE_TCHAIN) ? (uint32_t)F.chain_div : 1u;
  if (MODE == MODE_TCHAIN) L.rk = item * (uint32_t)F.tree_recs;  // the sample's first hit record
  RayP r;
  if (MODE == MODE_AA || ((MODE == MODE_CHAIN || MODE == MODE_TCHAIN) && F.spp > 0)) {
    const uint32_t pmix = (uint32_t)(it.y * S.res_x + it.x) * 0x9E3779B9u;
    float rx, ry, sx, sy;
    const int pos = F.perm ? (int)F.perm[item] : shuffle_source(F, pmix, it.sub);  // item = pixel * spp + sub
    sample_prologue_at(F, pmix, it.sub, pos, rx, ry, sx, sy);
    r = primary_ray(S, (float)it.x + rx, (float)it.y + ry);
    L.ls = mk(sx, sy, 0.0f);
  } else if (MODE == MODE_WHITTED_QUAD) {
    const int s = it.sub;
    L.ls = mk(((float)(s % F.grid_size) + 0.5f) / (float)F.grid_size,
              ((float)(s / F.grid_size) + 0.5f) / (float)F.grid_size, 0.0f);
    r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
  } else {  // MODE_WHITTED_POINT, and a Whitted frame's closest-chain pass (one lane per pixel)
    L.ls = mk(0.5f, 0.5f, 0.0f);
    r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
  }
  start_query<STATS, ACC>(S, L, r, false, 0.0f, C);
}

// Block size of path_persistent: kPBlock for the BVH; 256 for the Grid, whose per-block LDS
// copy of the macro-cell bitmap (16 KiB) has to fit the CU once per block.
template <int ACC>
__host__ __device__ constexpr int pblock() { return ACC == ACC_GRID ? 256 : kPBlock; }

template <bool TRI_ONLY, bool STATS, int MODE, int WAVES, int ACC>
__global__ void __launch_bounds__(pblock<ACC>(), WAVES) path_persistent(SceneArgs S, FrameArgs F) {
  constexpr int CAP = lds_cap(WAVES);
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_bytes[];
  uint32_t ov_desc[kMaxBvhDepth - CAP];
  float ov_t[kMaxBvhDepth - CAP];
  FrameStack fs;
  Counters C;
  for (int s = 0; s < ST_COUNT; s++) C.v[s] = 0;
  // (Measured alternative, kept out (round 3): the material and light tables copied into LDS after
  // the traversal stack, so shading reads them with ds_read instead of gathers queued behind the
  // node step's on the TA/TD path.  The kernel-local SceneArgs copy this needs moved kernel
  // arguments from SGPRs into VGPRs and left some table reads as flat loads: the headline kernel's
  // VGPR spills went 67 -> 113.)
  if (ACC == ACC_GRID) {  // the macro-cell occupancy bitmap, once per block
    for (int w = threadIdx.x; w < S.gmacro_words; w += pblock<ACC>()) ((LdsU32*)lds_bytes)[w] = S.gmacro[w];
    __syncthreads();
  }
  Lane L;
  L.item = kNoItem;
  L.fl = 0u;
  L.spa = threadIdx.x * 4u;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n_items = (uint32_t)F.n_items;
  bool exhausted = false;  // wave-uniform
  // Work partitions, one counter each (64 B apart): a wave on XCD x starts on items
  // [x * part_items, (x + 1) * part_items) — a band of tiles, so that XCD's L2 serves rays of
  // one screen region — and moves on to the next partition once that one is claimed.  Shards
  // the claim atomics over 8 words (MI355X_MICROARCH.md, dequeue); measured +0.3 %.
  // (Measured alternative, kept out (round 3): one partition per CU — 32 per XCD, a CU's waves
  // starting on a run of 4 consecutive tiles so that its L1 serves one small screen region, the CU's
  // slot from a per-frame (XCC id, HW_ID) table, and a 64-lane scan of the next partitions' counters
  // once a partition is used up: headline 1 677-1 711 against 1 692-1 743 Mrays/s, C3 / C4 / Grid
  // within 0.3 %, and 17 more VGPR spills in the mixed-primitive AA kernel.)
  uint32_t part = __builtin_amdgcn_s_getreg(GETREG_IMMED(3, 0, 20)) & 7u, parts_done = 0;  // HW_REG_XCC_ID
  uint64_t cyc[4] = {0, 0, 0, 0};  // stats builds: refill / node / shading / leaf-block cycles (wave-uniform)
  if (STATS && F.wave_times != nullptr && lane == 0)  // (a vector store by lane 0)
    F.wave_times[2 * ((blockIdx.x * blockDim.x + threadIdx.x) >> 6)] = __builtin_amdgcn_s_memrealtime();
  // MODE_SEQ tail (F.seq_cont): a lane runs a whole pixel's samples in order, so once every pixel
  // is claimed the frame's last ~quarter runs on waves whose lanes finish their last pixel at
  // different times (C4 at 1024^2: 0.56 node-loop SIMD efficiency, against 0.69 at 2048^2 with
  // 4x the pixels per lane).  Waves numbered past what the unfinished pixels need hand their
  // pixels over at sample boundaries and exit; the waves kept take them from the slots.
  // No register is added to the loop for this (its allocation sits on an edge): a
  // wave handing over sets `part` to kPartYield (no partition is claimed once the wave is
  // exhausted), and
  // the unfinished-pixel count is read from memory when it is needed.
  auto stamp = [&]() -> uint64_t {
    if (!STATS) return 0;
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
  };
  while (true) {
    const uint64_t t0 = stamp();
    // ---- refill idle lanes from the wave's current work partition (one atomic per wave)
    const uint64_t idle = __ballot(L.item == kNoItem);
    const int n_idle = __popcll(idle);
    if (!exhausted && (n_idle >= F.refill_min || n_idle == 64)) {
      const uint32_t pbeg = part * F.part_items;
      const uint32_t pn = pbeg < n_items ? min(F.part_items, n_items - pbeg) : 0u;
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(F.work_counter + 16u * part, (unsigned)n_idle);
      base = __shfl(base, 0, 64);
      if (base + (uint32_t)n_idle >= pn) {
        part = (part + 1u) & 7u;
        if (++parts_done == 8u) exhausted = true;
      }
      if (L.item == kNoItem) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        if (base + rank < pn) lane_init<STATS, MODE, ACC>(S, F, L, pbeg + base + rank, C);
      }
      // (Measured alternative, kept out: MODE_QSTREAM lanes that drew an empty slot claiming again, up to
      // three times, while refill_min lanes are idle — 1 863-1 869 against 1 868-1 875 Mrays/s on the Grid
      // headline at refill 16, profiles/r05_grid_qstream_reclaim_ab.jsonl.)
    }
    if (MODE == MODE_SEQ && exhausted && F.seq_cont && part != kPartYield) {
      const uint64_t idle2 = __ballot(L.item == kNoItem);
      const int n2 = __popcll(idle2);
      // About one iteration in sixteen (bits of the cycle counter), and on every try of a wave
      // with nothing to do: is this wave past the number the unfinished pixels need?  Then it
      // hands its pixels over (part = kPartYield) and exits once they are gone; with no pixel left, every
      // wave is.  A wave with nothing to do otherwise waits here for a handed-over pixel, so that
      // the loop's exit test stays the one-line test of the other modes (a test there reading
      // the pixel count raised the loop's VGPR spills 103 -> 216 and made C4 frames 6x slower).
      // The shared counters are read sparingly: thousands of waves polling one line slow the
      // pushes and pops on it.
      const uint64_t now = __builtin_amdgcn_s_memtime();
      bool look = (now & 0xF000ull) == 0ull;
      const bool try_pop = n2 == 64 || (n2 >= F.seq_pop_min && (now & 0x3000ull) == 0ull);
      uint32_t base = 0, k = 0, naps = 0;
      while (true) {
        if (look) {
          const uint32_t left = n_items - __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                                              F.work_counter + kSeqDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)(pblock<ACC>() / 64) +
                                                              (threadIdx.x >> 6));
          if ((uint64_t)wid * 6400u >= (uint64_t)left * (uint64_t)F.seq_slack) {
            part = kPartYield;
            break;
          }
        }
        if (!try_pop) break;
        if (lane == 0) {  // take up to n2 handed-over pixels
          const unsigned long long pp = __hip_atomic_load((unsigned long long*)(F.work_counter + kSeqPush),
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t pushed = min((uint32_t)pp, F.seq_cap), popped = (uint32_t)(pp >> 32);
          if (pushed > popped) {
            k = min((uint32_t)n2, pushed - popped);
            if (atomicCAS(F.work_counter + kSeqPop, popped, popped + k) != popped) k = 0;
            base = popped;
          }
        }
        k = __shfl(k, 0, 64);
        base = __shfl(base, 0, 64);
        if (k || n2 != 64) break;
        __builtin_amdgcn_s_sleep(127);  // ~8 k cycles between tries of an idle wave
        look = (++naps & 3u) == 0u;
      }
      if (k && L.item == kNoItem) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle2, 0u));
        if (rank < k) {
          unsigned long long v;  // the slot is written right after its push was counted
          while ((v = __hip_atomic_load(F.seq_cont + base + rank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0ull)
            __builtin_amdgcn_s_sleep(1);
          // The lane enters the shading pass as if sample smp - 1 of the pixel had just returned
          // (LF_RESUME): finish_sample, the one place a pixel's next sample starts, goes on from
          // there (a second inlined sample start here would cost registers in the loop).
          L.item = (uint32_t)v;
          const Item it = decode_item(F, S.res_x, S.res_y, L.item, 1);
          L.pmix = (uint32_t)(it.y * S.res_x + it.x) * 0x9E3779B9u;
          L.smp = ((uint32_t)(v >> 32) & 4095u) - 1u;
          L.rk = (uint32_t)(v >> 44);
          L.fsp = 0;
          L.fl = LF_RESUME;
        }
      }
    }
    const bool live = L.item != kNoItem;
    const bool in_trav = live && (L.fl & LF_TRAV);
    const uint64_t trav = __ballot(in_trav);
    const uint64_t ready = __ballot(live && !(L.fl & LF_TRAV));
    if (trav == 0 && ready == 0) {
      if (exhausted) break;
      continue;
    }
    const uint64_t t1 = stamp();
    // ---- one node step for every lane with a query in flight
    if (trav) {
      if (STATS && lane == 0) C.v[ST_WAVE_NODE_ITERS]++;
      if (ACC == ACC_GRID) {
        if (in_trav) grid_step<TRI_ONLY, STATS>(S, L, C, (const LdsU32*)lds_bytes, F.grid_walk, F.grid_pairs);
      } else {
        const bool wave_finite = __ballot(in_trav && !(L.fl & LF_FINITE)) == 0;
        // one primitive of a leaf per step (headline +1.4 %, C3 +0.4 %) in triangle scenes, except
        // in the replay pass, whose register allocation it tips (VGPR spills 42 -> 96, C4 1 290 ->
        // 770 Mrays/s), and in one-pass in-order frames (scratch 2 464 -> 2 496 B); mixed-primitive
        // scenes keep the whole-leaf step (C2, balls_low: 23 000 -> 20 800 Mrays/s with it)
#ifdef DRT_REPLAY_LEAF1  // (A/B) one primitive per step in the replay pass too
        constexpr int kLeaf1 = !TRI_ONLY || MODE == MODE_SEQ ? 0 : (MODE == MODE_SKEL || MODE == MODE_CHAIN ? 1 : 2);
#else
#ifdef DRT_CHAIN_LEAF1_2  // (A/B) the AA closest-chain pass leaves a one-primitive leaf step's last slot unread
        constexpr int kLeaf1 =
            !TRI_ONLY || kReadBack<MODE> || MODE == MODE_SEQ ? 0 : (MODE == MODE_SKEL || MODE == MODE_TCHAIN ? 1 : 2);
#else
        constexpr int kLeaf1 =
            !TRI_ONLY || kReadBack<MODE> || MODE == MODE_SEQ ? 0
                                                             : (MODE == MODE_SKEL || MODE == MODE_CHAIN || MODE == MODE_TCHAIN ? 1 : 2);
#endif
#endif
        // The shadow tree stays out of the path kernel (measured, round 4, headline 512^2 x 64 spp): its
        // lanes walked 26 % fewer node records per ray (75.8 -> 56.2 visits), but a wave whose lanes
        // mix closest-hit and shadow queries runs the binary and the 4-ary child tests one after the
        // other, and the 4-ary test's decode (~130 VALU) outweighs the gathers saved: 1 404 against
        // 1 509 Mrays/s with it switched off in the same build, and the code compiled into the loop
        // cost 1 509 against 1 757 Mrays/s by itself (tools/lib_matrix.sh).  The
        // streaming shadow kernel, whose waves hold shadow queries only, uses it.
        // The replay pass of two-pass in-order frames reads its closest hits back, so every lane that
        // traverses there holds a shadow query: its waves are homogeneous, as in the streaming kernel.
        constexpr bool kWide = kPathWide<MODE>;
        if (in_trav)
          node_step<TRI_ONLY, STATS, CAP, 0, kLeaf1, kWide>(S, L, (LdsByte*)lds_bytes, ov_desc, ov_t, wave_finite, C,
                                                            cyc[3]);
      }
    }
    const uint64_t t2 = stamp();
    // ---- batched shading for lanes whose query completed
    const bool done = live && !(L.fl & LF_TRAV);
    // Once every item is claimed, AA-style frames shade any ready lane (the frame is ending);
    // in-order (MODE_SEQ) frames reach that point with each lane still holding a pixel's
    // remaining samples, so they keep batching until half the live lanes are ready (C4:
    // shading SIMD efficiency 0.10 -> 0.33, +2.7 %; on MODE_AA the same rule costs 1.4 %).
    const bool drain = (MODE == MODE_SEQ || MODE == MODE_SKEL)
                           ? (exhausted && 2 * __popcll(ready) >= __popcll(ready | trav))
                           : exhausted;
    if (ready && (__popcll(ready) >= F.process_min || trav == 0 || drain)) {
      if (STATS) {
        if (lane == 0) C.v[ST_WAVE_PATH_ITERS]++;
        if (done) C.v[ST_LANE_PATH_ITERS]++;
      }
      if (done) {
        if (MODE == MODE_SEQ && part == kPartYield) L.fl |= LF_YIELD;
        if constexpr (MODE == MODE_QSTREAM) {  // the query's answer (a Grid miss of the grid box: shadowed)
          wf_st(&F.q_occ[L.item], (uint8_t)((L.fl & LF_HIT) ? 1 : 0));
          L.item = kNoItem;
        } else if constexpr (MODE == MODE_SKEL) skel_process<STATS, ACC>(S, F, L, C);
        else if constexpr (MODE == MODE_CHAIN) chain_process<STATS, ACC>(S, F, L, C);
        else lane_process<STATS, MODE, ACC>(S, F, L, fs, C);
      }
    }
    if (STATS) {
      const uint64_t t3 = stamp();
      cyc[0] += t1 - t0;
      cyc[1] += t2 - t1;
      cyc[2] += t3 - t2;
    }
  }
  flush_stats<STATS>(F, C);
  if (STATS && F.wave_times != nullptr && lane == 0)
    F.wave_times[2 * ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) + 1] = __builtin_amdgcn_s_memrealtime();
  if (STATS && lane == 0) {
    atomicAdd(&F.stats[ST_CYC_REFILL], (unsigned long long)cyc[0]);
    atomicAdd(&F.stats[ST_CYC_NODE], (unsigned long long)cyc[1]);
    atomicAdd(&F.stats[ST_CYC_PROC], (unsigned long long)cyc[2]);
    atomicAdd(&F.stats[ST_CYC_LEAF], (unsigned long long)cyc[3]);
  }
}

// ------------------------------------------------------------------------------------------
// Streaming traversal: BVH::Traverse (bvh.cpp:231-314 closest, :316-391 shadow) over an array
// of queries, one query per lane, lanes refilled from a global counter as they finish.  Only
// the traversal state is live (ray, slab constants, node, stack pointer, best hit), so the
// kernel runs at up to 8 waves per SIMD where the path kernel, which also carries shading
// state, holds 6.  The node step is the path kernel's, specialised for one query kind.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kTraceChunk = 256;  // queries claimed per wave per atomic
// shadow-query records through the scalar cache when a wave's visiting lanes share one (node_step UNI;
// -DDRT_UNI_FETCH, A/B): measured 2 418-2 447 against 2 487-2 495 Mrays/s on the headline and 3 284-3 356
// against 3 421-3 442 on C3 (profiles/r05_ab_uniform_node_fetch.jsonl) — the lanes of a wave leave a
// shared walk within a few steps, and the per-step readfirstlane / compare / divergent scalar path costs
// more than the vector loads it saves.  Off.
constexpr bool kUniFetch =
#ifdef DRT_UNI_FETCH
    true;
#else
    false;
#endif

struct TLane {
  uint32_t item, fl;
  RayP q;
  uint32_t cur, best_prim, spa;
  float best_t, thr;
};

// GV (round 6): the Grid scene's wavefront shadow queries on its shadow tree (node_step GV; S carries the
// Grid and, in its BVH fields, the tree): a ray that misses the grid box is occluded (grid.cpp:323), a
// certified hit is occluded, no hit is not, and the rest (no certificate, or a ray the tree does not
// take) go to A.fb_rays for grid_stream, which walks the Grid.
template <bool TRI_ONLY, int KIND, int WAVES, bool STATS, bool GV = false>
__global__ void __launch_bounds__(kPBlock, WAVES) trace_stream(SceneArgs S, TraceArgs A) {
  constexpr int CAP = lds_cap(WAVES);
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_bytes[];
  uint32_t ov_desc[kMaxBvhDepth - CAP];
  float ov_t[kMaxBvhDepth - CAP];
  Counters C;
  for (int s = 0; s < ST_COUNT; s++) C.v[s] = 0;
  uint64_t cyc_leaf = 0;
  TLane L;
  L.item = kNoItem;
  L.fl = 0u;
  L.spa = threadIdx.x * 4u;
  const uint32_t lane = threadIdx.x & 63u;
  // Queries are claimed kTraceChunk at a time per wave (one atomic), then handed to idle lanes
  // from that wave-private range: one counter word serves only ~90 dequeues/us
  // (MI355X_MICROARCH.md, dequeue), so a claim per refill would cap the kernel near 1 Gquery/s.
  uint32_t chunk_next = 0, chunk_end = 0;  // wave-uniform
  // sparse 2 (compact queries): chunk_next / chunk_end count the chunk's queries, chunk_base is its first
  // slot and chunk_cnt its four 64-slot groups' counts (one byte each)
  uint32_t chunk_base = 0, chunk_cnt = 0;  // wave-uniform
  bool exhausted = false;                  // wave-uniform: every partition's counter is past its end
  // partitions (TraceArgs::parts): a wave starts on its XCD's (HW_REG_XCC_ID), as path_persistent does
  uint32_t part = A.parts > 1 ? (__builtin_amdgcn_s_getreg(GETREG_IMMED(3, 0, 20)) & 7u) % (uint32_t)A.parts : 0u;
  uint32_t parts_done = 0;
  while (true) {
    const uint64_t idle = __ballot(L.item == kNoItem);
    const int n_idle = __popcll(idle);
    if (n_idle >= A.refill_min || n_idle == 64) {
      // a sparse query array (A.sparse: the wavefront replay's, thr < 0 = no query in the slot) is
      // walked until the idle lanes hold queries or fewer than refill_min lanes are left idle
      uint64_t want = idle;
      int n_want = n_idle;
      while (true) {
      while (chunk_next >= chunk_end && !exhausted) {  // claim from the wave's current partition
        const uint32_t pbeg = part * A.part_len, pend = min(pbeg + A.part_len, A.n);
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(A.counter + 16u * part, kTraceChunk);
        base = __shfl(base, 0, 64) + pbeg;
        chunk_next = base;
        chunk_end = base < pend ? min(base + kTraceChunk, pend) : base;
        if (A.sparse == 2) {  // the chunk's four group counts (band slots are a multiple of 256: one row)
          chunk_base = base;
          chunk_next = chunk_end = 0;
          if (base < pend) {
            const uint32_t row = base / A.band, o0 = base - row * A.band, bl = row / (uint32_t)A.pairs;
            chunk_cnt = *(const uint32_t*)(A.cnt + (size_t)bl * (A.band >> 6) + (o0 >> 6));
            chunk_end = (chunk_cnt & 0xffu) + ((chunk_cnt >> 8) & 0xffu) + ((chunk_cnt >> 16) & 0xffu) + (chunk_cnt >> 24);
          }
        }
        if (base + kTraceChunk >= pend) {  // this partition is claimed: the next one
          part = part + 1u == (uint32_t)A.parts ? 0u : part + 1u;
          if (++parts_done == (uint32_t)A.parts) exhausted = true;
        }
      }
      if (L.item == kNoItem) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
        const uint32_t it = chunk_next + rank;
        if (it < chunk_end) {
          uint32_t qs = it;  // the query's slot
          if (A.sparse == 2) {  // the it-th query of the chunk: group j's (it - its first query)-th slot
            const uint32_t p1 = chunk_cnt & 0xffu, p2 = p1 + ((chunk_cnt >> 8) & 0xffu), p3 = p2 + ((chunk_cnt >> 16) & 0xffu);
            const uint32_t j = (it >= p1 ? 1u : 0u) + (it >= p2 ? 1u : 0u) + (it >= p3 ? 1u : 0u);
            const uint32_t pre = j == 0u ? 0u : (j == 1u ? p1 : (j == 2u ? p2 : p3));
            qs = chunk_base + 64u * j + (it - pre);
          }
          // (interleaved records: rays_b = rays + 1, stride 2; or two arrays, stride 1)
          const size_t at = (size_t)qs * (uint32_t)A.stride;
          const float4 a = wf_ld(&A.rays[at]);
          // (an empty slot is thr < 0, wf_mark_empty; a NaN range is a query, answered 0, as MODE_QSTREAM
          // answers it — ADVICE r5: skipping it left a stale answer in occ_out)
          if (A.sparse != 1 || !(a.w < 0.0f)) {
          const float4 b = wf_ld(&A.rays_b[at]);
          L.item = A.sparse == 2 ? __float_as_uint(b.w) : it;  // (compact: the answer goes to the query's own slot)
          L.q = make_ray(mk(a.x, a.y, a.z), mk(b.x, b.y, b.z));
          L.thr = a.w;
          L.best_t = 3.402823466e+38f;
          L.best_prim = 0xFFFFFFFFu;
          L.spa &= kRowBytes - 1u;
          L.cur = S.root_desc;
          const bool fin = ray_finite(L.q);
          if constexpr (GV) {
            const bool wok = fin && wide_ray_ok(L.q);
            const bool missed = grid_box_missed(S, L.q);
            L.fl = LF_SHADOW | LF_FINITE | (missed ? LF_HIT : (wok ? (LF_TRAV | LF_WIDE) : LF_GVFB));
            L.cur = S.wroot;
            if (STATS) {
              C.v[ST_SHADOW]++;
              if (!missed && wok) C.v[ST_W_RAYS]++;
            }
          } else {
          float tmp;
          const bool root = box_hit(S.root_box[0], S.root_box[1], S.root_box[2], S.root_box[3], S.root_box[4],
                                    S.root_box[5], L.q, tmp);  // bvh.cpp:242 / :328
          L.fl = (KIND == 2 ? LF_SHADOW : 0u) | (root ? LF_TRAV : 0u) | (fin ? LF_FINITE : 0u);
          if (STATS) C.v[KIND == 2 ? ST_SHADOW : ST_CLOSEST]++;
          if (KIND == 2 && fin && S.wnodes != nullptr && wide_ray_ok(L.q)) {  // finite shadow rays: the 4-ary shadow tree
            if (STATS) C.v[ST_W_RAYS]++;
            L.fl |= LF_WIDE;
            L.cur = S.wroot;
          }
          }
          }
        }
      }
      chunk_next = min(chunk_next + (uint32_t)n_want, chunk_end);
      if (A.sparse != 1) break;
      want = __ballot(L.item == kNoItem);
      n_want = __popcll(want);
      if (n_want < A.refill_min || (exhausted && chunk_next >= chunk_end)) break;
      }
    }
    const bool in_trav = L.item != kNoItem && (L.fl & LF_TRAV);
    const uint64_t trav = __ballot(in_trav);
    if (trav) {
      if (STATS && lane == 0) C.v[ST_WAVE_NODE_ITERS]++;
      const bool wave_finite = __ballot(in_trav && !(L.fl & LF_FINITE)) == 0;
      // one primitive of a leaf per step in triangle scenes only, as in the path kernel (mixed-primitive
      // scenes measured ~10 % slower with it there)
      if (in_trav)
        node_step<TRI_ONLY, STATS, CAP, KIND, TRI_ONLY ? 1 : 0, KIND == 2, kUniFetch && KIND == 2 && !GV, GV>(
            S, L, (LdsByte*)lds_bytes, ov_desc, ov_t,
                                                                            wave_finite, C, cyc_leaf);
    }
    if (L.item != kNoItem && !(L.fl & LF_TRAV)) {  // query done: write its result
      if (GV && (L.fl & LF_GVFB)) {  // the Grid walk answers it (grid_fallback)
        const uint32_t k = atomicAdd(A.fb_count, 1u);
        A.fb_rays[2 * (size_t)k] = make_float4(L.q.o.x, L.q.o.y, L.q.o.z, L.thr);
        A.fb_rays[2 * (size_t)k + 1] = make_float4(L.q.d.x, L.q.d.y, L.q.d.z, __uint_as_float(L.item));
        if (STATS) C.v[ST_W_GRIDFB]++;
      } else if (KIND == 2) {
        wf_st(&A.occ_out[L.item], (uint8_t)((L.fl & LF_HIT) ? 1 : 0));
      } else {
        const bool hit = (L.fl & LF_HIT) != 0u;
        A.t_out[L.item] = hit ? L.best_t : 3.402823466e+38f;
        A.prim_out[L.item] = hit ? L.best_prim : 0xFFFFFFFFu;
      }
      L.item = kNoItem;
    } else if (!trav && exhausted && chunk_next >= chunk_end) {
      break;
    }
  }
  if (STATS) {
    for (int s = 0; s < ST_COUNT; s++) {
      unsigned long long v = C.v[s];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0 && v) atomicAdd(&A.stats[s], v);
    }
  }
}

// ------------------------------------------------------------------------------------------
// The Grid's wavefront shadow queries as their own streaming kernel (round 6): `Grid::Traverse(Ray&)`
// (grid.cpp:309-358) on the persistent stepper's grid_step, one query per lane, refilled from the compact
// query array as trace_stream refills (TraceArgs::sparse 2: a 256-query claim's four 64-slot group counts,
// the query's own slot in rays_b.w, the answer written there).  It replaces MODE_QSTREAM of the path
// kernel, whose lanes loaded every empty (thr < 0) slot of the marker layout to find the queries.
// ------------------------------------------------------------------------------------------
template <bool TRI_ONLY, int WAVES, bool STATS>
__global__ void __launch_bounds__(256, WAVES) grid_stream(SceneArgs S, TraceArgs A, int walk, int pairs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_bytes[];
  for (int w = threadIdx.x; w < S.gmacro_words; w += 256) ((LdsU32*)lds_bytes)[w] = S.gmacro[w];
  __syncthreads();
  Counters C;
  for (int s = 0; s < ST_COUNT; s++) C.v[s] = 0;
  Lane L;
  L.item = kNoItem;
  L.fl = 0u;
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t chunk_next = 0, chunk_end = 0, chunk_base = 0, chunk_cnt = 0;  // wave-uniform (as trace_stream)
  bool exhausted = false;
  // A.fb_rays (round 6): the queries the Grid scene's shadow tree left undecided (trace_stream GV), a
  // dense list of *A.fb_count queries, claimed 256 at a time
  const uint32_t fb_n = A.fb_rays ? __builtin_amdgcn_readfirstlane(*(volatile const uint32_t*)A.fb_count) : A.n;
  uint32_t part = A.parts > 1 ? (__builtin_amdgcn_s_getreg(GETREG_IMMED(3, 0, 20)) & 7u) % (uint32_t)A.parts : 0u;
  uint32_t parts_done = 0;
  while (true) {
    const uint64_t idle = __ballot(L.item == kNoItem);
    const int n_idle = __popcll(idle);
    if (n_idle >= A.refill_min || n_idle == 64) {
      while (chunk_next >= chunk_end && !exhausted) {  // claim 256 query slots of the wave's partition
        const uint32_t pbeg = part * A.part_len, pend = min(pbeg + A.part_len, fb_n);
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(A.counter + 16u * part, kTraceChunk);
        base = __shfl(base, 0, 64) + pbeg;
        chunk_base = base;
        chunk_next = chunk_end = 0;
        if (A.fb_rays) {  // the shadow tree's undecided queries: a dense list
          chunk_end = base < pend ? min(base + kTraceChunk, pend) - base : 0u;
        } else if (base < pend) {  // the chunk's four group counts (one row of the query array)
          const uint32_t row = base / A.band, o0 = base - row * A.band, bl = row / (uint32_t)A.pairs;
          chunk_cnt = *(const uint32_t*)(A.cnt + (size_t)bl * (A.band >> 6) + (o0 >> 6));
          chunk_end = (chunk_cnt & 0xffu) + ((chunk_cnt >> 8) & 0xffu) + ((chunk_cnt >> 16) & 0xffu) + (chunk_cnt >> 24);
        }
        if (base + kTraceChunk >= pend) {
          part = part + 1u == (uint32_t)A.parts ? 0u : part + 1u;
          if (++parts_done == (uint32_t)A.parts) exhausted = true;
        }
      }
      if (L.item == kNoItem) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        const uint32_t it = chunk_next + rank;
        if (it < chunk_end) {
          const uint32_t p1 = chunk_cnt & 0xffu, p2 = p1 + ((chunk_cnt >> 8) & 0xffu), p3 = p2 + ((chunk_cnt >> 16) & 0xffu);
          const uint32_t j = (it >= p1 ? 1u : 0u) + (it >= p2 ? 1u : 0u) + (it >= p3 ? 1u : 0u);
          const uint32_t pre = j == 0u ? 0u : (j == 1u ? p1 : (j == 2u ? p2 : p3));
          const size_t at = (size_t)(chunk_base + 64u * j + (it - pre)), fb = 2 * (size_t)(chunk_base + it);
          const float4 a = A.fb_rays ? A.fb_rays[fb] : wf_ld(&A.rays[at]);
          const float4 b = A.fb_rays ? A.fb_rays[fb + 1] : wf_ld(&A.rays_b[at]);
          L.item = __float_as_uint(b.w);
          L.fl = 0u;
          // a shadow ray that misses the grid box counts as shadowed (grid.cpp:323-324, Q8): start_query
          start_query<STATS, ACC_GRID>(S, L, make_ray(mk(a.x, a.y, a.z), mk(b.x, b.y, b.z)), true, a.w, C);
        }
      }
      chunk_next = min(chunk_next + (uint32_t)n_idle, chunk_end);
    }
    const bool in_trav = L.item != kNoItem && (L.fl & LF_TRAV);
    const uint64_t trav = __ballot(in_trav);
    if (trav) {
      if (STATS && lane == 0) C.v[ST_WAVE_NODE_ITERS]++;
      if (in_trav) grid_step<TRI_ONLY, STATS>(S, L, C, (const LdsU32*)lds_bytes, walk, pairs);
    }
    if (L.item != kNoItem && !(L.fl & LF_TRAV)) {  // query done: its answer to the query's own slot
      wf_st(&A.occ_out[L.item], (uint8_t)((L.fl & LF_HIT) ? 1 : 0));
      L.item = kNoItem;
    } else if (!trav && exhausted && chunk_next >= chunk_end) {
      break;
    }
  }
  if (STATS) {
    for (int s = 0; s < ST_COUNT; s++) {
      unsigned long long v = C.v[s];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0 && v) atomicAdd(&A.stats[s], v);
    }
  }
}

// The Grid scene's shadow queries that the shadow tree left undecided (trace_stream GV): each on
// Grid::Traverse(Ray&) (grid.cpp:309-358, grid_traverse), one per thread over the list trace_stream
// appended (A.fb_rays, *A.fb_count of them).
template <bool TRI_ONLY>
__global__ void __launch_bounds__(256) grid_fallback(SceneArgs S, TraceArgs A) {
  Counters C;
  const uint32_t n = *A.fb_count;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const float4 a = A.fb_rays[2 * (size_t)i], b = A.fb_rays[2 * (size_t)i + 1];
    const RayP r = make_ray(mk(a.x, a.y, a.z), mk(b.x, b.y, b.z));
    float t;
    uint32_t prim;
    const bool occ = grid_traverse<TRI_ONLY, false>(S, r, true, a.w, t, prim, C);
    A.occ_out[__float_as_uint(b.w)] = occ ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Wavefront replay (round 5; drt_kernels.hpp WfArgs): an AA / Whitted two-pass BVH frame without
// refraction, pass 2 as three launches — wf_gen, trace_stream over every shadow query of the frame,
// wf_combine — instead of the persistent MODE_AREPLAY kernel, whose waves interleave shading (a third
// of their lanes active) with the shadow traversal.  The arithmetic is lane_process's, in its order:
// setup_shadow's light point, ray and Phong factors per (level, light pair), the unshadowed terms added
// in pair order, the depth cut, and the mirror unwind.
// ------------------------------------------------------------------------------------------
// The sample's primary ray and light sample (seq_start_sample, MODE_AREPLAY / MODE_REPLAY); an in-order
// frame's lens draw from its recorded stream position `rk`.
__device__ __forceinline__ void wf_primary(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, const Item& it,
                                           uint32_t g, uint32_t pmix, uint32_t& rk, RayP& q, V3& ls) {
  if (F.spp > 0) {
    const uint32_t pixel = g / (uint32_t)F.nsub;
    float rx, ry, sx, sy;
    const int pos = F.perm ? (int)F.perm[(size_t)pixel * F.spp + it.sub] : shuffle_source(F, pmix, it.sub);
    sample_prologue_at(F, pmix, it.sub, pos, rx, ry, sx, sy);
    const float px = (float)it.x + rx, py = (float)it.y + ry;
    if (W.inorder && F.dof) {
      KRng rng{F.seed, pmix, rk};
      q = primary_ray_lens(S, dvf(mul(rnd_unit_disk(rng), S.aperture), 2.0f), px, py);
      rk = rng.k;
    } else {
      q = primary_ray(S, px, py);
    }
    ls = mk(sx, sy, 0.0f);
  } else {
    const int sb = it.sub;
    q = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
    ls = F.grid_res ? mk(((float)(sb % F.grid_size) + 0.5f) / (float)F.grid_size,
                         ((float)(sb / F.grid_size) + 0.5f) / (float)F.grid_size, 0.0f)
                    : mk(0.5f, 0.5f, 0.0f);
  }
}

__global__ void __launch_bounds__(256) wf_gen_kernel(SceneArgs S, FrameArgs F, WfArgs W) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;  // the slot's place in this chunk's buffers
  if (slot >= W.band * (uint32_t)W.bands) return;
  const bool in = slot < W.n_slots;  // (the last band's padding slots get empty queries only)
  const uint32_t g = W.slot0 + slot;  // the frame's sample slot
  const int md = F.max_depth;
  Item it{0, 0, 0, false};
  if (in) it = decode_item(F, S.res_x, S.res_y, g, F.nsub);
  int l = 0;  // the first level without shadow queries
#ifndef DRT_WF_PIECEWISE
  // every lane runs every level (padding lanes too): the query stores are whole-wave, and a compact
  // group's ballots see all 64 lanes
  RayP q{};
  V3 ls = mk(0, 0, 0);
  uint32_t rk = 0, rec = 0, pmix = 0;
  if (it.valid) {
    rec = F.chain_div > 1 ? (g - (uint32_t)it.sub) / (uint32_t)F.chain_div : g;
    pmix = (uint32_t)(it.y * S.res_x + it.x) * 0x9E3779B9u;
    rk = W.inorder ? F.skel_rk[g] : 0u;
    wf_primary(S, F, W, it, g, pmix, rk, q, ls);
  }
  bool live = it.valid;
  for (int lv = 0; lv <= md; lv++) {
    uint2 h = make_uint2(0u, 0xFFFFFFFFu);
    if (live) h = F.skel_hits[(size_t)rec * (uint32_t)(md + 1) + (uint32_t)lv];
    const bool hit = live && h.y != 0xFFFFFFFFu;
    RayP next;
    const bool more = wf_level_fw(S, F, W, slot, lv, q, live, hit, __uint_as_float(h.x), h.y, ls, pmix, rk, next);
    live = more;
    if (more) q = next;
  }
  l = W.levels;
#else
  if (it.valid) {
    const uint32_t rec = F.chain_div > 1 ? (g - (uint32_t)it.sub) / (uint32_t)F.chain_div : g;
    const uint32_t pmix = (uint32_t)(it.y * S.res_x + it.x) * 0x9E3779B9u;
    // an in-order frame's keyed stream from the sample's recorded position (MODE_REPLAY); an AA / Whitted
    // frame draws nothing after the prologue (Q16)
    uint32_t rk = W.inorder ? F.skel_rk[g] : 0u;
    RayP q;
    V3 ls;
    wf_primary(S, F, W, it, g, pmix, rk, q, ls);
    while (l <= md) {
      const uint2 h = F.skel_hits[(size_t)rec * (uint32_t)(md + 1) + (uint32_t)l];
      const bool hit = h.y != 0xFFFFFFFFu;
      RayP next;
      const bool more = wf_level(S, F, W, slot, l, q, hit, __uint_as_float(h.x), h.y, ls, pmix, rk, next);
      if (hit) l++;  // level l holds shadow queries
      if (!more) break;
      q = next;
    }
  }
#endif
  wf_mark_empty(W, l, slot);
}

// One sample's colour from its level records and shadow answers: the levels walked back from the last
// one, the unshadowed light terms added in the light loop's pair order, the depth cut and the mirror unwind.
__device__ __forceinline__ V3 wf_sample(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, uint32_t slot) {
  const size_t ns = W.n_slots;
  const int md = F.max_depth;
  // the last level of the chain: a miss, the depth cut, or a hit without a mirror child
  int last = 0;
  for (; last < md; last++) {
    const uint32_t fl = __float_as_uint(wf_ld(&W.lvl[(size_t)last * ns + slot]).w) >> 24;
    if (!(fl & WF_REFL)) break;
  }
  V3 c = mk(0, 0, 0);
  for (int l = last; l >= 0; l--) {
    const float4 rv = wf_ld(&W.lvl[(size_t)l * ns + slot]);
    const uint32_t w = __float_as_uint(rv.w), flags = w >> 24, mat = w & 0xffffffu;
    if (flags & WF_MISS) {
      c = mk(rv.x, rv.y, rv.z);
      continue;
    }
    const drt_material m = S.mats[mat];
    V3 acc = mk(0, 0, 0);
    for (int j = 0, u = 0; j < F.light_spp * S.n_lights; j++) {  // main.cpp:444-450, in the light loop's order
      if (!wf_pair_used(S, F, j)) continue;
      const size_t qi = wf_q(W, l, u++, slot);
      if (wf_ld(&W.occ[qi])) continue;
      const float2 nl = wf_ld(&W.nl[qi]);
      acc = add(acc, light_term(m, nl.x, nl.y, S.lights[light_of_pair(j, F)], F));
    }
    if (flags & WF_DEEP) {
      c = acc;
    } else {
      if (flags & WF_RN) {  // the mirror child returned c (main.cpp:513-518)
        const float kr = (flags & WF_KR1) ? 1.0f : m.refl;
        acc = add(acc, cmulc(mul(cclamp(c), kr), ld3(m.spec)));
      }
      c = cclamp(acc);
    }
  }
  return c;
}

__global__ void __launch_bounds__(256) wf_combine_kernel(SceneArgs S, FrameArgs F, WfArgs W) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= W.n_slots) return;
  const uint32_t g = W.slot0 + slot;
  const Item it = decode_item(F, S.res_x, S.res_y, g, F.nsub);
  const V3 c = it.valid ? wf_sample(S, F, W, slot) : mk(0, 0, 0);  // (zero: padding of a partial tile)
  F.samples[g] = make_float4(c.x, c.y, c.z, 0.0f);
}

// The pixel's framebuffer value, as reduce_kernel writes it: the ordered sum over its nsub sample colours
// (Color +=, main.cpp:664 / :694), times the scale (main.cpp:666 / :696), to the frame or the shard buffer.
__device__ __forceinline__ float* reduce_target(const ReduceArgs& A, uint32_t pidx) {
  if (A.full_frame) {
    const uint32_t per_tile = (uint32_t)(A.tile * A.tile);
    const uint32_t k = pidx / per_tile, pix = pidx - k * per_tile;
    uint32_t tx, ty;
    tile_of_position(A.shard + k * A.n_shards, A.tiles_x, tx, ty);
    const int x = (int)(tx * A.tile + pix % A.tile);
    const int y = (int)(ty * A.tile + pix / A.tile);
    if (x >= A.res_x || y >= A.res_y) return nullptr;
    return A.out + 3 * ((size_t)y * A.res_x + x);
  }
  return A.out + 3 * (size_t)pidx;
}

// wf_combine with the frame's reduce folded in (round 6): a block holds `ppb` whole pixels (ppb x nsub
// sample slots, nsub <= 1024), every thread combines its sample into LDS, then one thread per (pixel,
// channel) adds the pixel's samples in sample order — the same float additions, in the same order, as
// reduce_kernel — and writes the scaled value.  No sample buffer is written or read back, and a wavefront
// frame is one launch shorter.
__global__ void __launch_bounds__(1024) wf_combine_reduce_kernel(SceneArgs S, FrameArgs F, WfArgs W, ReduceArgs R,
                                                                 uint32_t ppb) {
  __shared__ float sc[3][1024];
  const uint32_t nsub = (uint32_t)R.nsub, per_block = ppb * nsub, t = threadIdx.x;
  const uint32_t base = blockIdx.x * per_block;  // the block's first chunk slot (a pixel's first sample)
  if (t < per_block) {
    const uint32_t slot = base + t;
    V3 c = mk(0, 0, 0);
    if (slot < W.n_slots) {
      const Item it = decode_item(F, S.res_x, S.res_y, W.slot0 + slot, F.nsub);
      if (it.valid) c = wf_sample(S, F, W, slot);
    }
    sc[0][t] = c.x;
    sc[1][t] = c.y;
    sc[2][t] = c.z;
  }
  __syncthreads();
  for (uint32_t w = t; w < 3u * ppb; w += blockDim.x) {  // (nsub < 3: more (pixel, channel) pairs than threads)
    const uint32_t p = w / 3u, ch = w - 3u * p;
    if (base + p * nsub >= W.n_slots) break;
    const float* v = sc[ch] + p * nsub;
    float r = 0.f;
#pragma unroll 8
    for (uint32_t i = 0; i < nsub; i++) r += v[i];
    float* o = reduce_target(R, (W.slot0 + base) / nsub + p);
    if (o) o[ch] = r * R.scale;
  }
}

void launch_wf_gen(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, hipStream_t st) {
  const uint32_t n = W.band * (uint32_t)W.bands;  // every band slot (padding included) gets its queries written
  hipLaunchKernelGGL(wf_gen_kernel, dim3((n + 255) / 256), dim3(256), 0, st, S, F, W);
}
void launch_wf_combine(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, hipStream_t st) {
  hipLaunchKernelGGL(wf_combine_kernel, dim3((W.n_slots + 255) / 256), dim3(256), 0, st, S, F, W);
}
// (the caller checks wf_can_fold_reduce: whole pixels per chunk, nsub <= 1024, not progressive)
void launch_wf_combine_reduce(const SceneArgs& S, const FrameArgs& F, const WfArgs& W, const ReduceArgs& R,
                              hipStream_t st) {
  const uint32_t nsub = (uint32_t)R.nsub, ppb = nsub >= 256u ? 1u : 256u / nsub, per_block = ppb * nsub;
  const uint32_t threads = (per_block + 63u) & ~63u;
  hipLaunchKernelGGL(wf_combine_reduce_kernel, dim3((W.n_slots + per_block - 1) / per_block), dim3(threads), 0, st, S,
                     F, W, R, ppb);
}

// Batched-query front end: rays n x {ox,oy,oz,dx,dy,dz} -> streaming-query records with the
// accelerator's range rule (BVH shadow: unit direction, |d| + EPSILON, bvh.cpp:321-322, :376).
__global__ void __launch_bounds__(256) trace_prep_kernel(const float* __restrict__ rays, int n, int shadow,
                                                         float4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* rr = rays + 6 * (size_t)i;
  V3 o = mk(rr[0], rr[1], rr[2]), d = mk(rr[3], rr[4], rr[5]);
  float thr = 0.0f;
  if (shadow) {
    thr = shadow_threshold(length(d));
    d = normalize(d);
  }
  out[2 * (size_t)i] = make_float4(o.x, o.y, o.z, thr);
  out[2 * (size_t)i + 1] = make_float4(d.x, d.y, d.z, 0.0f);
}

// HitRecord normal and object index of each closest-hit result (the trace_kernel epilogue).
__global__ void __launch_bounds__(256) trace_finish_kernel(SceneArgs S, const float4* __restrict__ q, int n,
                                                           float* t_out, const uint32_t* __restrict__ prim,
                                                           float* n_out, int32_t* obj_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = prim[i];
  if (p == 0xFFFFFFFFu) {
    n_out[3 * i] = 0.f; n_out[3 * i + 1] = 0.f; n_out[3 * i + 2] = 0.f;
    obj_out[i] = -1;
    return;
  }
  const float4 a = q[2 * (size_t)i], b = q[2 * (size_t)i + 1];
  const RayP r = make_ray(mk(a.x, a.y, a.z), mk(b.x, b.y, b.z));
  const V3 nn = prim_normal(S.prims, p, r, t_out[i]);
  n_out[3 * i] = nn.x; n_out[3 * i + 1] = nn.y; n_out[3 * i + 2] = nn.z;
  obj_out[i] = (int32_t)prim_object(S.prims[3 * p + 1]);
}

// Ordered sum over a pixel's items (Color += in sample order, main.cpp:664 / :694) and scale.
__global__ void __launch_bounds__(256) reduce_kernel(ReduceArgs A) {
  const uint32_t pidx = blockIdx.x * blockDim.x + threadIdx.x;
  if (pidx >= (uint32_t)A.n_my_tiles * (uint32_t)(A.tile * A.tile)) return;
  float r = 0.f, g = 0.f, b = 0.f;
  const float4* s = A.samples + (size_t)pidx * A.nsub;
  for (int i = 0; i < A.nsub; i++) {
    float4 v = s[i];
    r += v.x; g += v.y; b += v.z;
  }
  float* o = reduce_target(A, pidx);
  if (!o) return;
  if (A.prog_frame > 1) {  // lerp(a, b, t) = a + t * (b - a) in double (maths.h:56), t = 1.0 / FrameCount
    const double t = 1.0 / (double)A.prog_frame;
    o[0] = (float)((double)o[0] + t * ((double)r - (double)o[0]));
    o[1] = (float)((double)o[1] + t * ((double)g - (double)o[1]));
    o[2] = (float)((double)o[2] + t * ((double)b - (double)o[2]));
    return;
  }
  if (A.prog_frame == 0) {
    r *= A.scale; g *= A.scale; b *= A.scale;
  }
  o[0] = r; o[1] = g; o[2] = b;
}

// Shard-compact buffers (rank-major, floats_per_shard apart) -> full frame.
__global__ void __launch_bounds__(256) unshard_kernel(const float* __restrict__ shards, float* __restrict__ frame,
                                                      int tile, int tiles_x, int n_tiles, int n_shards,
                                                      int tiles_per_shard, int res_x, int res_y) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t per_tile = (uint64_t)tile * tile;
  if (i >= (uint64_t)n_tiles * per_tile) return;
  const uint32_t t = (uint32_t)(i / per_tile), pix = (uint32_t)(i - t * per_tile);
  const int x = (int)((t % tiles_x) * tile + pix % tile), y = (int)((t / tiles_x) * tile + pix / tile);
  if (x >= res_x || y >= res_y) return;
  const uint32_t p = position_of_tile(t % tiles_x, t / tiles_x, tiles_x);
  const uint32_t shard = p % n_shards, k = p / n_shards;
  const float* src = shards + ((size_t)shard * tiles_per_shard * per_tile + (size_t)k * per_tile + pix) * 3;
  float* o = frame + 3 * ((size_t)y * res_x + x);
  o[0] = src[0]; o[1] = src[1]; o[2] = src[2];
}

// Batched Traverse() queries.
template <int ACCEL, bool TRI_ONLY>
__global__ void __launch_bounds__(kBlock) trace_kernel(SceneArgs S, const float* __restrict__ rays, int n, int shadow,
                                                       float* t_out, float* n_out, int32_t* obj_out, uint8_t* occ_out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_stack[];
  TravStack tst{(LdsU32*)lds_stack + threadIdx.x, (LdsF32*)(lds_stack + kLdsStack * kBlock) + threadIdx.x};
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* rr = rays + 6 * (size_t)i;
  V3 o = mk(rr[0], rr[1], rr[2]), d = mk(rr[3], rr[4], rr[5]);
  Counters C;
  float t;
  uint32_t prim = 0;
  if (!shadow) {
    RayP r = make_ray(o, d);
    bool hit = traverse<ACCEL, TRI_ONLY, false>(S, r, false, 0.f, 0xFFFFFFFFu, t, prim, C, tst);
    if (hit) {
      V3 nn = prim_normal(S.prims, prim, r, t);
      t_out[i] = t;
      n_out[3 * i] = nn.x; n_out[3 * i + 1] = nn.y; n_out[3 * i + 2] = nn.z;
      obj_out[i] = (int32_t)prim_object(S.prims[3 * prim + 1]);
    } else {
      t_out[i] = 3.402823466e+38f;
      n_out[3 * i] = 0.f; n_out[3 * i + 1] = 0.f; n_out[3 * i + 2] = 0.f;
      obj_out[i] = -1;
    }
  } else {
    float len = length(d);
    RayP r;
    float thr;
    if (ACCEL == ACC_BVH) { thr = shadow_threshold(len); r = make_ray(o, normalize(d)); }
    else if (ACCEL == ACC_GRID) { thr = len; r = make_ray(o, normalize(d)); }
    else { thr = len; r = make_ray(o, d); }
    occ_out[i] = traverse<ACCEL, TRI_ONLY, false>(S, r, true, thr, 0xFFFFFFFFu, t, prim, C, tst) ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Host-side launchers (C++ linkage, called from drt_capi.hip)
// ------------------------------------------------------------------------------------------
constexpr size_t kStackLds = (size_t)kLdsStack * kBlock * 8;  // desc + t per entry

template <int A, bool T, int M>
static void launch_path_m(const SceneArgs& S, const FrameArgs& F, bool stats, hipStream_t st) {
  const uint64_t blocks = (F.n_items + kBlock - 1) / kBlock;
  if (stats) hipLaunchKernelGGL((path_kernel<A, T, true, M>), dim3((unsigned)blocks), dim3(kBlock), kStackLds, st, S, F);
  else hipLaunchKernelGGL((path_kernel<A, T, false, M>), dim3((unsigned)blocks), dim3(kBlock), kStackLds, st, S, F);
}
template <int A, bool T>
static void launch_path_t(const SceneArgs& S, const FrameArgs& F, bool stats, hipStream_t st) {
  switch (F.mode) {
    case MODE_AA: launch_path_m<A, T, MODE_AA>(S, F, stats, st); break;
    case MODE_SEQ: launch_path_m<A, T, MODE_SEQ>(S, F, stats, st); break;
    case MODE_PROG: launch_path_m<A, T, MODE_PROG>(S, F, stats, st); break;
    case MODE_WHITTED_QUAD: launch_path_m<A, T, MODE_WHITTED_QUAD>(S, F, stats, st); break;
    default: launch_path_m<A, T, MODE_WHITTED_POINT>(S, F, stats, st); break;
  }
}

template <bool T, bool ST, int M, int W, int A>
static void launch_persistent_w(const SceneArgs& S, const FrameArgs& F, hipStream_t st) {
  // the BVH kernel keeps its traversal stack's top in LDS; the Grid stepper needs none
  constexpr int B = pblock<A>();
  const size_t lds = A == ACC_BVH ? (size_t)lds_cap(W) * B * 8 : kMacroBits / 8;
  static int grid = 0;  // resident blocks across the device (per instantiation)
  if (!grid) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)path_persistent<T, ST, M, W, A>, B,
                                                       lds);
    grid = std::max(1, cus) * std::max(1, per_cu);
  }
  const uint64_t need = (F.n_items + B - 1) / B;
  const unsigned blocks = (unsigned)std::min<uint64_t>(need, (uint64_t)grid);
  hipLaunchKernelGGL((path_persistent<T, ST, M, W, A>), dim3(blocks), dim3(B), lds, st, S, F);
}
template <bool T, bool ST, int M, int A>
static void launch_persistent_m(const SceneArgs& S, const FrameArgs& F, hipStream_t st) {
  // register budget (waves/SIMD, DRT_WAVES).  BVH: 6 (80 VGPRs); 7 measured slower, and so were 5
  // and 4 (BVH 1541 / 1422 against 1770 Mrays/s at 6).  Grid: 5 (96 VGPRs) since its empty-cell
  // walk is capped per call (round 2: 1 101-1 177 against 1 039-1 085 at 6, interleaved runs;
  // 4 waves 983, 7 waves 880)
  if (A == ACC_GRID) {
    // (the Grid's closest-chain pass: 5 waves; 4 measured 1 364-1 369 against 1 424-1 427 Mrays/s,
    // 6 measured 1 318 against 1 381, profiles/r04_grid_chain_waves_ab.jsonl)
    if (F.waves == 7) launch_persistent_w<T, ST, M, 7, A>(S, F, st);
    else if (F.waves == 6) launch_persistent_w<T, ST, M, 6, A>(S, F, st);
    else launch_persistent_w<T, ST, M, 5, A>(S, F, st);
    return;
  }
  // (MODE_SKEL, the closest-chain pass, carries little state: 4 spills at 6 waves.  Measured at 4, 5,
  // 7 and 8 waves/SIMD on C4: 305, 280, 554 and 760 ms against 278 ms at 6.)
#ifdef DRT_REPLAY_LOW_WAVES
  if constexpr (kReplay<M>) {
    if (F.waves == 5) return launch_persistent_w<T, ST, M, 5, A>(S, F, st);
    if (F.waves == 4) return launch_persistent_w<T, ST, M, 4, A>(S, F, st);
  }
#endif
  if (F.waves == 7) launch_persistent_w<T, ST, M, 7, A>(S, F, st);
  else launch_persistent_w<T, ST, M, 6, A>(S, F, st);
}
template <bool T, bool ST, int A>
static void launch_persistent_t(const SceneArgs& S, const FrameArgs& F, hipStream_t st) {
  switch (F.mode) {
    case MODE_AA: launch_persistent_m<T, ST, MODE_AA, A>(S, F, st); break;
    case MODE_WHITTED_QUAD: launch_persistent_m<T, ST, MODE_WHITTED_QUAD, A>(S, F, st); break;
    case MODE_SEQ: launch_persistent_m<T, ST, MODE_SEQ, A>(S, F, st); break;
    case MODE_SKEL: launch_persistent_m<T, ST, MODE_SKEL, A>(S, F, st); break;
    case MODE_REPLAY: launch_persistent_m<T, ST, MODE_REPLAY, A>(S, F, st); break;
    case MODE_AREPLAY: launch_persistent_m<T, ST, MODE_AREPLAY, A>(S, F, st); break;
    case MODE_TCHAIN: launch_persistent_m<T, ST, MODE_TCHAIN, A>(S, F, st); break;
    case MODE_TREPLAY: launch_persistent_m<T, ST, MODE_TREPLAY, A>(S, F, st); break;
    case MODE_QSTREAM: if constexpr (A == ACC_GRID) launch_persistent_m<T, ST, MODE_QSTREAM, A>(S, F, st); break;
    case MODE_CHAIN: launch_persistent_m<T, ST, MODE_CHAIN, A>(S, F, st); break;
    case MODE_PROG: launch_persistent_m<T, ST, MODE_PROG, A>(S, F, st); break;
    default: launch_persistent_m<T, ST, MODE_WHITTED_POINT, A>(S, F, st); break;
  }
}
template <int A>
static void launch_persistent_a(const SceneArgs& S, const FrameArgs& F, bool tri_only, bool stats, hipStream_t st) {
  if (tri_only) { if (stats) launch_persistent_t<true, true, A>(S, F, st); else launch_persistent_t<true, false, A>(S, F, st); }
  else { if (stats) launch_persistent_t<false, true, A>(S, F, st); else launch_persistent_t<false, false, A>(S, F, st); }
}

// BVH always; Grid when its cells pack into 10 bits per axis (the stepper's cell encoding)
bool persistent_supported(int accel, const int gdim[3]) {
  return accel == ACC_BVH || (accel == ACC_GRID && gdim[0] <= 1024 && gdim[1] <= 1024 && gdim[2] <= 1024);
}

void launch_path_persistent(const SceneArgs& S, const FrameArgs& F, int accel, bool tri_only, bool stats,
                            hipStream_t st) {
  if (accel == ACC_GRID) launch_persistent_a<ACC_GRID>(S, F, tri_only, stats, st);
  else launch_persistent_a<ACC_BVH>(S, F, tri_only, stats, st);
}

void launch_path(const SceneArgs& S, const FrameArgs& F, int accel, bool tri_only, bool stats, hipStream_t st) {
  if (accel == ACC_BVH) { if (tri_only) launch_path_t<ACC_BVH, true>(S, F, stats, st); else launch_path_t<ACC_BVH, false>(S, F, stats, st); }
  else if (accel == ACC_GRID) { if (tri_only) launch_path_t<ACC_GRID, true>(S, F, stats, st); else launch_path_t<ACC_GRID, false>(S, F, stats, st); }
  else { if (tri_only) launch_path_t<ACC_NONE, true>(S, F, stats, st); else launch_path_t<ACC_NONE, false>(S, F, stats, st); }
}

void launch_shuffle(const FrameArgs& F, int res_x, int res_y, uint8_t* perm, hipStream_t st) {
  const uint32_t n_px = (uint32_t)F.n_my_tiles * F.tile * F.tile;
  hipLaunchKernelGGL(shuffle_kernel, dim3((n_px + kShuffleBlock - 1) / kShuffleBlock), dim3(kShuffleBlock), 0, st, F,
                     res_x, res_y, perm);
}

void launch_reduce(const ReduceArgs& A, hipStream_t st) {
  const uint32_t n = (uint32_t)A.n_my_tiles * A.tile * A.tile;
  hipLaunchKernelGGL(reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, st, A);
}

void launch_unshard(const float* shards, float* frame, int tile, int tiles_x, int n_tiles, int n_shards,
                    int tiles_per_shard, int res_x, int res_y, hipStream_t st) {
  const uint64_t n = (uint64_t)n_tiles * tile * tile;
  hipLaunchKernelGGL(unshard_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, shards, frame, tile, tiles_x,
                     n_tiles, n_shards, tiles_per_shard, res_x, res_y);
}

static bool env_fallback_kernel() {
  const char* e = getenv("DRT_GRID_TREE_FALLBACK_THREADS");
  return e && atoi(e) != 0;
}
template <bool T, int K, int W, bool ST, bool GV = false>
static void launch_stream_w(const SceneArgs& S, const TraceArgs& A, hipStream_t st) {
  const size_t lds = (size_t)lds_cap(W) * kPBlock * 8;
  static int grid = 0;  // resident blocks across the device (per instantiation)
  if (!grid) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)trace_stream<T, K, W, ST, GV>, kPBlock, lds);
    grid = std::max(1, cus) * std::max(1, per_cu);
  }
  const uint64_t need = ((uint64_t)A.n + kPBlock - 1) / kPBlock;
  const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(need, (uint64_t)grid));
  hipLaunchKernelGGL((trace_stream<T, K, W, ST, GV>), dim3(blocks), dim3(kPBlock), lds, st, S, A);
}
// the Grid scene's compact wavefront shadow queries on its shadow tree (trace_stream GV, triangle scenes),
// then grid_fallback on the Grid for the undecided ones (SG: the Grid's own SceneArgs, scene-order records)
template <bool T, int K, bool ST>
static void launch_stream_k(const SceneArgs& S, const TraceArgs& A, int waves, hipStream_t st) {
  if (waves >= 8) launch_stream_w<T, K, 8, ST>(S, A, st);
  else if (waves == 7) launch_stream_w<T, K, 7, ST>(S, A, st);
  else launch_stream_w<T, K, 6, ST>(S, A, st);
}
template <bool T, int W, bool ST>
static void launch_grid_stream_w(const SceneArgs& S, const TraceArgs& A, int walk, int pairs, hipStream_t st) {
  const size_t lds = kMacroBits / 8;
  static int grid = 0;  // resident blocks across the device (per instantiation)
  if (!grid) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)grid_stream<T, W, ST>, 256, lds);
    grid = std::max(1, cus) * std::max(1, per_cu);
  }
  const uint64_t need = ((uint64_t)A.n + 255) / 256;
  const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(need, (uint64_t)grid));
  hipLaunchKernelGGL((grid_stream<T, W, ST>), dim3(blocks), dim3(256), lds, st, S, A, walk, pairs);
}
// (A.fb_rays / fb_count; fb_counter: a zeroed claim counter for the second launch)
void launch_grid_tree_stream(const SceneArgs& ST_, const SceneArgs& SG, const TraceArgs& A, bool stats, int waves,
                             int walk, int pairs, unsigned int* fb_counter, hipStream_t st) {
  if (stats) launch_stream_w<true, 2, 7, true, true>(ST_, A, st);
  else if (waves <= 6) launch_stream_w<true, 2, 6, false, true>(ST_, A, st);
  else launch_stream_w<true, 2, 7, false, true>(ST_, A, st);
  if (env_fallback_kernel()) {  // (A/B) one query per thread, no refill
    static int blocks = 0;
    if (!blocks) {
      int dev = 0, cus = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      blocks = std::max(1, cus) * 8;
    }
    hipLaunchKernelGGL((grid_fallback<true>), dim3(blocks), dim3(256), 0, st, SG, A);
    return;
  }
  // grid_stream over the undecided queries' list: the persistent Grid stepper, refilled (its grid is
  // sized for the whole query array; waves past the list's end retire at once)
  TraceArgs B = A;
  B.counter = fb_counter;
  B.parts = 1;
  B.part_len = A.n;
  B.refill_min = 16;
  // (a stats frame counts each query once, in trace_stream: wide_grid_walks of them walked here)
  launch_grid_stream_w<true, 7, false>(SG, B, walk, pairs, st);
}
// the Grid's compact wavefront shadow queries (grid_stream); waves per SIMD 5, 6 or 7
void launch_grid_stream(const SceneArgs& S, const TraceArgs& A, bool tri_only, bool stats, int waves, int walk, int pairs,
                        hipStream_t st) {
  if (tri_only) {
    if (stats) launch_grid_stream_w<true, 7, true>(S, A, walk, pairs, st);
    else if (waves <= 5) launch_grid_stream_w<true, 5, false>(S, A, walk, pairs, st);
    else if (waves == 6) launch_grid_stream_w<true, 6, false>(S, A, walk, pairs, st);
    else launch_grid_stream_w<true, 7, false>(S, A, walk, pairs, st);
  } else {
    if (stats) launch_grid_stream_w<false, 7, true>(S, A, walk, pairs, st);
    else launch_grid_stream_w<false, 7, false>(S, A, walk, pairs, st);
  }
}

void launch_trace_stream(const SceneArgs& S, const TraceArgs& A, bool shadow, bool tri_only, bool stats, int waves,
                         hipStream_t st) {
  if (tri_only) {
    if (shadow) { if (stats) launch_stream_k<true, 2, true>(S, A, waves, st); else launch_stream_k<true, 2, false>(S, A, waves, st); }
    else { if (stats) launch_stream_k<true, 1, true>(S, A, waves, st); else launch_stream_k<true, 1, false>(S, A, waves, st); }
  } else {
    if (shadow) { if (stats) launch_stream_k<false, 2, true>(S, A, waves, st); else launch_stream_k<false, 2, false>(S, A, waves, st); }
    else { if (stats) launch_stream_k<false, 1, true>(S, A, waves, st); else launch_stream_k<false, 1, false>(S, A, waves, st); }
  }
}
void launch_trace_prep(const float* rays, int n, int shadow, float4* out, hipStream_t st) {
  hipLaunchKernelGGL(trace_prep_kernel, dim3((n + 255) / 256), dim3(256), 0, st, rays, n, shadow, out);
}
void launch_trace_finish(const SceneArgs& S, const float4* q, int n, float* t, const uint32_t* prim, float* nrm,
                         int32_t* obj, hipStream_t st) {
  hipLaunchKernelGGL(trace_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, st, S, q, n, t, prim, nrm, obj);
}

void launch_trace(const SceneArgs& S, int accel, bool tri_only, const float* rays, int n, int shadow, float* t,
                  float* nrm, int32_t* obj, uint8_t* occ, hipStream_t st) {
  dim3 g((n + kBlock - 1) / kBlock), b(kBlock);
#define DRT_TRACE(A, T) hipLaunchKernelGGL((trace_kernel<A, T>), g, b, kStackLds, st, S, rays, n, shadow, t, nrm, obj, occ)
  if (accel == ACC_BVH) { if (tri_only) DRT_TRACE(ACC_BVH, true); else DRT_TRACE(ACC_BVH, false); }
  else if (accel == ACC_GRID) { if (tri_only) DRT_TRACE(ACC_GRID, true); else DRT_TRACE(ACC_GRID, false); }
  else { if (tri_only) DRT_TRACE(ACC_NONE, true); else DRT_TRACE(ACC_NONE, false); }
#undef DRT_TRACE
}

}  // namespace drt
