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
template <bool TRI_ONLY, bool STATS>
__device__ __forceinline__ bool bvh_traverse(const SceneArgs& S, const RayP& r, bool shadow, float shadow_thr,
                                             float& best_t, uint32_t& best_prim, Counters& C) {
  float tmp;
  if (!box_hit(S.root_box[0], S.root_box[1], S.root_box[2], S.root_box[3], S.root_box[4], S.root_box[5], r, tmp))
    return false;
  uint32_t st_desc[kMaxBvhDepth];
  float st_t[kMaxBvhDepth];
  int sp = 0;
  uint32_t cur = S.root_desc;
  best_t = 3.402823466e+38f;  // HitRecord t = FLT_MAX
  bool hit = false;
  const float4* __restrict__ nodes = S.nodes;
  while (true) {
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
        bool left_first = shadow ? (tL <= tR) : (tL < tR);
        cur = left_first ? d.x : d.y;
        st_desc[sp] = left_first ? d.y : d.x;
        st_t[sp] = left_first ? tR : tL;
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
      if (shadow || st_t[sp] < best_t) {
        cur = st_desc[sp];
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
  if (r.sx) { txmin = (x0 - ox) * r.ix; txmax = (x1 - ox) * r.ix; } else { txmin = (x1 - ox) * r.ix; txmax = (x0 - ox) * r.ix; }
  if (r.sy) { tymin = (y0 - oy) * r.iy; tymax = (y1 - oy) * r.iy; } else { tymin = (y1 - oy) * r.iy; tymax = (y0 - oy) * r.iy; }
  if (r.sz) { tzmin = (z0 - oz) * r.iz; tzmax = (z1 - oz) * r.iz; } else { tzmin = (z1 - oz) * r.iz; tzmax = (z0 - oz) * r.iz; }
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
                                         float& t, uint32_t& prim, Counters& C) {
  if (STATS) C.v[shadow ? ST_SHADOW : ST_CLOSEST]++;
  if (ACCEL == ACC_BVH) return bvh_traverse<TRI_ONLY, STATS>(S, r, shadow, thr, t, prim, C);
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
__device__ V3 trace_path(const SceneArgs& S, const FrameArgs& F, RayP q, V3 ls, KRng& rng, Counters& C) {
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
    float t = 0.f;
    uint32_t prim = 0;
    const bool hit = traverse<ACCEL, TRI_ONLY, STATS>(S, q, shadow, thr, hitPrim, t, prim, C);

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
    } else {  // result of the shadow query of light j (main.cpp:444-450)
      if (!hit) {
        const drt_material& m = S.mats[mat];
        V3 diff = mul(mul(ld3(m.diff), m.kd), NdotL);
        V3 spec = mul(mul(ld3(m.spec), m.ks), powf(NdotH, m.shine));
        acc = add(acc, add(diff, spec));
      }
      j++;
      after_lights = (j >= S.n_lights);
    }

    if (!ret && !after_lights) {  // set up the shadow ray of light j (main.cpp:386-422)
      const drt_light& L0 = S.lights[j];
      if (L0.type == DRT_LIGHT_QUAD) lightPos = add(add(ld3(L0.pos), mul(ld3(L0.e1), ls.x)), mul(ld3(L0.e2), ls.y));
      else lightPos = ld3(L0.pos);
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
  const uint32_t t = F.shard + k * F.n_shards;
  const uint32_t tx = t % F.tiles_x, ty = t / F.tiles_x;
  it.x = (int)(tx * F.tile + pix % F.tile);
  it.y = (int)(ty * F.tile + pix / F.tile);
  it.valid = it.x < res_x && it.y < res_y;
  return it;
}

// Pixel jitter r[p] and the shuffled light sample s[p] of sample p, straight from the keyed
// stream: r uses calls 4p, 4p+1; s uses 4q+2, 4q+3 of the sample q that the Fisher-Yates pass
// (calls 4spp .. 5spp-2) moved to slot p.  Tracking slot p backwards through the swaps gives q.
__device__ __forceinline__ void sample_prologue(const FrameArgs& F, uint32_t pmix, int p, float& rx, float& ry,
                                                float& sx, float& sy) {
  const int n = F.n_sqrt;
  const int spp = (int)F.spp;
  float ex = (float)keyed_rand(F.seed, pmix, 4u * p) / 32767.0f;
  float ey = (float)keyed_rand(F.seed, pmix, 4u * p + 1u) / 32767.0f;
  rx = ((float)(p % n) + ex) / (float)n;
  ry = ((float)(p / n) + ey) / (float)n;
  int pos = p;
  for (int i = 1; i < spp; i++) {
    int jj = keyed_rand(F.seed, pmix, 4u * spp + (uint32_t)(spp - 1 - i)) % (i + 1);
    if (pos == i) pos = jj;
    else if (pos == jj) pos = i;
  }
  sx = (float)keyed_rand(F.seed, pmix, 4u * pos + 2u) / 32767.0f;
  sy = (float)keyed_rand(F.seed, pmix, 4u * pos + 3u) / 32767.0f;
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

template <int ACCEL, bool TRI_ONLY, bool STATS>
__global__ void __launch_bounds__(256) path_kernel(SceneArgs S, FrameArgs F) {
  const uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Counters C;
  for (int s = 0; s < ST_COUNT; s++) C.v[s] = 0;
  if (item < F.n_items) {
    const int per_pixel = (F.mode == MODE_SEQ) ? 1 : F.nsub;
    Item it = decode_item(F, S.res_x, S.res_y, item, per_pixel);
    V3 color = mk(0, 0, 0);
    if (it.valid) {
      const uint32_t P = (uint32_t)(it.y * S.res_x + it.x);
      const uint32_t pmix = P * 0x9E3779B9u;
      KRng rng{F.seed, pmix, 0};
      if (F.mode == MODE_AA) {
        float rx, ry, sx, sy;
        sample_prologue(F, pmix, it.sub, rx, ry, sx, sy);
        RayP r = primary_ray(S, (float)it.x + rx, (float)it.y + ry);
        if (STATS) C.v[ST_SAMPLES]++;
        color = trace_path<ACCEL, TRI_ONLY, STATS, false>(S, F, r, mk(sx, sy, 0.0f), rng, C);
      } else if (F.mode == MODE_SEQ) {
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
            V3 c = trace_path<ACCEL, TRI_ONLY, STATS, true>(S, F, r, mk(sx, sy, 0.0f), rng, C);
            color = add(color, c);
          }
        } else {  // Whitted with glossy reflection: each light sample in order on one stream
          RayP r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
          const int ns = F.grid_res ? (int)F.grid_res : 1;
          for (int s = 0; s < ns; s++) {
            V3 ls = F.grid_res ? mk(((float)(s % F.grid_size) + 0.5f) / (float)F.grid_size,
                                    ((float)(s / F.grid_size) + 0.5f) / (float)F.grid_size, 0.0f)
                               : mk(0.5f, 0.5f, 0.0f);
            if (STATS) C.v[ST_SAMPLES]++;
            color = add(color, trace_path<ACCEL, TRI_ONLY, STATS, true>(S, F, r, ls, rng, C));
          }
        }
      } else if (F.mode == MODE_WHITTED_QUAD) {
        const int s = it.sub;
        V3 ls = mk(((float)(s % F.grid_size) + 0.5f) / (float)F.grid_size,
                   ((float)(s / F.grid_size) + 0.5f) / (float)F.grid_size, 0.0f);
        RayP r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
        if (STATS) C.v[ST_SAMPLES]++;
        color = trace_path<ACCEL, TRI_ONLY, STATS, false>(S, F, r, ls, rng, C);
      } else {
        RayP r = primary_ray(S, (float)it.x + 0.5f, (float)it.y + 0.5f);
        if (STATS) C.v[ST_SAMPLES]++;
        color = trace_path<ACCEL, TRI_ONLY, STATS, false>(S, F, r, mk(0.5f, 0.5f, 0.0f), rng, C);
      }
    }
    F.samples[item] = make_float4(color.x, color.y, color.z, 0.0f);
  }
  flush_stats<STATS>(F, C);
}

// Ordered sum over a pixel's items (Color += in sample order, main.cpp:664 / :694) and scale.
__global__ void __launch_bounds__(256) reduce_kernel(ReduceArgs A) {
  const uint32_t pidx = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t per_tile = (uint32_t)(A.tile * A.tile);
  if (pidx >= (uint32_t)A.n_my_tiles * per_tile) return;
  float r = 0.f, g = 0.f, b = 0.f;
  const float4* s = A.samples + (size_t)pidx * A.nsub;
  for (int i = 0; i < A.nsub; i++) {
    float4 v = s[i];
    r += v.x; g += v.y; b += v.z;
  }
  r *= A.scale; g *= A.scale; b *= A.scale;
  if (A.full_frame) {
    const uint32_t k = pidx / per_tile, pix = pidx - k * per_tile;
    const uint32_t t = A.shard + k * A.n_shards;
    const int x = (int)((t % A.tiles_x) * A.tile + pix % A.tile);
    const int y = (int)((t / A.tiles_x) * A.tile + pix / A.tile);
    if (x >= A.res_x || y >= A.res_y) return;
    float* o = A.out + 3 * ((size_t)y * A.res_x + x);
    o[0] = r; o[1] = g; o[2] = b;
  } else {
    float* o = A.out + 3 * (size_t)pidx;
    o[0] = r; o[1] = g; o[2] = b;
  }
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
  const uint32_t shard = t % n_shards, k = t / n_shards;
  const float* src = shards + ((size_t)shard * tiles_per_shard * per_tile + (size_t)k * per_tile + pix) * 3;
  float* o = frame + 3 * ((size_t)y * res_x + x);
  o[0] = src[0]; o[1] = src[1]; o[2] = src[2];
}

// Batched Traverse() queries.
template <int ACCEL, bool TRI_ONLY>
__global__ void __launch_bounds__(256) trace_kernel(SceneArgs S, const float* __restrict__ rays, int n, int shadow,
                                                    float* t_out, float* n_out, int32_t* obj_out, uint8_t* occ_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* rr = rays + 6 * (size_t)i;
  V3 o = mk(rr[0], rr[1], rr[2]), d = mk(rr[3], rr[4], rr[5]);
  Counters C;
  float t;
  uint32_t prim = 0;
  if (!shadow) {
    RayP r = make_ray(o, d);
    bool hit = traverse<ACCEL, TRI_ONLY, false>(S, r, false, 0.f, 0xFFFFFFFFu, t, prim, C);
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
    occ_out[i] = traverse<ACCEL, TRI_ONLY, false>(S, r, true, thr, 0xFFFFFFFFu, t, prim, C) ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------------
// Host-side launchers (C++ linkage, called from drt_capi.hip)
// ------------------------------------------------------------------------------------------
template <int A, bool T>
static void launch_path_t(const SceneArgs& S, const FrameArgs& F, bool stats, hipStream_t st) {
  const uint64_t blocks = (F.n_items + 255) / 256;
  if (stats) hipLaunchKernelGGL((path_kernel<A, T, true>), dim3((unsigned)blocks), dim3(256), 0, st, S, F);
  else hipLaunchKernelGGL((path_kernel<A, T, false>), dim3((unsigned)blocks), dim3(256), 0, st, S, F);
}

void launch_path(const SceneArgs& S, const FrameArgs& F, int accel, bool tri_only, bool stats, hipStream_t st) {
  if (accel == ACC_BVH) { if (tri_only) launch_path_t<ACC_BVH, true>(S, F, stats, st); else launch_path_t<ACC_BVH, false>(S, F, stats, st); }
  else if (accel == ACC_GRID) { if (tri_only) launch_path_t<ACC_GRID, true>(S, F, stats, st); else launch_path_t<ACC_GRID, false>(S, F, stats, st); }
  else { if (tri_only) launch_path_t<ACC_NONE, true>(S, F, stats, st); else launch_path_t<ACC_NONE, false>(S, F, stats, st); }
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

void launch_trace(const SceneArgs& S, int accel, bool tri_only, const float* rays, int n, int shadow, float* t,
                  float* nrm, int32_t* obj, uint8_t* occ, hipStream_t st) {
  dim3 g((n + 255) / 256), b(256);
#define DRT_TRACE(A, T) hipLaunchKernelGGL((trace_kernel<A, T>), g, b, 0, st, S, rays, n, shadow, t, nrm, obj, occ)
  if (accel == ACC_BVH) { if (tri_only) DRT_TRACE(ACC_BVH, true); else DRT_TRACE(ACC_BVH, false); }
  else if (accel == ACC_GRID) { if (tri_only) DRT_TRACE(ACC_GRID, true); else DRT_TRACE(ACC_GRID, false); }
  else { if (tri_only) DRT_TRACE(ACC_NONE, true); else DRT_TRACE(ACC_NONE, false); }
#undef DRT_TRACE
}

}  // namespace drt
