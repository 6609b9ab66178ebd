// drt_device.hpp — device-side building blocks of the gfx950 ray tracer.
//
// Numerics contract: every expression keeps the reference's operand order, float/double
// promotions and comparison semantics (NaN included), and the translation unit is compiled
// with -ffp-contract=off, so nothing is fused into an FMA.  Division and sqrt are the
// correctly rounded sequences hipcc emits by default (v_div_scale/fmas/fixup,
// refined v_sqrt), which equal the reference's `(float)(1.0/(double)x)` results because one
// IEEE operation evaluated in double and rounded to float is correctly rounded (53 >= 2*24+2).
// Transcendentals (powf, expf, double pow) are ROCm's ocml versions: they may differ from
// glibc by <= 1 ulp, which is why image parity is stated as a per-channel tolerance.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "drt_layout.hpp"

namespace drt {

// ------------------------------------------------------------------------------------------
// 1.0f / a, correctly rounded.  For 2^-125 <= |a| <= 2^125, v_rcp_f32 (<= 1 ulp) refined by one
// FMA Newton step (e = 1 - a*r exact, r + r*e) rounds correctly for EVERY input: checked
// exhaustively on gfx950 against the IEEE division over all 2^32 bit patterns (tools/rcp_check.hip,
// 0 mismatches, profiles/r02_rcp_check.json).  Three VALU instead of the ~10 of hipcc's
// div_scale / div_fmas / div_fixup expansion.  Zeros, infinities, NaNs and the reciprocals that
// would be denormal or overflow take the full division (a branch that no wave takes in practice).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float rcp_rn(float a) {
  const float m = __builtin_fabsf(a);
  if (__builtin_expect(m >= 0x1p-125f && m <= 0x1p125f, 1)) {
    const float r = __builtin_amdgcn_rcpf(a);
    return __builtin_fmaf(__builtin_fmaf(-a, r, 1.0f), r, r);
  }
  return 1.0f / a;
}

// ------------------------------------------------------------------------------------------
// Vector / Color (vector.cpp:4-102, color.h:38-75)
// ------------------------------------------------------------------------------------------
struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 mul(V3 a, float f) { return mk(a.x * f, a.y * f, a.z * f); }
__device__ __forceinline__ V3 dvf(V3 a, float f) { return mk(a.x / f, a.y / f, a.z / f); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 u, V3 v) {
  return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
__device__ __forceinline__ float length(V3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ V3 normalize(V3 a) {  // vector.cpp:68: l = 1.0/len in double -> float
  float l = 1.0f / length(a);
  return mk(a.x * l, a.y * l, a.z * l);
}
__device__ __forceinline__ V3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

__device__ __forceinline__ float clamp01(float v) {  // CLAMP(0.0, R, 1.0) (color.h:11)
  return (v < 0.0f) ? 0.0f : ((v > 1.0f) ? 1.0f : v);
}
__device__ __forceinline__ V3 cclamp(V3 c) { return mk(clamp01(c.x), clamp01(c.y), clamp01(c.z)); }
__device__ __forceinline__ V3 cmulc(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }  // std::max
__device__ __forceinline__ float max3(float a, float b, float c) {  // macros.h:8
  return (a > b) ? ((a > c) ? a : c) : ((b > c) ? b : c);
}
__device__ __forceinline__ float min3(float a, float b, float c) {  // macros.h:5
  return (a < b) ? ((a < c) ? a : c) : ((b < c) ? b : c);
}

// (double)t > EPSILON (0.001) for a float t  <=>  t >= 0.001f, because 0.001f is the smallest
// float above 0.001; likewise fabs(x) < EPSILON  <=>  fabsf(x) < 0.001f.
constexpr float kEpsF = 0.001f;

// ------------------------------------------------------------------------------------------
// Keyed RNG — the k-th CRT rand() call inside pixel P.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ int keyed_rand(uint32_t seed, uint32_t pix_mix, uint32_t k) {
  return (int)(mix32(seed ^ mix32(pix_mix ^ mix32(k))) >> 17);
}
struct KRng {
  uint32_t seed, pmix, k;
  __device__ __forceinline__ int rand_() { return keyed_rand(seed, pmix, k++); }
  // maths.h:80: (float)rand() / ((float)RAND_MAX + 1.0) == r * 2^-15 exactly
  __device__ __forceinline__ float rand_float() { return (float)rand_() * (1.0f / 32768.0f); }
};
// maths.h:101-116 as g++ evaluates them: the first draw lands in the LAST component.
__device__ __forceinline__ V3 rnd_unit_disk(KRng& g) {
  V3 p;
  do {
    float fy = g.rand_float();
    float fx = g.rand_float();
    p = sub(mul(mk(fx, fy, 0.0f), 2.0f), mk(1.0f, 1.0f, 0.0f));
  } while (dot(p, p) >= 1.0f);
  return p;
}
__device__ __forceinline__ V3 rnd_unit_sphere(KRng& g) {
  V3 p;
  do {
    float fz = g.rand_float();
    float fy = g.rand_float();
    float fx = g.rand_float();
    p = sub(mul(mk(fx, fy, fz), 2.0f), mk(1.0f, 1.0f, 1.0f));
  } while (dot(p, p) >= 1.0f);
  return p;
}

// ------------------------------------------------------------------------------------------
// Ray with its per-axis slab constants (boundingBox.cpp:64-124 recomputes 1.0/dx per box;
// the value is the same every time, so it is computed once per ray).
// ------------------------------------------------------------------------------------------
struct RayP {
  V3 o, d;
  float ix, iy, iz;   // (float)(1.0 / d)
  // slab sign selectors (boundingBox.cpp:69-101: inv >= 0, false for NaN), recomputed on use so
  // they are never carried as lane masks across loops
  __device__ __forceinline__ bool sx() const { return ix >= 0.0f; }
  __device__ __forceinline__ bool sy() const { return iy >= 0.0f; }
  __device__ __forceinline__ bool sz() const { return iz >= 0.0f; }
};
__device__ __forceinline__ RayP make_ray(V3 o, V3 d) {
  RayP r;
  r.o = o; r.d = d;
  r.ix = 1.0f / d.x; r.iy = 1.0f / d.y; r.iz = 1.0f / d.z;
  return r;
}

// AABB::hit (boundingBox.cpp:64-124) + isInside (boundingBox.cpp:41-44) folded into the
// caller's "if inside: t = 0" (bvh.cpp:256-257).
__device__ __forceinline__ bool box_hit(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                        const RayP& r, float& t) {
  float txmin = ((r.sx() ? mnx : mxx) - r.o.x) * r.ix;
  float txmax = ((r.sx() ? mxx : mnx) - r.o.x) * r.ix;
  float tymin = ((r.sy() ? mny : mxy) - r.o.y) * r.iy;
  float tymax = ((r.sy() ? mxy : mny) - r.o.y) * r.iy;
  float tzmin = ((r.sz() ? mnz : mxz) - r.o.z) * r.iz;
  float tzmax = ((r.sz() ? mxz : mnz) - r.o.z) * r.iz;
  float t0 = max3(txmin, tymin, tzmin);
  float t1 = min3(txmax, tymax, tzmax);
  t = (t0 < 0.0f) ? t1 : t0;
  return (t0 < t1) && (t1 > 0.0f);
}
// Same test for rays whose three (float)(1.0/d) are finite.  Then no slab product can be NaN
// ((x - o) is finite, inv finite), and for NaN-free operands MAX3/MIN3's ternary chains and
// v_max3_f32 / v_min3_f32 select the same value (they may differ only in the sign of a zero
// result, which no later comparison or selection can observe), so the result is identical.
__device__ __forceinline__ bool box_hit_finite(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                               const RayP& r, float& t) {
  const float ax = (mnx - r.o.x) * r.ix, bx = (mxx - r.o.x) * r.ix;
  const float ay = (mny - r.o.y) * r.iy, by = (mxy - r.o.y) * r.iy;
  const float az = (mnz - r.o.z) * r.iz, bz = (mxz - r.o.z) * r.iz;
  const float t0 = fmaxf(fmaxf(r.sx() ? ax : bx, r.sy() ? ay : by), r.sz() ? az : bz);
  const float t1 = fminf(fminf(r.sx() ? bx : ax, r.sy() ? by : ay), r.sz() ? bz : az);
  t = (t0 < 0.0f) ? t1 : t0;
  return (t0 < t1) && (t1 > 0.0f);
}
__device__ __forceinline__ bool inv_finite(const RayP& r) {
  return fabsf(r.ix) < __builtin_inff() && fabsf(r.iy) < __builtin_inff() && fabsf(r.iz) < __builtin_inff();
}

__device__ __forceinline__ bool box_inside(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, V3 p) {
  return ((p.x > mnx && p.x < mxx) && (p.y > mny && p.y < mxy) && (p.z > mnz && p.z < mxz));
}

// ------------------------------------------------------------------------------------------
// Primitive intersection (scene.cpp:44-278).  Records: see drt_layout.hpp.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool hit_triangle(const float4& q0, const float4& q1, const float4& q2, const RayP& r,
                                             float& t) {  // scene.cpp:44-92
  V3 v0 = mk(q0.x, q0.y, q0.z), e1 = mk(q1.x, q1.y, q1.z), e2 = mk(q2.x, q2.y, q2.z);
  V3 h = cross(r.d, e2);
  float a = dot(e1, h);
  float f = rcp_rn(a);  // scene.cpp:56: f = 1.0/a
  V3 s = sub(r.o, v0);
  float u = f * dot(s, h);
  if (u < 0.0f || u > 1.0f) return false;
  V3 q = cross(s, e1);
  float v = f * dot(r.d, q);
  if (v < 0.0f || u + v > 1.0f) return false;
  t = f * dot(e2, q);
  return t >= kEpsF;
}

__device__ __forceinline__ bool hit_sphere(const float4& q0, const float4& q1, const RayP& r, float& t) {
  V3 c = mk(q0.x, q0.y, q0.z);  // scene.cpp:152-197
  float rad = q1.x;
  V3 oc = sub(r.o, c);
  float a = dot(r.d, r.d);
  float b = 2.0f * dot(oc, r.d);
  float cc = dot(oc, oc) - rad * rad;
  float disc = b * b - 4.0f * a * cc;
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc);
  float t1 = (-b - sq) / (2.0f * a);
  float t2 = (-b + sq) / (2.0f * a);
  if (t1 >= kEpsF) { t = t1; return true; }
  if (t2 >= kEpsF) { t = t2; return true; }
  return false;
}

__device__ __forceinline__ bool hit_plane(const float4& q0, const float4& q1, const RayP& r, float& t) {
  V3 pn = mk(q0.x, q0.y, q0.z);  // scene.cpp:118-149
  float pnrd = dot(pn, r.d);
  if (fabsf(pnrd) < kEpsF) return false;
  float tt = -(dot(pn, r.o) + q1.x) / pnrd;
  if (tt > 0.0f) { t = tt; return true; }
  return false;
}

__device__ __forceinline__ bool hit_box(const float4& q0, const float4& q1, const RayP& r, float& t) {
  V3 mn = mk(q0.x, q0.y, q0.z), mx = mk(q1.x, q1.y, q1.z);  // scene.cpp:218-278
  float tmin = (mn.x - r.o.x) / r.d.x;
  float tmax = (mx.x - r.o.x) / r.d.x;
  if (tmin > tmax) { float s = tmin; tmin = tmax; tmax = s; }
  float tymin = (mn.y - r.o.y) / r.d.y;
  float tymax = (mx.y - r.o.y) / r.d.y;
  if (tymin > tymax) { float s = tymin; tymin = tymax; tymax = s; }
  if ((tmin > tymax) || (tymin > tmax)) return false;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  float tzmin = (mn.z - r.o.z) / r.d.z;
  float tzmax = (mx.z - r.o.z) / r.d.z;
  if (tzmin > tzmax) { float s = tzmin; tzmin = tzmax; tzmax = s; }
  if ((tmin > tzmax) || (tzmin > tmax)) return false;
  if (tzmin > tmin) tmin = tzmin;
  if (tmin >= kEpsF) { t = tmin; return true; }
  return false;
}

// hit_triangle without its early exits: every lane computes u, v and t and the three tests
// are combined with non-short-circuit ands.  Same operations in the same order, so identical
// results (a NaN u or v passes both, as in the reference's ||-chains); t is written always and
// meaningful only when the test returns true.
__device__ __forceinline__ bool hit_triangle_sel(const float4& q0, const float4& q1, const float4& q2, const RayP& r,
                                                 float& t) {
  V3 v0 = mk(q0.x, q0.y, q0.z), e1 = mk(q1.x, q1.y, q1.z), e2 = mk(q2.x, q2.y, q2.z);
  V3 h = cross(r.d, e2);
  float a = dot(e1, h);
  float f = rcp_rn(a);  // scene.cpp:56: f = 1.0/a
  V3 s = sub(r.o, v0);
  float u = f * dot(s, h);
  V3 q = cross(s, e1);
  float v = f * dot(r.d, q);
  t = f * dot(e2, q);
  return !(u < 0.0f || u > 1.0f) & !(v < 0.0f || u + v > 1.0f) & (t >= kEpsF);
}

// Object::hit on an already loaded record (q2 is only read for triangles).
template <bool TRI_ONLY>
__device__ __forceinline__ bool hit_prim_rec(const float4& q0, const float4& q1, const float4& q2, const RayP& r,
                                             float& t) {
  if (TRI_ONLY) return hit_triangle(q0, q1, q2, r, t);
  switch (prim_type(q0)) {
    case PRIM_TRIANGLE: return hit_triangle(q0, q1, q2, r, t);
    case PRIM_SPHERE: return hit_sphere(q0, q1, r, t);
    case PRIM_PLANE: return hit_plane(q0, q1, r, t);
    default: return hit_box(q0, q1, r, t);
  }
}

template <bool TRI_ONLY>
__device__ __forceinline__ bool hit_prim(const float4* __restrict__ prims, uint32_t i, const RayP& r, float& t) {
  const float4 q0 = prims[3 * i];
  const float4 q1 = prims[3 * i + 1];
  if (TRI_ONLY) {
    const float4 q2 = prims[3 * i + 2];
    return hit_triangle(q0, q1, q2, r, t);
  }
  switch (prim_type(q0)) {
    case PRIM_TRIANGLE: {
      const float4 q2 = prims[3 * i + 2];
      return hit_triangle(q0, q1, q2, r, t);
    }
    case PRIM_SPHERE: return hit_sphere(q0, q1, r, t);
    case PRIM_PLANE: return hit_plane(q0, q1, r, t);
    default: return hit_box(q0, q1, r, t);
  }
}

// HitRecord.normal of a hit at distance t (the same expressions the hit routines evaluate).
__device__ __forceinline__ V3 prim_normal(const float4* __restrict__ prims, uint32_t i, const RayP& r, float t) {
  const float4 q0 = prims[3 * i];
  const float4 q1 = prims[3 * i + 1];
  switch (prim_type(q0)) {
    case PRIM_TRIANGLE: {
      const float4 q2 = prims[3 * i + 2];
      return normalize(cross(mk(q1.x, q1.y, q1.z), mk(q2.x, q2.y, q2.z)));
    }
    case PRIM_SPHERE: return normalize(sub(add(r.o, mul(r.d, t)), mk(q0.x, q0.y, q0.z)));
    case PRIM_PLANE: return mk(q0.x, q0.y, q0.z);
    default: {
      V3 hp = add(r.o, mul(r.d, t));
      V3 n = mk(0.f, 0.f, 0.f);
      if (fabsf(hp.x - q0.x) < kEpsF) n = mk(-1.f, 0.f, 0.f);
      else if (fabsf(hp.x - q1.x) < kEpsF) n = mk(1.f, 0.f, 0.f);
      else if (fabsf(hp.y - q0.y) < kEpsF) n = mk(0.f, -1.f, 0.f);
      else if (fabsf(hp.y - q1.y) < kEpsF) n = mk(0.f, 1.f, 0.f);
      else if (fabsf(hp.z - q0.z) < kEpsF) n = mk(0.f, 0.f, -1.f);
      else if (fabsf(hp.z - q1.z) < kEpsF) n = mk(0.f, 0.f, 1.f);
      return n;
    }
  }
}

}  // namespace drt
