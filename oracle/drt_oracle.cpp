// drt_oracle.cpp — CPU ORACLE (test infrastructure only; see drt_oracle.h header comment).
//
// A deliberately literal C++ restatement of the reference CPU renderer's hot path.  Every
// floating-point expression keeps the reference's operand order, promotions to double and
// comparison semantics (NaN included) so that results are bit-comparable.  Build with
// -ffp-contract=off (oracle/Makefile) so no multiply-add is ever fused.
//
// Reference = rita-mota/DistributionRayTracer @ 2025-06-14, paths below relative to
// DistributionRayTracer/.
#include "drt_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// ------------------------------------------------------------------------------------------
// Constants: macros.h:1 (EPSILON is a double), main.cpp:34 (MAX_DEPTH), maths.h:8 (PI float),
// MSVC CRT RAND_MAX (the reference is an MSVC project, DistributionRayTracer.vcxproj).
// ------------------------------------------------------------------------------------------
constexpr double kEps = 0.001;
constexpr float kPI = 3.141592653589793238462f;
constexpr int kRandMax = 0x7FFF;

// ------------------------------------------------------------------------------------------
// Vector (vector.cpp:4-102).  Free functions; each mirrors the member operator it restates.
// ------------------------------------------------------------------------------------------
struct V3 {
  float x, y, z;
};
inline V3 mk(float x, float y, float z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }      // vector.cpp:30
inline V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }      // vector.cpp:39
inline V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }                            // vector.cpp:35
inline V3 mul(V3 a, float f) { return mk(a.x * f, a.y * f, a.z * f); }          // vector.cpp:45
inline V3 dvf(V3 a, float f) { return mk(a.x / f, a.y / f, a.z / f); }          // vector.cpp:55
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }      // vector.cpp:50
inline V3 cross(V3 u, V3 v) {                                                   // vector.cpp:87
  return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
inline float length(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }  // vector.cpp:4 (float sqrt)
inline V3 normalize(V3 a) {                                                     // vector.cpp:68
  float l = (float)(1.0 / (double)length(a));
  return mk(a.x * l, a.y * l, a.z * l);
}
inline float axis_of(V3 a, int axis) { return axis == 0 ? a.x : (axis == 1 ? a.y : a.z); }  // vector.cpp:9

// Color (color.h:38-75)
struct C3 {
  float r, g, b;
};
inline C3 cmk(float r, float g, float b) { return C3{r, g, b}; }
inline C3 cadd(C3 a, C3 b) { return cmk(a.r + b.r, a.g + b.g, a.b + b.b); }
inline C3 csub(C3 a, C3 b) { return cmk(a.r - b.r, a.g - b.g, a.b - b.b); }
inline C3 cmul(C3 a, float c) { return cmk(a.r * c, a.g * c, a.b * c); }
inline C3 cmulc(C3 a, C3 b) { return cmk(a.r * b.r, a.g * b.g, a.b * b.b); }
inline float clamp01(float v) {  // CLAMP(0.0, R, 1.0): double-typed ternary, color.h:11
  double d = v;
  return (float)((d < 0.0) ? 0.0 : ((d > 1.0) ? 1.0 : d));
}
inline C3 cclamp(C3 a) { return cmk(clamp01(a.r), clamp01(a.g), clamp01(a.b)); }   // color.h:40
inline C3 cexp(C3 a) { return cmk(std::exp(a.r), std::exp(a.g), std::exp(a.b)); }  // color.h:47 (expf)

// libstdc++ std::min/std::max as the reference calls them (bvh.cpp:111-126, main.cpp:406)
inline float smin(float a, float b) { return (b < a) ? b : a; }
inline float smax(float a, float b) { return (a < b) ? b : a; }
inline float max3(float a, float b, float c) { return (a > b) ? ((a > c) ? a : c) : ((b > c) ? b : c); }  // macros.h:8
inline float min3(float a, float b, float c) { return (a < b) ? ((a < c) ? a : c) : ((b < c) ? b : c); }  // macros.h:5
inline double dclamp(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }         // maths.h:65

struct Ray {
  V3 o, d;
};

// ------------------------------------------------------------------------------------------
// AABB (boundingBox.cpp)
// ------------------------------------------------------------------------------------------
struct AABB {
  V3 mn, mx;
};
inline AABB default_aabb() { return AABB{mk(-1.f, -1.f, -1.f), mk(1.f, 1.f, 1.f)}; }  // boundingBox.cpp:8
inline bool aabb_inside(const AABB& b, V3 p) {                                         // boundingBox.cpp:41
  return ((p.x > b.mn.x && p.x < b.mx.x) && (p.y > b.mn.y && p.y < b.mx.y) && (p.z > b.mn.z && p.z < b.mx.z));
}
inline V3 aabb_centroid(const AABB& b) { return dvf(add(b.mn, b.mx), 2.0f); }           // boundingBox.cpp:47
inline void aabb_extend(AABB& a, const AABB& b) {                                        // boundingBox.cpp:52
  if (a.mn.x > b.mn.x) a.mn.x = b.mn.x;
  if (a.mn.y > b.mn.y) a.mn.y = b.mn.y;
  if (a.mn.z > b.mn.z) a.mn.z = b.mn.z;
  if (a.mx.x < b.mx.x) a.mx.x = b.mx.x;
  if (a.mx.y < b.mx.y) a.mx.y = b.mx.y;
  if (a.mx.z < b.mx.z) a.mx.z = b.mx.z;
}
inline bool aabb_hit(const AABB& bx, const Ray& r, float& t) {  // boundingBox.cpp:64-124
  float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
  float txmin, tymin, tzmin, txmax, tymax, tzmax;
  float a = (float)(1.0 / dx);
  if (a >= 0) { txmin = (bx.mn.x - ox) * a; txmax = (bx.mx.x - ox) * a; }
  else        { txmin = (bx.mx.x - ox) * a; txmax = (bx.mn.x - ox) * a; }
  float b = (float)(1.0 / dy);
  if (b >= 0) { tymin = (bx.mn.y - oy) * b; tymax = (bx.mx.y - oy) * b; }
  else        { tymin = (bx.mx.y - oy) * b; tymax = (bx.mn.y - oy) * b; }
  float c = (float)(1.0 / dz);
  if (c >= 0) { tzmin = (bx.mn.z - oz) * c; tzmax = (bx.mx.z - oz) * c; }
  else        { tzmin = (bx.mx.z - oz) * c; tzmax = (bx.mn.z - oz) * c; }
  double t0 = max3(txmin, tymin, tzmin);
  double t1 = min3(txmax, tymax, tzmax);
  t = (float)((t0 < 0) ? t1 : t0);
  return (t0 < t1 && t1 > 0);
}

// ------------------------------------------------------------------------------------------
// Scene model (scene.h, scene.cpp)
// ------------------------------------------------------------------------------------------
struct Material {  // scene.h:34-66; m_Refl := Ks (scene.h:42)
  C3 diff;
  float kd;
  C3 spec;
  float ks, shine, refl, T, ior;
};
Material default_material() {  // scene.h:38 (used for objects declared before any `mat`, which is UB upstream)
  return Material{cmk(0.2f, 0.2f, 0.2f), 0.2f, cmk(1.f, 1.f, 1.f), 0.8f, 20.f, 1.0f, 0.0f, 1.0f};
}

struct Object {  // scene.h:109-180
  int type = ORC_OBJ_TRIANGLE;
  int mat = -1;
  V3 a{}, b{}, c{};  // triangle points / sphere centre / plane normal / box min,max
  float r = 0.f;     // sphere radius
  float D = 0.f;     // plane offset
  AABB box{};        // GetBoundingBox()
};

struct Hit {  // scene.h:24 HitRecord
  bool isHit = false;
  V3 normal{0.f, 0.f, 0.f};
  float t = FLT_MAX;
};

Hit hit_triangle(const Object& o, const Ray& r) {  // scene.cpp:44-92 (Moller-Trumbore)
  Hit rec;
  V3 v0 = o.a, v1 = o.b, v2 = o.c;
  // scene.cpp:50-51 computes and discards a normal first: no observable effect.
  V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
  V3 h = cross(r.d, e2);
  float a = dot(e1, h);
  float f = 1.0f / a;
  V3 s = sub(r.o, v0);
  float u = f * dot(s, h);
  if (u < 0.0 || u > 1.0) return rec;
  V3 q = cross(s, e1);
  float v = f * dot(r.d, q);
  if (v < 0.0 || u + v > 1.0) return rec;
  float t = f * dot(e2, q);
  if ((double)t > kEps) {
    rec.t = t;
    rec.isHit = true;
    rec.normal = normalize(cross(e1, e2));
  }
  return rec;
}

Hit hit_plane(const Object& o, const Ray& r) {  // scene.cpp:118-149
  Hit rec;
  float pnrd = dot(o.a, r.d);
  if (std::fabs(pnrd) < kEps) return rec;
  float t = -(dot(o.a, r.o) + o.D) / pnrd;
  if (t > 0) {
    rec.t = t;
    rec.normal = o.a;
    rec.isHit = true;
  }
  return rec;
}

Hit hit_sphere(const Object& o, const Ray& r) {  // scene.cpp:152-197 (motion blur is dead code)
  Hit rec;
  V3 oc = sub(r.o, o.a);
  float a = dot(r.d, r.d);
  float b = 2.0f * dot(oc, r.d);
  float c = dot(oc, oc) - o.r * o.r;
  float disc = b * b - 4 * a * c;
  if (disc < 0) return rec;
  float sq = std::sqrt(disc);
  float t1 = (-b - sq) / (2.0f * a);
  float t2 = (-b + sq) / (2.0f * a);
  if ((double)t1 > kEps) rec.t = t1;
  else if ((double)t2 > kEps) rec.t = t2;
  else return rec;
  rec.isHit = true;
  rec.normal = normalize(sub(add(r.o, mul(r.d, rec.t)), o.a));
  return rec;
}

Hit hit_box(const Object& o, const Ray& ray) {  // scene.cpp:218-278
  Hit rec;
  V3 mn = o.a, mx = o.b;
  float tmin = (mn.x - ray.o.x) / ray.d.x;
  float tmax = (mx.x - ray.o.x) / ray.d.x;
  if (tmin > tmax) std::swap(tmin, tmax);
  float tymin = (mn.y - ray.o.y) / ray.d.y;
  float tymax = (mx.y - ray.o.y) / ray.d.y;
  if (tymin > tymax) std::swap(tymin, tymax);
  if ((tmin > tymax) || (tymin > tmax)) return rec;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  float tzmin = (mn.z - ray.o.z) / ray.d.z;
  float tzmax = (mx.z - ray.o.z) / ray.d.z;
  if (tzmin > tzmax) std::swap(tzmin, tzmax);
  if ((tmin > tzmax) || (tzmin > tmax)) return rec;
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  if ((double)tmin > kEps) {
    rec.t = tmin;
    rec.isHit = true;
    V3 hp = add(ray.o, mul(ray.d, tmin));
    V3 n = mk(0.f, 0.f, 0.f);
    if (std::fabs(hp.x - mn.x) < kEps) n = mk(-1.f, 0.f, 0.f);
    else if (std::fabs(hp.x - mx.x) < kEps) n = mk(1.f, 0.f, 0.f);
    else if (std::fabs(hp.y - mn.y) < kEps) n = mk(0.f, -1.f, 0.f);
    else if (std::fabs(hp.y - mx.y) < kEps) n = mk(0.f, 1.f, 0.f);
    else if (std::fabs(hp.z - mn.z) < kEps) n = mk(0.f, 0.f, -1.f);
    else if (std::fabs(hp.z - mx.z) < kEps) n = mk(0.f, 0.f, 1.f);
    rec.normal = n;
  }
  return rec;
}

inline Hit hit_object(const Object& o, const Ray& r) {  // virtual Object::hit dispatch
  switch (o.type) {
    case ORC_OBJ_TRIANGLE: return hit_triangle(o, r);
    case ORC_OBJ_SPHERE: return hit_sphere(o, r);
    case ORC_OBJ_PLANE: return hit_plane(o, r);
    default: return hit_box(o, r);
  }
}

struct Light {  // scene.h:68-107
  int quad = 0;
  V3 pos{};
  C3 emission{};
  V3 e1{}, e2{};
  uint32_t gridRes = 0;
  V3 area_point(V3 s) const { return add(add(pos, mul(e1, s.x)), mul(e2, s.y)); }  // scene.h:103
};

struct Camera {  // camera.h:12-101
  V3 eye{}, at{}, up{};
  float fovy = 0, vnear = 0, vfar = 0, plane_dist = 0, focal_ratio = 0, aperture = 0, w = 0, h = 0;
  int res_x = 0, res_y = 0;
  V3 u{}, v{}, n{};
  void init(V3 from, V3 At, V3 Up, float angle, float hither, float yon, int rx, int ry, float ap_ratio,
            float f_ratio) {  // camera.h:32-61
    eye = from; at = At; up = Up; fovy = angle; vnear = hither; vfar = yon; res_x = rx; res_y = ry;
    focal_ratio = f_ratio;
    n = sub(eye, at);
    plane_dist = length(n);
    n = dvf(n, plane_dist);
    u = cross(up, n);
    u = dvf(u, length(u));
    v = cross(n, u);
    h = 2 * plane_dist * std::tan((kPI * angle / 180) / 2.0f);
    w = ((float)res_x / res_y) * h;
    aperture = ap_ratio * (w / res_x);
  }
  void set_eye(V3 from) {  // camera.h:63-72: frame and plane distance only; w, h, aperture stay
    eye = from;
    n = sub(eye, at);
    plane_dist = length(n);
    n = dvf(n, plane_dist);
    u = cross(up, n);
    u = dvf(u, length(u));
    v = cross(n, u);
  }
  Ray primary(V3 ps) const {  // camera.h:74-83
    float a = (float)((double)(ps.x / res_x) - 0.5);
    float b = (float)((double)(ps.y / res_y) - 0.5);
    V3 dir = normalize(sub(add(mul(mul(u, w), a), mul(mul(v, h), b)), mul(n, plane_dist)));
    return Ray{eye, dir};
  }
  Ray primary_lens(V3 lens, V3 ps) const {  // camera.h:86-101
    V3 eo = add(add(eye, mul(u, lens.x)), mul(v, lens.y));
    float px = ((ps.x / res_x) - 0.5f) * w * focal_ratio;
    float py = ((ps.y / res_y) - 0.5f) * h * focal_ratio;
    float f = plane_dist * focal_ratio;
    V3 dir = normalize(sub(add(mul(u, px - lens.x), mul(v, py - lens.y)), mul(n, f)));
    return Ray{eo, dir};
  }
};

struct SkyFace {
  std::vector<uint8_t> img;  // bottom-up rows (DevIL IL_ORIGIN_LOWER_LEFT, scene.cpp:345-346)
  unsigned resX = 0, resY = 0, bpp = 3;
};

// ------------------------------------------------------------------------------------------
// Keyed RNG standing in for CRT rand().  Calls are made in exactly the
// order the reference makes them; g++ evaluates constructor arguments right-to-left, so
// `Vector(rand_float(), rand_float(), ...)` receives its FIRST draw in its LAST component
// (pinned against maths.h compiled by g++, oracle/ref_harness.cpp).
// ------------------------------------------------------------------------------------------
inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
struct KRng {
  uint32_t seed, pix, k;
  uint32_t shift = 17;    // 15-bit draws (MSVC CRT); 1 = 31-bit draws (glibc, harness pinning only)
  int rmax = kRandMax;
  uint32_t* lcg = nullptr;  // orc_options.lcg: the MSVC CRT rand() state shared by the whole frame
  int rand_() {
    if (lcg) {  // MSVC rand(): holdrand = holdrand * 214013 + 2531011; return (holdrand >> 16) & 0x7fff
      *lcg = *lcg * 214013u + 2531011u;
      return (int)((*lcg >> 16) & 0x7fffu);
    }
    uint32_t h = mix32(seed ^ mix32(pix * 0x9E3779B9u ^ mix32(k++)));
    return (int)(h >> shift);
  }
  float rand_float() { return (float)((double)(float)rand_() / ((double)(float)rmax + 1.0)); }  // maths.h:80
};
V3 rnd_unit_disk(KRng& g) {  // maths.h:101-107
  V3 p;
  do {
    float fy = g.rand_float();
    float fx = g.rand_float();
    p = sub(mul(mk(fx, fy, 0.0f), 2.0f), mk(1.0f, 1.0f, 0.0f));
  } while ((double)dot(p, p) >= 1.0);
  return p;
}
V3 rnd_unit_sphere(KRng& g) {  // maths.h:110-116
  V3 p;
  do {
    float fz = g.rand_float();
    float fy = g.rand_float();
    float fx = g.rand_float();
    p = sub(mul(mk(fx, fy, fz), 2.0f), mk(1.0f, 1.0f, 1.0f));
  } while ((double)dot(p, p) >= 1.0);
  return p;
}

struct Stats {
  uint64_t cc = 0, sc = 0, ci = 0, cl = 0, si = 0, sl = 0, cp = 0, sp = 0, samples = 0;
};

// ------------------------------------------------------------------------------------------
// BVH (bvh.cpp) — same build (binned SAH, 12 buckets, std::sort per axis), same traversal.
// ------------------------------------------------------------------------------------------
struct BVHNode {
  AABB box{};
  bool leaf = false;
  uint32_t n_objs = 0;
  uint32_t index = 0;
};

struct BVH {
  std::vector<BVHNode> nodes;
  std::vector<int> objects;  // object ids in leaf order
  std::vector<V3> centroid;  // per object id: GetBoundingBox().centroid()
  const std::vector<Object>* objs = nullptr;

  void build(const std::vector<Object>& o) {  // bvh.cpp:27-44
    objs = &o;
    nodes.clear(); objects.clear(); centroid.clear();
    AABB world{mk(FLT_MAX, FLT_MAX, FLT_MAX), mk(-FLT_MAX, -FLT_MAX, -FLT_MAX)};
    centroid.resize(o.size());
    for (size_t i = 0; i < o.size(); i++) {
      aabb_extend(world, o[i].box);
      objects.push_back((int)i);
      centroid[i] = aabb_centroid(o[i].box);
    }
    world.mn.x = (float)((double)world.mn.x - kEps); world.mn.y = (float)((double)world.mn.y - kEps);
    world.mn.z = (float)((double)world.mn.z - kEps);
    world.mx.x = (float)((double)world.mx.x + kEps); world.mx.y = (float)((double)world.mx.y + kEps);
    world.mx.z = (float)((double)world.mx.z + kEps);
    BVHNode root; root.box = world;
    nodes.push_back(root);
    build_recursive(0, (int)objects.size(), 0);
  }

  void sort_axis(int l, int r, int axis) {  // std::sort with BVH::Comparator (rayAccelerator.h:41-50)
    const V3* c = centroid.data();
    std::sort(objects.begin() + l, objects.begin() + r,
              [c, axis](int a, int b) { return axis_of(c[a], axis) < axis_of(c[b], axis); });
  }

  void build_recursive(int left_index, int right_index, int node) {  // bvh.cpp:62-227
    const int BUCKET_COUNT = 12;
    const float TRAVERSAL_COST = 1.0f, INTERSECTION_COST = 1.0f;
    int n_objects = right_index - left_index;
    if (n_objects <= 2) { nodes[node].leaf = true; nodes[node].index = left_index; nodes[node].n_objs = n_objects; return; }
    AABB box = nodes[node].box;
    V3 ext = sub(box.mx, box.mn);
    float psa = 2.0f * (ext.x * ext.y + ext.x * ext.z + ext.y * ext.z);
    int best_axis = 0;
    float best_cost = FLT_MAX;
    int best_split = left_index;
    for (int axis = 0; axis < 3; axis++) {
      sort_axis(left_index, right_index, axis);
      struct Bucket { int count = 0; V3 mn = {FLT_MAX, FLT_MAX, FLT_MAX}; V3 mx = {-FLT_MAX, -FLT_MAX, -FLT_MAX}; };
      Bucket buckets[BUCKET_COUNT];
      float min_bound = axis_of(box.mn, axis), max_bound = axis_of(box.mx, axis);
      float scale = (max_bound - min_bound) > 0.0f ? BUCKET_COUNT / (max_bound - min_bound) : 0.0f;
      for (int i = left_index; i < right_index; i++) {
        int id = objects[i];
        float cen = axis_of(centroid[id], axis);
        int bi = std::min(BUCKET_COUNT - 1, (int)((cen - min_bound) * scale));
        Bucket& bk = buckets[bi];
        bk.count++;
        const AABB& ob = (*objs)[id].box;
        bk.mn = mk(smin(bk.mn.x, ob.mn.x), smin(bk.mn.y, ob.mn.y), smin(bk.mn.z, ob.mn.z));
        bk.mx = mk(smax(bk.mx.x, ob.mx.x), smax(bk.mx.y, ob.mx.y), smax(bk.mx.z, ob.mx.z));
      }
      for (int i = 1; i < BUCKET_COUNT; i++) {
        V3 lmn = {FLT_MAX, FLT_MAX, FLT_MAX}, lmx = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        V3 rmn = {FLT_MAX, FLT_MAX, FLT_MAX}, rmx = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        int lc = 0, rc = 0;
        for (int j = 0; j < i; j++) {
          lmn = mk(smin(lmn.x, buckets[j].mn.x), smin(lmn.y, buckets[j].mn.y), smin(lmn.z, buckets[j].mn.z));
          lmx = mk(smax(lmx.x, buckets[j].mx.x), smax(lmx.y, buckets[j].mx.y), smax(lmx.z, buckets[j].mx.z));
          lc += buckets[j].count;
        }
        for (int j = i; j < BUCKET_COUNT; j++) {
          rmn = mk(smin(rmn.x, buckets[j].mn.x), smin(rmn.y, buckets[j].mn.y), smin(rmn.z, buckets[j].mn.z));
          rmx = mk(smax(rmx.x, buckets[j].mx.x), smax(rmx.y, buckets[j].mx.y), smax(rmx.z, buckets[j].mx.z));
          rc += buckets[j].count;
        }
        V3 le = sub(lmx, lmn);
        float la = 2.0f * (le.x * le.y + le.x * le.z + le.y * le.z);
        V3 re = sub(rmx, rmn);
        float ra = 2.0f * (re.x * re.y + re.x * re.z + re.y * re.z);
        float cost = TRAVERSAL_COST + (lc * la + rc * ra) * INTERSECTION_COST / psa;
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = axis;
          int count = 0;
          for (int j = 0; j < i; j++) count += buckets[j].count;
          best_split = left_index + count;
        }
      }
    }
    if (best_split <= left_index || best_split >= right_index || best_cost >= n_objects * INTERSECTION_COST) {
      nodes[node].leaf = true; nodes[node].index = left_index; nodes[node].n_objs = n_objects;
      return;
    }
    sort_axis(left_index, right_index, best_axis);
    int left_node = (int)nodes.size();
    nodes[node].leaf = false;
    nodes[node].index = left_node;
    AABB lb{mk(FLT_MAX, FLT_MAX, FLT_MAX), mk(-FLT_MAX, -FLT_MAX, -FLT_MAX)};
    AABB rb = lb;
    for (int i = left_index; i < best_split; i++) aabb_extend(lb, (*objs)[objects[i]].box);
    for (int i = best_split; i < right_index; i++) aabb_extend(rb, (*objs)[objects[i]].box);
    BVHNode ln, rn;
    ln.box = lb; rn.box = rb;
    nodes.push_back(ln);
    nodes.push_back(rn);
    build_recursive(left_index, best_split, left_node);
    build_recursive(best_split, right_index, left_node + 1);
  }

  struct SItem { int node; float t; };

  bool closest(const Ray& ray, int& hit_obj, Hit& hitRec, Stats& st) const {  // bvh.cpp:231-314
    st.cc++;
    float tmp;
    bool hit = false;
    SItem stackbuf[128];
    std::vector<SItem> big;
    int sp = 0;
    Hit rec;
    int cur = 0;
    Ray lr = ray;
    hitRec = rec;
    if (!aabb_hit(nodes[0].box, lr, tmp)) return false;
    while (true) {
      const BVHNode& cn = nodes[cur];
      if (!cn.leaf) {
        st.ci++;
        int li = cn.index;
        const BVHNode& L = nodes[li];
        const BVHNode& R = nodes[li + 1];
        float tL, tR;
        bool hL = aabb_hit(L.box, lr, tL);
        bool hR = aabb_hit(R.box, lr, tR);
        if (aabb_inside(L.box, ray.o)) tL = 0;
        if (aabb_inside(R.box, ray.o)) tR = 0;
        if (hL && hR) {
          SItem it;
          if (tL < tR) { cur = li; it = SItem{li + 1, tR}; }
          else { cur = li + 1; it = SItem{li, tL}; }
          if (sp < 128) stackbuf[sp++] = it; else { big.push_back(it); sp++; }
          continue;
        } else {
          if (hL) { cur = li; continue; }
          if (hR) { cur = li + 1; continue; }
        }
      } else {
        st.cl++;
        int nObj = cn.n_objs, oi = cn.index;
        for (int i = 0; i < nObj; i++) {
          int obj = objects[oi + i];
          st.cp++;
          rec = hit_object((*objs)[obj], lr);
          if (rec.isHit && rec.t < hitRec.t) { hitRec = rec; hit_obj = obj; hit = true; }
        }
      }
      bool better = false;
      while (sp > 0) {
        SItem it;
        if (sp > 128) { it = big.back(); big.pop_back(); } else it = stackbuf[sp - 1];
        sp--;
        if (it.t < hitRec.t) { cur = it.node; better = true; break; }
      }
      if (!better) break;
    }
    return hit;
  }

  bool shadow(Ray& ray, Stats& st) const {  // bvh.cpp:316-391
    st.sc++;
    float tmp;
    SItem stackbuf[128];
    std::vector<SItem> big;
    int sp = 0;
    Hit rec;
    double len = length(ray.d);
    ray.d = normalize(ray.d);
    Ray lr = ray;
    int cur = 0;
    if (!aabb_hit(nodes[0].box, lr, tmp)) return false;
    while (true) {
      const BVHNode& cn = nodes[cur];
      if (!cn.leaf) {
        st.si++;
        int li = cn.index;
        const BVHNode& L = nodes[li];
        const BVHNode& R = nodes[li + 1];
        float tL, tR;
        bool hL = aabb_hit(L.box, lr, tL);
        bool hR = aabb_hit(R.box, lr, tR);
        if (aabb_inside(L.box, ray.o)) tL = 0;
        if (aabb_inside(R.box, ray.o)) tR = 0;
        if (hL && hR) {
          SItem it;
          if (tL <= tR) { cur = li; it = SItem{li + 1, tR}; }
          else { cur = li + 1; it = SItem{li, tL}; }
          if (sp < 128) stackbuf[sp++] = it; else { big.push_back(it); sp++; }
          continue;
        } else {
          if (hL) { cur = li; continue; }
          if (hR) { cur = li + 1; continue; }
        }
      } else {
        st.sl++;
        int nObj = cn.n_objs, oi = cn.index;
        for (int i = 0; i < nObj; i++) {
          st.sp++;
          rec = hit_object((*objs)[objects[oi + i]], lr);
          if (rec.isHit && (double)rec.t <= len + kEps) return true;
        }
      }
      if (sp == 0) return false;
      SItem it;
      if (sp > 128) { it = big.back(); big.pop_back(); } else it = stackbuf[sp - 1];
      sp--;
      cur = it.node;
    }
  }
};

// ------------------------------------------------------------------------------------------
// Uniform grid (grid.cpp) — Amanatides & Woo with the reference's double stepping.
// ------------------------------------------------------------------------------------------
struct Grid {
  int nx = 0, ny = 0, nz = 0;
  float m = 2.0f;
  AABB bbox{};
  std::vector<int64_t> cell_start;  // CSR of cells[] (grid.cpp:71-91); insertion order kept
  std::vector<int32_t> cell_objs;
  const std::vector<Object>* objs = nullptr;

  void build(const std::vector<Object>& o) {  // grid.cpp:30-97
    objs = &o;
    AABB gb{mk(FLT_MAX, FLT_MAX, FLT_MAX), mk(-FLT_MAX, -FLT_MAX, -FLT_MAX)};
    for (auto& ob : o) aabb_extend(gb, ob.box);
    gb.mn.x = (float)((double)gb.mn.x - kEps); gb.mn.y = (float)((double)gb.mn.y - kEps);
    gb.mn.z = (float)((double)gb.mn.z - kEps);
    gb.mx.x = (float)((double)gb.mx.x + kEps); gb.mx.y = (float)((double)gb.mx.y + kEps);
    gb.mx.z = (float)((double)gb.mx.z + kEps);
    bbox = gb;
    double wx = bbox.mx.x - bbox.mn.x, wy = bbox.mx.y - bbox.mn.y, wz = bbox.mx.z - bbox.mn.z;
    double s = std::pow((int)o.size() / (wx * wy * wz), 0.3333333);
    nx = (int)(m * wx * s + 1);
    ny = (int)(m * wy * s + 1);
    nz = (int)(m * wz * s + 1);
    int64_t cells = (int64_t)nx * ny * nz;
    std::vector<std::vector<int32_t>> tmp((size_t)cells);
    for (size_t i = 0; i < o.size(); i++) {
      const AABB& ob = o[i].box;
      int ixmin = (int)dclamp((ob.mn.x - bbox.mn.x) * nx / (bbox.mx.x - bbox.mn.x), 0, nx - 1);
      int iymin = (int)dclamp((ob.mn.y - bbox.mn.y) * ny / (bbox.mx.y - bbox.mn.y), 0, ny - 1);
      int izmin = (int)dclamp((ob.mn.z - bbox.mn.z) * nz / (bbox.mx.z - bbox.mn.z), 0, nz - 1);
      int ixmax = (int)dclamp((ob.mx.x - bbox.mn.x) * nx / (bbox.mx.x - bbox.mn.x), 0, nx - 1);
      int iymax = (int)dclamp((ob.mx.y - bbox.mn.y) * ny / (bbox.mx.y - bbox.mn.y), 0, ny - 1);
      int izmax = (int)dclamp((ob.mx.z - bbox.mn.z) * nz / (bbox.mx.z - bbox.mn.z), 0, nz - 1);
      for (int iz = izmin; iz <= izmax; iz++)
        for (int iy = iymin; iy <= iymax; iy++)
          for (int ix = ixmin; ix <= ixmax; ix++) tmp[(size_t)(ix + nx * iy + nx * ny * iz)].push_back((int32_t)i);
    }
    cell_start.assign((size_t)cells + 1, 0);
    for (int64_t c = 0; c < cells; c++) cell_start[c + 1] = cell_start[c] + (int64_t)tmp[c].size();
    cell_objs.resize((size_t)cell_start[cells]);
    for (int64_t c = 0; c < cells; c++) std::copy(tmp[c].begin(), tmp[c].end(), cell_objs.begin() + cell_start[c]);
  }

  bool init_traverse(const Ray& ray, int& ix, int& iy, int& iz, double& dtx, double& dty, double& dtz,
                     double& txn, double& tyn, double& tzn, int& ixs, int& iys, int& izs, int& ixe, int& iye,
                     int& ize) const {  // grid.cpp:100-244
    float t0, t1;
    float ox = ray.o.x, oy = ray.o.y, oz = ray.o.z, dx = ray.d.x, dy = ray.d.y, dz = ray.d.z;
    float x0 = bbox.mn.x, y0 = bbox.mn.y, z0 = bbox.mn.z, x1 = bbox.mx.x, y1 = bbox.mx.y, z1 = bbox.mx.z;
    float txmin, tymin, tzmin, txmax, tymax, tzmax;
    float a = (float)(1.0 / dx);
    if (a >= 0) { txmin = (x0 - ox) * a; txmax = (x1 - ox) * a; } else { txmin = (x1 - ox) * a; txmax = (x0 - ox) * a; }
    float b = (float)(1.0 / dy);
    if (b >= 0) { tymin = (y0 - oy) * b; tymax = (y1 - oy) * b; } else { tymin = (y1 - oy) * b; tymax = (y0 - oy) * b; }
    float c = (float)(1.0 / dz);
    if (c >= 0) { tzmin = (z0 - oz) * c; tzmax = (z1 - oz) * c; } else { tzmin = (z1 - oz) * c; tzmax = (z0 - oz) * c; }
    if (txmin > tymin) t0 = txmin; else t0 = tymin;
    if (tzmin > t0) t0 = tzmin;
    if (txmax < tymax) t1 = txmax; else t1 = tymax;
    if (tzmax < t1) t1 = tzmax;
    if (t0 > t1 || t1 < 0) return false;
    if (aabb_inside(bbox, ray.o)) {
      ix = (int)dclamp((ox - x0) * nx / (x1 - x0), 0, nx - 1);
      iy = (int)dclamp((oy - y0) * ny / (y1 - y0), 0, ny - 1);
      iz = (int)dclamp((oz - z0) * nz / (z1 - z0), 0, nz - 1);
    } else {
      V3 p = add(ray.o, mul(ray.d, t0));
      ix = (int)dclamp((p.x - x0) * nx / (x1 - x0), 0, nx - 1);
      iy = (int)dclamp((p.y - y0) * ny / (y1 - y0), 0, ny - 1);
      iz = (int)dclamp((p.z - z0) * nz / (z1 - z0), 0, nz - 1);
    }
    dtx = (txmax - txmin) / nx;
    dty = (tymax - tymin) / ny;
    dtz = (tzmax - tzmin) / nz;
    if (dx > 0) { txn = txmin + (ix + 1) * dtx; ixs = +1; ixe = nx; }
    else { txn = txmin + (nx - ix) * dtx; ixs = -1; ixe = -1; }
    if (dx == 0.0) txn = FLT_MAX;
    if (dy > 0) { tyn = tymin + (iy + 1) * dty; iys = +1; iye = ny; }
    else { tyn = tymin + (ny - iy) * dty; iys = -1; iye = -1; }
    if (dy == 0.0) tyn = FLT_MAX;
    if (dz > 0) { tzn = tzmin + (iz + 1) * dtz; izs = +1; ize = nz; }
    else { tzn = tzmin + (nz - iz) * dtz; izs = -1; ize = -1; }
    if (dz == 0.0) tzn = FLT_MAX;
    return true;
  }

  bool closest(const Ray& ray, int& hit_obj, Hit& hitRec, Stats& st) const {  // grid.cpp:247-306
    st.cc++;
    int ix, iy, iz, ixs, iys, izs, ixe, iye, ize;
    double txn, tyn, tzn, dtx, dty, dtz;
    if (!init_traverse(ray, ix, iy, iz, dtx, dty, dtz, txn, tyn, tzn, ixs, iys, izs, ixe, iye, ize)) return false;
    int closestObj = -1;
    while (true) {
      st.cl++;
      int64_t cidx = (int64_t)ix + (int64_t)nx * iy + (int64_t)nx * ny * iz;
      for (int64_t q = cell_start[cidx]; q < cell_start[cidx + 1]; q++) {
        int obj = cell_objs[q];
        st.cp++;
        Hit rec = hit_object((*objs)[obj], ray);
        if (rec.isHit && rec.t < hitRec.t) { hitRec.t = rec.t; hitRec.isHit = true; hitRec.normal = rec.normal; closestObj = obj; }
      }
      if (txn < tyn && txn < tzn) {
        if (hitRec.t < txn) { hit_obj = closestObj; return true; }
        txn += dtx; ix += ixs;
        if (ix == ixe) return false;
      } else if (tyn < tzn) {
        if (hitRec.t < tyn) { hit_obj = closestObj; return true; }
        tyn += dty; iy += iys;
        if (iy == iye) return false;
      } else {
        if (hitRec.t < tzn) { hit_obj = closestObj; return true; }
        tzn += dtz; iz += izs;
        if (iz == ize) return false;
      }
    }
  }

  bool shadow(Ray& ray, Stats& st) const {  // grid.cpp:309-358
    st.sc++;
    double len = length(ray.d);
    ray.d = normalize(ray.d);
    int ix, iy, iz, ixs, iys, izs, ixe, iye, ize;
    double txn, tyn, tzn, dtx, dty, dtz;
    if (!init_traverse(ray, ix, iy, iz, dtx, dty, dtz, txn, tyn, tzn, ixs, iys, izs, ixe, iye, ize)) return true;
    while (true) {
      st.sl++;
      int64_t cidx = (int64_t)ix + (int64_t)nx * iy + (int64_t)nx * ny * iz;
      for (int64_t q = cell_start[cidx]; q < cell_start[cidx + 1]; q++) {
        st.sp++;
        Hit rec = hit_object((*objs)[cell_objs[q]], ray);
        if (rec.isHit && (double)rec.t < len) return true;
      }
      if (txn < tyn && txn < tzn) {
        txn += dtx; ix += ixs;
        if (ix == ixe) return false;
      } else {
        if (tyn < tzn) { tyn += dty; iy += iys; if (iy == iye) return false; }
        else { tzn += dtz; iz += izs; if (iz == ize) return false; }
      }
    }
  }
};

}  // namespace

// ------------------------------------------------------------------------------------------
// The scene object behind the C API.
// ------------------------------------------------------------------------------------------
struct orc_scene {
  std::vector<Object> objects;
  std::vector<Light> lights;
  std::vector<Material> materials;
  int cur_mat = -1;
  Camera cam;
  bool has_cam = false;
  C3 bg{0.f, 0.f, 0.f};
  uint32_t spp = 0;
  int accel = ORC_ACCEL_NONE;
  bool sky = false;
  std::string env;
  SkyFace faces[6];
  int faces_loaded = 0;
  BVH bvh;
  Grid grid;
  bool built = false;
  // per-render knobs
  int max_depth = 4;
  float roughness = 0.0f;
  int light_spp = 1;  // extension: shadow samples per quad light per hit (1 = main.cpp:391)

  void add_object(Object o) {
    o.mat = cur_mat;
    objects.push_back(o);
  }
  const Material& mat_of(int obj) const {
    static const Material dflt = default_material();
    int m = objects[obj].mat;
    return m < 0 ? dflt : materials[m];
  }

  C3 skybox_color(V3 dir) const;  // scene.cpp:380-458
  C3 background(const Ray& r) const { return sky ? skybox_color(r.d) : bg; }
  C3 ray_tracing(Ray ray, int depth, float ior_1, V3 ls, KRng& rng, Stats& st) const;  // main.cpp:294-521
};

namespace {

Object make_triangle(V3 p0, V3 p1, V3 p2) {  // scene.cpp:10-39
  Object o;
  o.type = ORC_OBJ_TRIANGLE;
  o.a = p0; o.b = p1; o.c = p2;
  V3 Min = mk(+FLT_MAX, +FLT_MAX, +FLT_MAX), Max = mk(-FLT_MAX, -FLT_MAX, -FLT_MAX);
  V3 pts[3] = {p0, p1, p2};
  for (auto& p : pts) {
    if (p.x < Min.x) Min.x = p.x;
    if (p.x > Max.x) Max.x = p.x;
    if (p.y < Min.y) Min.y = p.y;
    if (p.y > Max.y) Max.y = p.y;
    if (p.z < Min.z) Min.z = p.z;
    if (p.z > Max.z) Max.z = p.z;
  }
  const float e = (float)kEps;  // Vector::operator-=(const float) (vector.cpp:78)
  Min.x -= e; Min.y -= e; Min.z -= e;
  Max.x += e; Max.y += e; Max.z += e;
  o.box = AABB{Min, Max};
  return o;
}
Object make_sphere(V3 c, float r) {  // scene.h:157, scene.cpp:201-206
  Object o;
  o.type = ORC_OBJ_SPHERE;
  o.a = c; o.r = r;
  o.box = AABB{sub(c, mk(r, r, r)), add(c, mk(r, r, r))};
  return o;
}
Object make_plane_nd(V3 n, float d) {  // scene.cpp:96-98; default AABB (scene.h:116)
  Object o;
  o.type = ORC_OBJ_PLANE;
  o.a = n; o.D = d;
  o.box = default_aabb();
  return o;
}
Object make_plane_pts(V3 p0, V3 p1, V3 p2) {  // scene.cpp:100-114
  Object o;
  o.type = ORC_OBJ_PLANE;
  V3 pn = cross(sub(p1, p0), sub(p2, p0));
  float l = length(pn);
  if (l == 0.0) {
    std::cerr << "DEGENERATED PLANE!\n";
    o.a = pn; o.D = 0.0f;  // D is left uninitialised upstream
  } else {
    pn = normalize(pn);
    o.a = pn;
    o.D = -dot(pn, p0);
  }
  o.box = default_aabb();
  return o;
}
Object make_box(V3 mn, V3 mx) {  // scene.cpp:208-216
  Object o;
  o.type = ORC_OBJ_BOX;
  o.a = mn; o.b = mx;
  o.box = AABB{mn, mx};
  return o;
}

inline float u8tofloat(uint8_t x) { return (float)(x / 255.99f); }  // maths.h:133

}  // namespace

C3 orc_scene::skybox_color(V3 cc) const {  // scene.cpp:380-458
  float ma;
  int side;
  enum { RIGHT, LEFT, TOP, BOTTOM, FRONT, BACK };
  if (std::fabs(cc.x) > std::fabs(cc.y)) { ma = std::fabs(cc.x); side = cc.x >= 0 ? LEFT : RIGHT; }
  else { ma = std::fabs(cc.y); side = cc.y >= 0 ? TOP : BOTTOM; }
  if (std::fabs(cc.z) > ma) { ma = std::fabs(cc.z); side = cc.z >= 0 ? FRONT : BACK; }
  float sc = 0, tc = 0;
  switch (side) {
    case RIGHT: sc = -cc.z; tc = cc.y; break;
    case LEFT: sc = cc.z; tc = cc.y; break;
    case TOP: sc = -cc.x; tc = -cc.z; break;
    case BOTTOM: sc = -cc.x; tc = cc.z; break;
    case FRONT: sc = -cc.x; tc = cc.y; break;
    default: sc = cc.x; tc = cc.y; break;
  }
  double invMa = 1 / ma;  // int / float -> float division, widened
  float s = (float)((sc * invMa + 1) / 2);
  float t = (float)((tc * invMa + 1) / 2);
  const SkyFace& f = faces[side];
  if (f.img.empty()) return cmk(0, 0, 0);
  unsigned width = f.resX, height = f.resY, bpp = f.bpp;
  unsigned xp = (unsigned)(int)((float)(width - 1) * s);
  unsigned yp = (unsigned)(int)((float)(height - 1) * t);
  size_t base = ((size_t)yp * width + xp) * bpp;
  return cmk(u8tofloat(f.img[base]), u8tofloat(f.img[base + 1]), u8tofloat(f.img[base + 2]));
}

C3 orc_scene::ray_tracing(Ray ray, int depth, float ior_1, V3 lightSample, KRng& rng, Stats& st) const {
  // main.cpp:294-521
  C3 acc = cmk(0, 0, 0);
  int hitObj = -1;
  Hit closestHit;
  const int num_lights = (int)lights.size();
  const int num_objects = (int)objects.size();
  if (accel == ORC_ACCEL_NONE) {  // main.cpp:310-336
    for (int i = 0; i < num_objects; i++) {
      Hit aux = hit_object(objects[i], ray);
      if (aux.isHit && aux.t < closestHit.t) { closestHit = aux; hitObj = i; }
    }
    if (hitObj < 0) return cclamp(background(ray));
  } else if (accel == ORC_ACCEL_GRID) {  // main.cpp:339-347
    if (!grid.closest(ray, hitObj, closestHit, st)) return cclamp(background(ray));
    if (hitObj < 0) return cclamp(background(ray));  // upstream dereferences NULL here (grid.cpp:279)
  } else {  // main.cpp:350-358
    if (!bvh.closest(ray, hitObj, closestHit, st)) return cclamp(background(ray));
  }
  V3 hitPoint = add(ray.o, mul(ray.d, closestHit.t));  // main.cpp:361
  V3 N = normalize(closestHit.normal);
  bool outside = dot(ray.d, N) < 0.0f;
  if (!outside) N = neg(N);
  const Material& m = mat_of(hitObj);
  C3 diff_color = m.diff, spec_color = m.spec;
  float kr = m.refl, kd = m.kd, ks = m.ks, shine = m.shine, ior2 = m.ior, trans = m.T;
  ray.d = normalize(ray.d);  // `-ray.direction.normalize()` normalises in place (main.cpp:377)
  V3 V = neg(ray.d);
  const float offset = 1e-4f;
  V3 lightPos = mk(0, 0, 0);
  // light_spp extension: a quad light takes m = light_spp points
  // ((k % g + s.x) / g, (k / g + s.y) / g), g = floor(sqrt(m)), and each unshadowed term is
  // scaled by 1/m; m = 1 is the reference's loop exactly.
  int lgrid = 1;
  while ((lgrid + 1) * (lgrid + 1) <= light_spp) lgrid++;
  const float linv = 1.0f / (float)light_spp;
  for (int j = 0; j < num_lights; j++)  // main.cpp:383-451
  for (int k = 0; k < (lights[j].quad ? light_spp : 1); k++) {
    const Light& light = lights[j];
    V3 ls = lightSample;
    if (light.quad && light_spp > 1)
      ls = mk(((float)(k % lgrid) + lightSample.x) / (float)lgrid, ((float)(k / lgrid) + lightSample.y) / (float)lgrid,
              0.0f);
    if (light.quad) lightPos = light.area_point(ls);
    else lightPos = light.pos;
    V3 L = sub(lightPos, hitPoint);
    V3 Ls = L;
    L = normalize(L);
    V3 H = normalize(add(L, V));
    float NdotL = smax(dot(N, L), 0.0f);
    float NdotH = smax(dot(N, H), 0.0f);
    V3 shadowDir = (accel == ORC_ACCEL_BVH) ? Ls : L;  // main.cpp:411-420 (GRID falls to the else)
    Ray shadowRay{add(hitPoint, mul(N, offset)), shadowDir};
    bool inShadow = false;
    if (accel == ORC_ACCEL_GRID) inShadow = grid.shadow(shadowRay, st);
    else if (accel == ORC_ACCEL_BVH) inShadow = bvh.shadow(shadowRay, st);
    else {
      for (int o = 0; o < num_objects; o++) {
        if (o == hitObj) continue;
        Hit sh = hit_object(objects[o], shadowRay);
        if (sh.isHit && sh.t > offset && sh.t < length(L)) { inShadow = true; break; }
      }
    }
    if (!inShadow) {
      C3 diffuseTerm = cmul(cmul(diff_color, kd), NdotL);
      C3 specularTerm = cmul(cmul(spec_color, ks), std::pow(NdotH, shine));  // std::pow(float,float) = powf
      C3 term = cadd(diffuseTerm, specularTerm);
      if (light.quad && light_spp > 1) term = cmul(term, linv);
      acc = cadd(acc, term);
    }
  }
  if (depth > max_depth) return acc;  // main.cpp:454 (unclamped)
  float kr_fresnel = kr;
  if (!outside) ior2 = 1.0;
  float eta = ior_1 / ior2;
  V3 Vt = sub(mul(N, dot(V, N)), V);
  float sin_i = length(Vt);
  V3 t = dvf(Vt, length(Vt));
  float sin_t = eta * sin_i;
  if (trans == 1 && sin_t < 1) {  // main.cpp:465-498
    float sin_t2 = (float)std::pow((double)sin_t, 2.0);
    float cos_t = std::sqrt(1 - sin_t2);
    V3 r_t = normalize(add(mul(t, sin_t), mul(neg(N), cos_t)));
    float cos_i = dot(N, V);
    float cosTheta = (ior_1 > ior2) ? cos_t : cos_i;
    float r0 = (ior_1 - ior2) / (ior_1 + ior2);
    r0 = (float)std::pow((double)r0, 2.0);
    kr_fresnel = (float)((double)r0 + (double)(1.0f - r0) * std::pow((double)(1.0f - cosTheta), 5.0));
    Ray refractRay{sub(hitPoint, mul(N, offset)), r_t};
    C3 refractColor = cclamp(ray_tracing(refractRay, depth + 1, ior2, lightPos, rng, st));
    if (!outside) {
      C3 one = cmk(1.0f, 1.0f, 1.0f);
      refractColor = cmulc(refractColor, cexp(cmul(csub(one, diff_color), -closestHit.t)));
    }
    acc = cadd(acc, cmul(refractColor, 1 - kr_fresnel));
  } else if (trans > 0.0f && sin_t >= 1) {
    kr_fresnel = 1;
  }
  if (ks > 0) {  // main.cpp:504-518
    V3 reflectDir = sub(mul(mul(N, dot(V, N)), 2.0f), V);
    V3 sph = rnd_unit_sphere(rng);
    reflectDir = normalize(add(reflectDir, mul(sph, roughness)));
    Ray reflectRay{add(hitPoint, mul(N, offset)), reflectDir};
    C3 reflectColor = cclamp(ray_tracing(reflectRay, depth + 1, ior_1, lightPos, rng, st));
    float k_ref = kr_fresnel;
    if (dot(reflectDir, N) > 0) acc = cadd(acc, cmulc(cmul(reflectColor, k_ref), spec_color));
  }
  return cclamp(acc);
}

// ==========================================================================================
// C API
// ==========================================================================================
extern "C" {

// The first n draws of the CRT rand() sequence orc_options.lcg uses (MSVC: srand(seed), then rand()).
void orc_crt_rand(uint32_t seed, int n, int32_t* out) {
  uint32_t state = seed;
  KRng g{0, 0, 0};
  g.lcg = &state;
  for (int i = 0; i < n; i++) out[i] = g.rand_();
}

uint32_t orc_keyed_rand(uint32_t seed, uint32_t pixel, uint32_t k) {
  KRng g{seed, pixel, k};
  return (uint32_t)g.rand_();
}

orc_scene* orc_scene_new(void) { return new orc_scene(); }
void orc_scene_free(orc_scene* s) { delete s; }

static V3 v3p(const float* p) { return mk(p[0], p[1], p[2]); }

int orc_scene_set_camera(orc_scene* s, const float eye[3], const float at[3], const float up[3], float fovy,
                         float hither, int rx, int ry, float ap, float fr) {
  s->cam.init(v3p(eye), v3p(at), v3p(up), fovy, hither, (float)(1000.0 * hither), rx, ry, ap, fr);
  s->has_cam = true;
  return 0;
}
int orc_scene_set_background(orc_scene* s, const float rgb[3]) { s->bg = cmk(rgb[0], rgb[1], rgb[2]); return 0; }
int orc_scene_set_accel(orc_scene* s, int a) { s->accel = a; s->built = false; return 0; }
int orc_scene_set_spp(orc_scene* s, uint32_t spp) { s->spp = spp; return 0; }
int orc_scene_add_material(orc_scene* s, const float d[3], double kd, const float sp[3], double ks, double shine,
                           double t, double ior) {
  Material m;
  m.diff = cmk(d[0], d[1], d[2]);
  m.kd = (float)kd;
  m.spec = cmk(sp[0], sp[1], sp[2]);
  m.ks = (float)ks;
  m.shine = (float)shine;
  m.refl = (float)ks;
  m.T = (float)t;
  m.ior = (float)ior;
  s->materials.push_back(m);
  s->cur_mat = (int)s->materials.size() - 1;
  return s->cur_mat;
}
int orc_scene_use_material(orc_scene* s, int m) { s->cur_mat = m; return 0; }
int orc_scene_add_sphere(orc_scene* s, const float c[3], float r) { s->add_object(make_sphere(v3p(c), r)); s->built = false; return (int)s->objects.size() - 1; }
int orc_scene_add_triangle(orc_scene* s, const float a[3], const float b[3], const float c[3]) {
  s->add_object(make_triangle(v3p(a), v3p(b), v3p(c)));
  s->built = false;
  return (int)s->objects.size() - 1;
}
int orc_scene_add_triangles(orc_scene* s, const float* v, int n) {
  s->objects.reserve(s->objects.size() + n);
  for (int i = 0; i < n; i++) s->add_object(make_triangle(v3p(v + 9 * i), v3p(v + 9 * i + 3), v3p(v + 9 * i + 6)));
  s->built = false;
  return (int)s->objects.size() - 1;
}
int orc_scene_add_plane_pts(orc_scene* s, const float a[3], const float b[3], const float c[3]) {
  s->add_object(make_plane_pts(v3p(a), v3p(b), v3p(c)));
  s->built = false;
  return (int)s->objects.size() - 1;
}
int orc_scene_add_plane_nd(orc_scene* s, const float n[3], float d) { s->add_object(make_plane_nd(v3p(n), d)); s->built = false; return (int)s->objects.size() - 1; }
int orc_scene_add_box(orc_scene* s, const float a[3], const float b[3]) { s->add_object(make_box(v3p(a), v3p(b))); s->built = false; return (int)s->objects.size() - 1; }
int orc_scene_add_light_point(orc_scene* s, const float p[3], const float c[3]) {  // scene.h:97
  Light l;
  l.quad = 0; l.pos = v3p(p); l.emission = cmk(c[0], c[1], c[2]);
  s->lights.push_back(l);
  return (int)s->lights.size() - 1;
}
int orc_scene_add_light_quad(orc_scene* s, const float p[3], const float c[3], const float v1[3], const float v2[3],
                             uint32_t g) {  // scene.h:84-95
  Light l;
  l.quad = 1; l.pos = v3p(p); l.emission = cmk(c[0], c[1], c[2]); l.gridRes = g;
  l.e1 = sub(v3p(v1), l.pos);
  l.e2 = sub(v3p(v2), l.pos);
  s->lights.push_back(l);
  return (int)s->lights.size() - 1;
}

int orc_scene_set_skybox_face(orc_scene* s, int face, int w, int h, int bpp, const uint8_t* px) {
  if (face < 0 || face > 5 || w <= 0 || h <= 0 || (bpp != 3 && bpp != 4)) return -1;
  SkyFace& f = s->faces[face];
  f.resX = w; f.resY = h; f.bpp = bpp;
  f.img.assign(px, px + (size_t)w * h * bpp);
  int n = 0;
  for (auto& ff : s->faces) n += !ff.img.empty();
  s->faces_loaded = n;
  return 0;
}

const char* orc_scene_env(const orc_scene* s) { return s->env.c_str(); }

int orc_scene_info(const orc_scene* s, orc_info* o) {
  o->res_x = s->cam.res_x; o->res_y = s->cam.res_y; o->spp = s->spp; o->accel = s->accel;
  o->n_objects = (int)s->objects.size(); o->n_lights = (int)s->lights.size();
  o->n_materials = (int)s->materials.size();
  o->has_env = s->sky ? 1 : 0;
  o->skybox_loaded = s->faces_loaded == 6;
  o->aperture = s->cam.aperture;
  return 0;
}

// P3F loader (scene.cpp:466-740), iostream-based exactly like the reference.
orc_scene* orc_scene_load_p3f(const char* name) {
  std::ifstream file(name, std::ios::in);
  if (!file) return nullptr;
  orc_scene* s = new orc_scene();
  std::string cmd;
  char token[256];
  auto next_token = [&](const char* nm) {  // scene.cpp:466
    file >> token;
    if (strcmp(token, nm)) std::cerr << "'" << nm << "' expected.\n";
  };
  auto rv = [&](V3& v) { file >> v.x >> v.y >> v.z; };
  auto rc = [&](C3& c) { file >> c.r >> c.g >> c.b; };
  if (file >> cmd) {
    while (true) {
      if (cmd == "accel") {
        std::string t;
        file >> t;
        if (t == "none") s->accel = ORC_ACCEL_NONE;
        else if (t == "grid") s->accel = ORC_ACCEL_GRID;
        else if (t == "bvh") s->accel = ORC_ACCEL_BVH;
        else { printf("Unsupported acceleration type\n"); break; }
      } else if (cmd == "spp") {
        unsigned spp; file >> spp; s->spp = spp;
      } else if (cmd == "mat") {
        double Kd, Ks, Shine, T, ior;
        C3 cd, cs;
        rc(cd); file >> Kd; rc(cs); file >> Ks >> Shine >> T >> ior;
        float d3[3] = {cd.r, cd.g, cd.b}, s3[3] = {cs.r, cs.g, cs.b};
        orc_scene_add_material(s, d3, Kd, s3, Ks, Shine, T, ior);
      } else if (cmd == "s") {
        V3 c; float r; rv(c); file >> r;
        s->add_object(make_sphere(c, r));
      } else if (cmd == "box") {
        V3 a, b; rv(a); rv(b);
        s->add_object(make_box(a, b));
      } else if (cmd == "p") {
        unsigned tv; file >> tv;
        if (tv == 3) { V3 a, b, c; rv(a); rv(b); rv(c); s->add_object(make_triangle(a, b, c)); }
        else { std::cerr << "Unsupported number of vertices.\n"; break; }
      } else if (cmd == "mesh") {
        unsigned tv, tf, P0, P1, P2;
        file >> tv >> tf;
        std::vector<V3> verts(tv);
        for (unsigned i = 0; i < tv; i++) { V3 v; rv(v); verts[i] = v; }
        s->objects.reserve(s->objects.size() + tf);
        for (unsigned i = 0; i < tf; i++) {
          file >> P0 >> P1 >> P2;
          if (P0 > 0) { P0 -= 1; P1 -= 1; P2 -= 1; }
          else { P0 += tv; P1 += tv; P2 += tv; }
          if (P0 >= tv || P1 >= tv || P2 >= tv) { std::cerr << "mesh index out of range\n"; break; }
          s->add_object(make_triangle(verts[P0], verts[P1], verts[P2]));
        }
      } else if (cmd == "npl") {
        V3 n; float d; rv(n); file >> d;
        s->add_object(make_plane_nd(n, d));
      } else if (cmd == "pl") {
        V3 a, b, c; rv(a); rv(b); rv(c);
        s->add_object(make_plane_pts(a, b, c));
      } else if (cmd == "light") {
        V3 pos; C3 col; V3 v1, v2; unsigned g;
        std::string type;
        file >> type;
        if (type == "punctual") {
          rv(pos); rc(col);
          float p3[3] = {pos.x, pos.y, pos.z}, c3[3] = {col.r, col.g, col.b};
          orc_scene_add_light_point(s, p3, c3);
        } else if (type == "quad") {
          rv(pos); rc(col); rv(v1); rv(v2); file >> g;
          float p3[3] = {pos.x, pos.y, pos.z}, c3[3] = {col.r, col.g, col.b}, a3[3] = {v1.x, v1.y, v1.z},
                b3[3] = {v2.x, v2.y, v2.z};
          orc_scene_add_light_quad(s, p3, c3, a3, b3, g);
        } else { std::cerr << "Unsupported light type.\n"; break; }
      } else if (cmd == "camera") {
        V3 up, from, at; float fov, hither; int xres, yres; float fr, ar;
        next_token("eye"); rv(from);
        next_token("at"); rv(at);
        next_token("up"); rv(up);
        next_token("angle"); file >> fov;
        next_token("hither"); file >> hither;
        next_token("resolution"); file >> xres >> yres;
        next_token("aperture"); file >> ar;
        next_token("focal"); file >> fr;
        s->cam.init(from, at, up, fov, hither, (float)(1000.0 * hither), xres, yres, ar, fr);
        s->has_cam = true;
      } else if (cmd == "bclr") {
        C3 c; rc(c); s->bg = c;
      } else if (cmd == "env") {
        file >> token;
        s->env = token;
        s->sky = true;
      } else if (cmd[0] == '#') {
        file.ignore(1024, '\n');
      } else {
        std::cerr << "unknown command '" << cmd << "'.\n";
        break;
      }
      if (!(file >> cmd)) break;
    }
  }
  return s;
}

int orc_scene_build(orc_scene* s) {  // main.cpp:1023-1049
  if (s->accel == ORC_ACCEL_GRID) s->grid.build(s->objects);
  else if (s->accel == ORC_ACCEL_BVH) s->bvh.build(s->objects);
  s->built = true;
  return 0;
}

int orc_bvh_num_nodes(const orc_scene* s) { return (int)s->bvh.nodes.size(); }
int orc_bvh_export(const orc_scene* s, float* boxes, uint32_t* leaf, uint32_t* index, uint32_t* nobjs,
                   int32_t* order) {
  const auto& nd = s->bvh.nodes;
  for (size_t i = 0; i < nd.size(); i++) {
    const AABB& b = nd[i].box;
    float* o = boxes + 6 * i;
    o[0] = b.mn.x; o[1] = b.mn.y; o[2] = b.mn.z; o[3] = b.mx.x; o[4] = b.mx.y; o[5] = b.mx.z;
    leaf[i] = nd[i].leaf; index[i] = nd[i].index; nobjs[i] = nd[i].leaf ? nd[i].n_objs : 0;
  }
  for (size_t i = 0; i < s->bvh.objects.size(); i++) order[i] = s->bvh.objects[i];
  return 0;
}
int orc_grid_export_dims(const orc_scene* s, int dims[3], float bmin[3], float bmax[3], int64_t* n_refs) {
  const Grid& g = s->grid;
  dims[0] = g.nx; dims[1] = g.ny; dims[2] = g.nz;
  bmin[0] = g.bbox.mn.x; bmin[1] = g.bbox.mn.y; bmin[2] = g.bbox.mn.z;
  bmax[0] = g.bbox.mx.x; bmax[1] = g.bbox.mx.y; bmax[2] = g.bbox.mx.z;
  *n_refs = (int64_t)g.cell_objs.size();
  return 0;
}
int orc_grid_export(const orc_scene* s, int64_t* cs, int32_t* co) {
  std::copy(s->grid.cell_start.begin(), s->grid.cell_start.end(), cs);
  std::copy(s->grid.cell_objs.begin(), s->grid.cell_objs.end(), co);
  return 0;
}

static bool closest_any(const orc_scene* s, const Ray& r, int& obj, Hit& h, Stats& st) {
  obj = -1;
  h = Hit();
  if (s->accel == ORC_ACCEL_BVH) return s->bvh.closest(r, obj, h, st);
  if (s->accel == ORC_ACCEL_GRID) return s->grid.closest(r, obj, h, st);
  for (int i = 0; i < (int)s->objects.size(); i++) {
    Hit a = hit_object(s->objects[i], r);
    if (a.isHit && a.t < h.t) { h = a; obj = i; }
  }
  return obj >= 0;
}

int orc_trace_closest(orc_scene* s, const float* rays, int n, float* t, float* nrm, int32_t* obj) {
  if (!s->built) orc_scene_build(s);
#pragma omp parallel for schedule(dynamic, 256)
  for (int i = 0; i < n; i++) {
    Ray r{v3p(rays + 6 * i), v3p(rays + 6 * i + 3)};
    Stats st;
    int o;
    Hit h;
    bool hit = closest_any(s, r, o, h, st);
    t[i] = hit ? h.t : FLT_MAX;
    nrm[3 * i] = hit ? h.normal.x : 0.f; nrm[3 * i + 1] = hit ? h.normal.y : 0.f; nrm[3 * i + 2] = hit ? h.normal.z : 0.f;
    obj[i] = hit ? o : -1;
  }
  return 0;
}

int orc_trace_shadow(orc_scene* s, const float* rays, int n, uint8_t* occ) {
  if (!s->built) orc_scene_build(s);
#pragma omp parallel for schedule(dynamic, 256)
  for (int i = 0; i < n; i++) {
    Ray r{v3p(rays + 6 * i), v3p(rays + 6 * i + 3)};
    Stats st;
    bool o;
    if (s->accel == ORC_ACCEL_BVH) o = s->bvh.shadow(r, st);
    else if (s->accel == ORC_ACCEL_GRID) o = s->grid.shadow(r, st);
    else {  // NONE: main.cpp:432-439 without the self-skip (no hit object in a raw query), range = |d|
      o = false;
      float len = length(r.d);
      for (auto& ob : s->objects) {
        Hit h = hit_object(ob, r);
        if (h.isHit && h.t > 1e-4f && h.t < len) { o = true; break; }
      }
    }
    occ[i] = o ? 1 : 0;
  }
  return 0;
}

int orc_object_hit(orc_scene* s, int obj, const float* rays, int n, float* t, float* nrm, uint8_t* ishit) {
  if (obj < 0 || obj >= (int)s->objects.size()) return -1;
  for (int i = 0; i < n; i++) {
    Ray r{v3p(rays + 6 * i), v3p(rays + 6 * i + 3)};
    Hit h = hit_object(s->objects[obj], r);
    t[i] = h.t; ishit[i] = h.isHit;
    nrm[3 * i] = h.normal.x; nrm[3 * i + 1] = h.normal.y; nrm[3 * i + 2] = h.normal.z;
  }
  return 0;
}

int orc_object_bbox(const orc_scene* s, int obj, float out[6]) {
  if (obj < 0 || obj >= (int)s->objects.size()) return -1;
  const AABB& b = s->objects[obj].box;
  out[0] = b.mn.x; out[1] = b.mn.y; out[2] = b.mn.z; out[3] = b.mx.x; out[4] = b.mx.y; out[5] = b.mx.z;
  return 0;
}

int orc_rnd(uint32_t seed, uint32_t pix, int n, int sphere, int glibc_rand_max, float* out, uint32_t* calls) {
  KRng g{seed, pix, 0};
  if (glibc_rand_max) { g.shift = 1; g.rmax = 0x7FFFFFFF; }
  for (int i = 0; i < n; i++) {
    uint32_t k0 = g.k;
    V3 p = sphere ? rnd_unit_sphere(g) : rnd_unit_disk(g);
    out[3 * i] = p.x; out[3 * i + 1] = p.y; out[3 * i + 2] = p.z;
    calls[i] = g.k - k0;
  }
  return 0;
}

int orc_aabb_hit(const float* boxes, const float* rays, int n, uint8_t* hit, float* t, uint8_t* inside) {
  for (int i = 0; i < n; i++) {
    AABB b{v3p(boxes + 6 * i), v3p(boxes + 6 * i + 3)};
    Ray r{v3p(rays + 6 * i), v3p(rays + 6 * i + 3)};
    float tt = 0;
    hit[i] = aabb_hit(b, r, tt) ? 1 : 0;
    t[i] = tt;
    inside[i] = aabb_inside(b, r.o) ? 1 : 0;
  }
  return 0;
}

int orc_scene_set_eye(orc_scene* s, const float eye[3]) {  // Camera::SetEye (camera.h:63-72)
  if (!s->has_cam) return -1;
  s->cam.set_eye(v3p(eye));
  return 0;
}

int orc_camera_frame(const orc_scene* s, float* frame) {
  const Camera& c = s->cam;
  frame[0] = c.plane_dist; frame[1] = c.aperture; frame[2] = c.w; frame[3] = c.h;
  frame[4] = c.u.x; frame[5] = c.u.y; frame[6] = c.u.z;
  frame[7] = c.v.x; frame[8] = c.v.y; frame[9] = c.v.z;
  frame[10] = c.n.x; frame[11] = c.n.y; frame[12] = c.n.z;
  return 0;
}

int orc_light_points(const orc_scene* s, int light, const float* smp, int n, float* out) {
  if (light < 0 || light >= (int)s->lights.size()) return -1;
  for (int i = 0; i < n; i++) {
    V3 q = s->lights[light].area_point(v3p(smp + 3 * i));
    out[3 * i] = q.x; out[3 * i + 1] = q.y; out[3 * i + 2] = q.z;
  }
  return 0;
}

int orc_vector_ops(const float* a, const float* b, int n, float* nrm, float* len, float* crs, float* dotv) {
  for (int i = 0; i < n; i++) {
    V3 u = v3p(a + 3 * i), v = v3p(b + 3 * i);
    len[i] = length(u);
    dotv[i] = dot(u, v);
    V3 c = cross(u, v);
    crs[3 * i] = c.x; crs[3 * i + 1] = c.y; crs[3 * i + 2] = c.z;
    V3 w = normalize(u);
    nrm[3 * i] = w.x; nrm[3 * i + 1] = w.y; nrm[3 * i + 2] = w.z;
  }
  return 0;
}

int orc_color_ops(const float* c, int n, float* clamped, float* ex, uint8_t* u8) {
  for (int i = 0; i < n; i++) {
    C3 k = cmk(c[3 * i], c[3 * i + 1], c[3 * i + 2]);
    C3 a = cclamp(k), e = cexp(k);
    clamped[3 * i] = a.r; clamped[3 * i + 1] = a.g; clamped[3 * i + 2] = a.b;
    ex[3 * i] = e.r; ex[3 * i + 1] = e.g; ex[3 * i + 2] = e.b;
    for (int q = 0; q < 3; q++) {  // maths.h:126-130
      float x = c[3 * i + q];
      u8[3 * i + q] = ((x * 255.99f) >= 255.0f ? 255 : (uint8_t)(x * 255.99f));
    }
  }
  return 0;
}

int orc_primary_rays(const orc_scene* s, const float* smp, int n, int dof, float* rays) {
  for (int i = 0; i < n; i++) {
    V3 ps = mk(smp[4 * i], smp[4 * i + 1], 0.0f);
    V3 lens = mk(smp[4 * i + 2], smp[4 * i + 3], 0.0f);
    Ray r = dof ? s->cam.primary_lens(lens, ps) : s->cam.primary(ps);
    float* o = rays + 6 * i;
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z; o[3] = r.d.x; o[4] = r.d.y; o[5] = r.d.z;
  }
  return 0;
}

int orc_skybox_color(const orc_scene* s, const float* d, int n, float* rgb) {
  for (int i = 0; i < n; i++) {
    C3 c = s->skybox_color(v3p(d + 3 * i));
    rgb[3 * i] = c.r; rgb[3 * i + 1] = c.g; rgb[3 * i + 2] = c.b;
  }
  return 0;
}

int orc_ray_color(orc_scene* s, const float* rays, const float* ls, int n, int depth, float ior, uint32_t seed,
                  uint32_t pixel, float* rgb) {
  if (!s->built) orc_scene_build(s);
  Stats st;
  KRng g{seed, pixel, 0};
  for (int i = 0; i < n; i++) {
    Ray r{v3p(rays + 6 * i), v3p(rays + 6 * i + 3)};
    C3 c = s->ray_tracing(r, depth, ior, v3p(ls + 3 * i), g, st);
    rgb[3 * i] = c.r; rgb[3 * i + 1] = c.g; rgb[3 * i + 2] = c.b;
  }
  return 0;
}

// renderScene zone B (main.cpp:603-721) with the keyed RNG, one pixel = one RNG stream.
int orc_render(orc_scene* s, uint32_t seed, const orc_options* opt, float* rgb, orc_stats* out_stats) {
  if (!s->has_cam) return -1;
  if (!s->built) orc_scene_build(s);
  s->max_depth = opt ? opt->max_depth : 4;
  s->roughness = opt ? opt->roughness : 0.0f;
  s->light_spp = (opt && opt->light_spp > 1) ? opt->light_spp : 1;
  const int RX = s->cam.res_x, RY = s->cam.res_y;
  int y0 = 0, y1 = RY;
  if (opt && opt->row_end > opt->row_begin) { y0 = std::max(0, opt->row_begin); y1 = std::min(RY, opt->row_end); }
  const uint32_t spp = s->spp;
  const bool AA = spp != 0;                                // main.cpp:1005-1010
  const bool DOF = (s->cam.aperture != 0) && AA;           // main.cpp:1013-1017
  const long prog = opt ? opt->progressive_frame : 0;      // FrameCount of zone A, 0 = zone B
  if (prog >= 10000) return 0;                             // FrameCount == MAX_SAMPLES: no render (main.cpp:537)
  int threads = (opt && opt->threads > 0) ? opt->threads : 0;
  const bool lcg = opt && opt->lcg;  // one CRT rand() sequence in pixel order: one thread
  uint32_t lcg_state = lcg ? opt->lcg_seed : 0u;
  if (lcg) threads = 1;
#ifdef _OPENMP
  int nthr = threads > 0 ? threads : omp_get_max_threads();
#else
  int nthr = 1;
#endif
  std::vector<Stats> tst((size_t)nthr);
  const int64_t npx = (int64_t)(y1 - y0) * RX;
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthr)
  for (int64_t q = 0; q < npx; q++) {
    int y = y0 + (int)(q / RX), x = (int)(q % RX);
#ifdef _OPENMP
    Stats& st = tst[(size_t)omp_get_thread_num()];
#else
    Stats& st = tst[0];
#endif
    KRng g{seed, (uint32_t)(y * RX + x), 0};
    if (lcg) g.lcg = &lcg_state;
    C3 color = cmk(0, 0, 0);
    if (prog > 0) {  // zone A (main.cpp:540-586): one jittered sample, lerped into the frame
      V3 ps;
      ps.x = (float)((double)x + (double)g.rand_() / ((double)kRandMax + 1.0));  // rand_double (maths.h:88)
      ps.y = (float)((double)y + (double)g.rand_() / ((double)kRandMax + 1.0));
      ps.z = 0.0f;
      Ray ray;
      if (!DOF) ray = s->cam.primary(ps);
      else ray = s->cam.primary_lens(dvf(mul(rnd_unit_disk(g), s->cam.aperture), 2.0f), ps);
      const float ly = g.rand_float();  // Vector(rand_float(), rand_float(), 0.0f): right to left
      const float lx = g.rand_float();
      st.samples++;
      color = s->ray_tracing(ray, 1, 1.0f, mk(lx, ly, 0.0f), g, st);
      size_t ic = (size_t)3 * ((size_t)x + (size_t)RX * y);
      const float c3[3] = {color.r, color.g, color.b};
      for (int k = 0; k < 3; k++)  // lerp(a, b, t) = a + t * (b - a) in double (maths.h:56)
        rgb[ic + k] = prog == 1 ? c3[k] : (float)((double)rgb[ic + k] + (1.0 / (double)prog) *
                                                                       ((double)c3[k] - (double)rgb[ic + k]));
      continue;
    }
    if (AA) {  // main.cpp:618-671
      int n = (int)std::sqrt((double)spp);
      std::vector<V3> r(spp), sm(spp);
      for (int p = 0; p < (int)spp; p++) {
        int row = p / n, col = p % n;
        float ex = (float)g.rand_() / (float)kRandMax;
        float ey = (float)g.rand_() / (float)kRandMax;
        r[p] = mk((col + ex) / n, (row + ey) / n, 0.0f);
        ex = (float)g.rand_() / (float)kRandMax;
        ey = (float)g.rand_() / (float)kRandMax;
        sm[p] = mk(ex, ey, 0.0f);
      }
      for (int i = (int)spp - 1; i > 0; i--) {
        int j = g.rand_() % (i + 1);
        std::swap(sm[i], sm[j]);
      }
      for (int p = 0; p < (int)spp; p++) {
        V3 ps = mk(x + r[p].x, y + r[p].y, 0.0f);
        Ray ray;
        if (!DOF) ray = s->cam.primary(ps);
        else {
          V3 lens = dvf(mul(rnd_unit_disk(g), s->cam.aperture), 2.0f);
          ray = s->cam.primary_lens(lens, ps);
        }
        st.samples++;
        color = cadd(color, s->ray_tracing(ray, 1, 1.0f, sm[p], g, st));
      }
      color = cmul(color, (float)(1.0 / ((float)spp)));
    } else {  // main.cpp:674-703
      V3 ps = mk(x + 0.5f, y + 0.5f, 0.0f);
      Ray ray1 = s->cam.primary(ps);
      const Light* light = s->lights.empty() ? nullptr : &s->lights[0];
      if (light && light->quad) {
        const int lightSamples = (int)light->gridRes;
        C3 temp = cmk(0, 0, 0);
        for (int k = 0; k < lightSamples; k++) {
          int gs = (int)std::sqrt((double)lightSamples);
          float u = (k % gs + 0.5f) / gs;
          float v = (k / gs + 0.5f) / gs;
          st.samples++;
          temp = cadd(temp, s->ray_tracing(ray1, 1, 1.0f, mk(u, v, 0.0f), g, st));
        }
        color = cmul(temp, 1.0f / lightSamples);
      } else {
        st.samples++;
        color = s->ray_tracing(ray1, 1, 1.0f, mk(0.5f, 0.5f, 0.0f), g, st);
      }
    }
    size_t ic = (size_t)3 * ((size_t)x + (size_t)RX * y);
    rgb[ic] = color.r; rgb[ic + 1] = color.g; rgb[ic + 2] = color.b;
  }
  if (out_stats) {
    Stats t;
    for (auto& a : tst) {
      t.cc += a.cc; t.sc += a.sc; t.ci += a.ci; t.cl += a.cl; t.si += a.si; t.sl += a.sl; t.cp += a.cp; t.sp += a.sp;
      t.samples += a.samples;
    }
    out_stats->closest_calls = t.cc; out_stats->shadow_calls = t.sc;
    out_stats->closest_inner = t.ci; out_stats->closest_leaf = t.cl;
    out_stats->shadow_inner = t.si; out_stats->shadow_leaf = t.sl;
    out_stats->closest_prims = t.cp; out_stats->shadow_prims = t.sp;
    out_stats->samples = t.samples;
  }
  return 0;
}

}  // extern "C"
