// drt_cpu.cpp — the scalar host path of the C++ API (include/drt_scene.hpp): AABB tests, the
// primitives' hit(), Camera::PrimaryRay, Scene::GetSkyboxColor / LoadSkybox, and the CPU
// BVH::Traverse / Grid::Traverse.  One ray at a time, no device: what the reference's own
// callers and tests use ("a scalar Traverse stays for CPU use and tests"); frames
// and batched queries run on the GPU (include/drt.h).
//
// Every expression keeps the reference's operand order and float/double promotions (compiled
// with -ffp-contract=off), so results are bit-identical to the reference's functions cited below
// (tests/test_cpp_api.py checks them against the reference-produced goldens and the oracle).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/drt_host.h"
#include "../../../include/drt_scene.hpp"

namespace drt {

static constexpr double kEps = 0.001;  // macros.h:1 (a double)

static inline float max3(float a, float b, float c) { return (a > b) ? ((a > c) ? a : c) : ((b > c) ? b : c); }  // macros.h:8
static inline float min3(float a, float b, float c) { return (a < b) ? ((a < c) ? a : c) : ((b < c) ? b : c); }  // macros.h:5
static inline double dclamp(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }           // maths.h:65

// ---------------------------------------------------------------- AABB (boundingBox.cpp)
bool AABB::isInside(const Vector& p) const {  // boundingBox.cpp:41-44
  return ((p.x > min.x && p.x < max.x) && (p.y > min.y && p.y < max.y) && (p.z > min.z && p.z < max.z));
}

bool AABB::hit(const Ray& r, float& t) const {  // boundingBox.cpp:64-124
  const float ox = r.origin.x, oy = r.origin.y, oz = r.origin.z;
  const float dx = r.direction.x, dy = r.direction.y, dz = r.direction.z;
  float txmin, tymin, tzmin, txmax, tymax, tzmax;
  const float a = (float)(1.0 / dx);
  if (a >= 0) { txmin = (min.x - ox) * a; txmax = (max.x - ox) * a; }
  else { txmin = (max.x - ox) * a; txmax = (min.x - ox) * a; }
  const float b = (float)(1.0 / dy);
  if (b >= 0) { tymin = (min.y - oy) * b; tymax = (max.y - oy) * b; }
  else { tymin = (max.y - oy) * b; tymax = (min.y - oy) * b; }
  const float c = (float)(1.0 / dz);
  if (c >= 0) { tzmin = (min.z - oz) * c; tzmax = (max.z - oz) * c; }
  else { tzmin = (max.z - oz) * c; tzmax = (min.z - oz) * c; }
  const double t0 = max3(txmin, tymin, tzmin);
  const double t1 = min3(txmax, tymax, tzmax);
  t = (float)((t0 < 0) ? t1 : t0);
  return (t0 < t1 && t1 > 0);
}

// ---------------------------------------------------------------- primitives (scene.cpp)
HitRecord Triangle::hit(const Ray& r) const {  // scene.cpp:44-92 (Moller-Trumbore, no parallel test)
  HitRecord rec;
  const Vector e1 = points[1] - points[0], e2 = points[2] - points[0];
  const Vector h = r.direction % e2;
  const float a = e1 * h;
  const float f = 1.0f / a;
  const Vector s = r.origin - points[0];
  const float u = f * (s * h);
  if (u < 0.0 || u > 1.0) return rec;
  const Vector q = s % e1;
  const float v = f * (r.direction * q);
  if (v < 0.0 || u + v > 1.0) return rec;
  const float t = f * (e2 * q);
  if ((double)t > kEps) {
    rec.t = t;
    rec.isHit = true;
    rec.normal = (e1 % e2).normalize();
  }
  return rec;
}

HitRecord Plane::hit(const Ray& r) const {  // scene.cpp:118-149
  HitRecord rec;
  const float pnrd = PN * r.direction;
  if (std::fabs(pnrd) < kEps) return rec;
  const float t = -((PN * r.origin) + D) / pnrd;
  if (t > 0) {
    rec.t = t;
    rec.normal = PN;
    rec.isHit = true;
  }
  return rec;
}

HitRecord Sphere::hit(const Ray& r) const {  // scene.cpp:152-197 (the motion-blur branch is dead)
  HitRecord rec;
  const Vector oc = r.origin - center;
  const float a = r.direction * r.direction;
  const float b = 2.0f * (oc * r.direction);
  const float c = (oc * oc) - radius * radius;
  const float disc = b * b - 4 * a * c;
  if (disc < 0) return rec;
  const float sq = std::sqrt(disc);
  const float t1 = (-b - sq) / (2.0f * a);
  const float t2 = (-b + sq) / (2.0f * a);
  if ((double)t1 > kEps) rec.t = t1;
  else if ((double)t2 > kEps) rec.t = t2;
  else return rec;
  rec.isHit = true;
  rec.normal = ((r.origin + r.direction * rec.t) - center).normalize();
  return rec;
}

HitRecord aaBox::hit(const Ray& ray) const {  // scene.cpp:218-278
  HitRecord rec;
  float tmin = (min.x - ray.origin.x) / ray.direction.x;
  float tmax = (max.x - ray.origin.x) / ray.direction.x;
  if (tmin > tmax) std::swap(tmin, tmax);
  float tymin = (min.y - ray.origin.y) / ray.direction.y;
  float tymax = (max.y - ray.origin.y) / ray.direction.y;
  if (tymin > tymax) std::swap(tymin, tymax);
  if ((tmin > tymax) || (tymin > tmax)) return rec;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  float tzmin = (min.z - ray.origin.z) / ray.direction.z;
  float tzmax = (max.z - ray.origin.z) / ray.direction.z;
  if (tzmin > tzmax) std::swap(tzmin, tzmax);
  if ((tmin > tzmax) || (tzmin > tmax)) return rec;
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  if ((double)tmin > kEps) {
    rec.t = tmin;
    rec.isHit = true;
    const Vector hp = ray.origin + ray.direction * tmin;
    Vector n(0.f, 0.f, 0.f);
    if (std::fabs(hp.x - min.x) < kEps) n = Vector(-1.f, 0.f, 0.f);
    else if (std::fabs(hp.x - max.x) < kEps) n = Vector(1.f, 0.f, 0.f);
    else if (std::fabs(hp.y - min.y) < kEps) n = Vector(0.f, -1.f, 0.f);
    else if (std::fabs(hp.y - max.y) < kEps) n = Vector(0.f, 1.f, 0.f);
    else if (std::fabs(hp.z - min.z) < kEps) n = Vector(0.f, 0.f, -1.f);
    else if (std::fabs(hp.z - max.z) < kEps) n = Vector(0.f, 0.f, 1.f);
    rec.normal = n;
  }
  return rec;
}

// ---------------------------------------------------------------- camera (camera.h:74-101)
Ray Camera::PrimaryRay(const Vector& ps) const {
  const float a = (float)((double)(ps.x / res_x) - 0.5);  // the 0.5 is a double upstream
  const float b = (float)((double)(ps.y / res_y) - 0.5);
  Vector dir = ((u * w) * a + (v * h) * b) - n * plane_dist;
  return Ray(eye, dir.normalize());
}

Ray Camera::PrimaryRay(const Vector& lens, const Vector& ps) const {
  const Vector eo = (eye + u * lens.x) + v * lens.y;
  const float px = ((ps.x / res_x) - 0.5f) * w * focal_ratio;
  const float py = ((ps.y / res_y) - 0.5f) * h * focal_ratio;
  const float f = plane_dist * focal_ratio;
  Vector dir = (u * (px - lens.x) + v * (py - lens.y)) - n * f;
  return Ray(eo, dir.normalize());
}

// ---------------------------------------------------------------- skybox (scene.cpp:329-458)
Color Scene::GetSkyboxColor(const Ray& r) const {  // scene.cpp:380-458
  const Vector& cc = r.direction;
  float ma;
  int side;
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
  const double invMa = 1 / ma;  // int / float: a float division, widened
  const float s = (float)((sc * invMa + 1) / 2);
  const float t = (float)((tc * invMa + 1) / 2);
  const SkyboxFace& f = skybox_img[side];
  if (f.img.empty()) return Color(0.f, 0.f, 0.f);
  // the reference's clamps of xp / yp are no-ops (scene.cpp:448-451)
  const unsigned xp = (unsigned)(int)((float)(f.resX - 1) * s);
  const unsigned yp = (unsigned)(int)((float)(f.resY - 1) * t);
  const size_t base = ((size_t)yp * (unsigned)f.resX + xp) * (unsigned)f.BPP;
  auto u8f = [](uint8_t x) { return (float)(x / 255.99f); };  // maths.h:133
  return Color(u8f(f.img[base]), u8f(f.img[base + 1]), u8f(f.img[base + 2]));
}

namespace {

std::mutex g_decoder_mu;
drt_image_decoder g_decoder = nullptr;
void* g_decoder_user = nullptr;

// Binary PPM (P6, maxval <= 255), rows top-down as in the file.
bool read_ppm(const std::string& path, int& w, int& h, std::vector<uint8_t>& px) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::string magic;
  f >> magic;
  if (magic != "P6") return false;
  auto next_int = [&](int& v) {
    while (true) {
      f >> std::ws;
      if (f.peek() == '#') { std::string line; std::getline(f, line); continue; }
      return bool(f >> v);
    }
  };
  int maxval = 0;
  if (!next_int(w) || !next_int(h) || !next_int(maxval) || w <= 0 || h <= 0 || maxval <= 0 || maxval > 255) return false;
  f.get();  // the single whitespace byte before the raster
  px.resize((size_t)w * h * 3);
  f.read((char*)px.data(), (std::streamsize)px.size());
  return (size_t)f.gcount() == px.size();
}

// One face, rows returned bottom-up (DevIL with IL_ORIGIN_LOWER_LEFT, scene.cpp:344-346).
bool load_face(const std::string& dir, const char* name, SkyboxFace& out) {
  int w = 0, h = 0, bpp = 3;
  std::vector<uint8_t> top_down;
  bool ok = false;
  {
    std::lock_guard<std::mutex> lk(g_decoder_mu);
    if (g_decoder) {
      uint8_t* px = nullptr;
      const std::string jpg = dir + "/" + name + ".jpg";
      if (g_decoder(jpg.c_str(), &w, &h, &bpp, &px, g_decoder_user) == 0 && px && w > 0 && h > 0 &&
          (bpp == 3 || bpp == 4)) {
        top_down.assign(px, px + (size_t)w * h * bpp);
        ok = true;
      }
      free(px);
    }
  }
  if (!ok) {
    bpp = 3;
    ok = read_ppm(dir + "/" + name + ".ppm", w, h, top_down);
  }
  if (!ok) return false;
  out.resX = w; out.resY = h; out.BPP = bpp;
  out.img.resize(top_down.size());
  const size_t row = (size_t)w * bpp;
  for (int y = 0; y < h; y++) memcpy(&out.img[(size_t)y * row], &top_down[(size_t)(h - 1 - y) * row], row);
  return true;
}

}  // namespace

bool Scene::LoadSkybox(const char* sky_dir) {  // scene.cpp:329-378
  static const char* kFaces[6] = {"right", "left", "top", "bottom", "front", "back"};
  if (!sky_dir) return false;
  SkyboxFace faces[6];
  for (int i = 0; i < 6; i++)
    if (!load_face(sky_dir, kFaces[i], faces[i])) return false;
  for (int i = 0; i < 6; i++) skybox_img[i] = std::move(faces[i]);
  return true;
}

// ---------------------------------------------------------------- BVH::Traverse (bvh.cpp:231-391)
namespace {
struct StackItem {
  uint32_t node;
  float t;
};
}  // namespace

bool BVH::Traverse(Ray& ray, Object** hit_obj, HitRecord& hitRec) const {  // bvh.cpp:231-314
  hitRec = HitRecord();
  if (nodes.empty()) return false;
  float tmp;
  if (!nodes[0].bbox.hit(ray, tmp)) return false;
  std::vector<StackItem> stack;
  bool hit = false;
  uint32_t cur = 0;
  while (true) {
    const Node& cn = nodes[cur];
    if (!cn.leaf) {
      const uint32_t li = cn.index;
      const Node& L = nodes[li];
      const Node& R = nodes[li + 1];
      float tL, tR;
      const bool hL = L.bbox.hit(ray, tL);
      const bool hR = R.bbox.hit(ray, tR);
      if (L.bbox.isInside(ray.origin)) tL = 0;
      if (R.bbox.isInside(ray.origin)) tR = 0;
      if (hL && hR) {  // nearer child first, ties to the right; the other one waits with its t
        if (tL < tR) { cur = li; stack.push_back({li + 1, tR}); }
        else { cur = li + 1; stack.push_back({li, tL}); }
        continue;
      }
      if (hL) { cur = li; continue; }
      if (hR) { cur = li + 1; continue; }
    } else {
      for (uint32_t i = 0; i < cn.n_objs; i++) {
        Object* o = objects[cn.index + i];
        const HitRecord rec = o->hit(ray);
        if (rec.isHit && rec.t < hitRec.t) {
          hitRec = rec;
          if (hit_obj) *hit_obj = o;
          hit = true;
        }
      }
    }
    bool next = false;  // pop until an entry could still hold a nearer hit (bvh.cpp:299-308)
    while (!stack.empty()) {
      const StackItem it = stack.back();
      stack.pop_back();
      if (it.t < hitRec.t) { cur = it.node; next = true; break; }
    }
    if (!next) return hit;
  }
}

bool BVH::Traverse(Ray& ray) const {  // bvh.cpp:316-391
  const double len = ray.direction.length();
  ray.direction.normalize();  // the caller's ray is normalised (bvh.cpp:321-322)
  if (nodes.empty()) return false;
  float tmp;
  if (!nodes[0].bbox.hit(ray, tmp)) return false;
  std::vector<StackItem> stack;
  uint32_t cur = 0;
  while (true) {
    const Node& cn = nodes[cur];
    if (!cn.leaf) {
      const uint32_t li = cn.index;
      const Node& L = nodes[li];
      const Node& R = nodes[li + 1];
      float tL, tR;
      const bool hL = L.bbox.hit(ray, tL);
      const bool hR = R.bbox.hit(ray, tR);
      if (L.bbox.isInside(ray.origin)) tL = 0;
      if (R.bbox.isInside(ray.origin)) tR = 0;
      if (hL && hR) {  // ties to the left here
        if (tL <= tR) { cur = li; stack.push_back({li + 1, tR}); }
        else { cur = li + 1; stack.push_back({li, tL}); }
        continue;
      }
      if (hL) { cur = li; continue; }
      if (hR) { cur = li + 1; continue; }
    } else {
      for (uint32_t i = 0; i < cn.n_objs; i++) {
        const HitRecord rec = objects[cn.index + i]->hit(ray);
        if (rec.isHit && (double)rec.t <= len + kEps) return true;
      }
    }
    if (stack.empty()) return false;  // popped without t-pruning (bvh.cpp:381-387)
    cur = stack.back().node;
    stack.pop_back();
  }
}

// ---------------------------------------------------------------- Grid::Traverse (grid.cpp:100-358)
bool Grid::Init_Traverse(const Ray& ray, int& ix, int& iy, int& iz, double& dtx, double& dty, double& dtz,
                         double& txn, double& tyn, double& tzn, int& ixs, int& iys, int& izs, int& ixe, int& iye,
                         int& ize) const {  // grid.cpp:100-244
  const float ox = ray.origin.x, oy = ray.origin.y, oz = ray.origin.z;
  const float dx = ray.direction.x, dy = ray.direction.y, dz = ray.direction.z;
  const float x0 = bbox.min.x, y0 = bbox.min.y, z0 = bbox.min.z, x1 = bbox.max.x, y1 = bbox.max.y, z1 = bbox.max.z;
  float txmin, tymin, tzmin, txmax, tymax, tzmax;
  const float a = (float)(1.0 / dx);
  if (a >= 0) { txmin = (x0 - ox) * a; txmax = (x1 - ox) * a; } else { txmin = (x1 - ox) * a; txmax = (x0 - ox) * a; }
  const float b = (float)(1.0 / dy);
  if (b >= 0) { tymin = (y0 - oy) * b; tymax = (y1 - oy) * b; } else { tymin = (y1 - oy) * b; tymax = (y0 - oy) * b; }
  const float c = (float)(1.0 / dz);
  if (c >= 0) { tzmin = (z0 - oz) * c; tzmax = (z1 - oz) * c; } else { tzmin = (z1 - oz) * c; tzmax = (z0 - oz) * c; }
  float t0, t1;
  if (txmin > tymin) t0 = txmin; else t0 = tymin;
  if (tzmin > t0) t0 = tzmin;
  if (txmax < tymax) t1 = txmax; else t1 = tymax;
  if (tzmax < t1) t1 = tzmax;
  if (t0 > t1 || t1 < 0) return false;
  if (bbox.isInside(ray.origin)) {
    ix = (int)dclamp((ox - x0) * nx / (x1 - x0), 0, nx - 1);
    iy = (int)dclamp((oy - y0) * ny / (y1 - y0), 0, ny - 1);
    iz = (int)dclamp((oz - z0) * nz / (z1 - z0), 0, nz - 1);
  } else {
    const Vector p = ray.origin + ray.direction * t0;
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

bool Grid::Traverse(Ray& ray, Object** hitobject, HitRecord& hitRec) const {  // grid.cpp:247-306
  hitRec = HitRecord();
  if (cell_start.empty()) return false;
  int ix, iy, iz, ixs, iys, izs, ixe, iye, ize;
  double txn, tyn, tzn, dtx, dty, dtz;
  if (!Init_Traverse(ray, ix, iy, iz, dtx, dty, dtz, txn, tyn, tzn, ixs, iys, izs, ixe, iye, ize)) return false;
  Object* closest = nullptr;
  while (true) {
    const int64_t cidx = (int64_t)ix + (int64_t)nx * iy + (int64_t)nx * ny * iz;
    for (int64_t q = cell_start[(size_t)cidx]; q < cell_start[(size_t)cidx + 1]; q++) {
      Object* o = objects[(size_t)cell_objs[(size_t)q]];
      const HitRecord rec = o->hit(ray);
      if (rec.isHit && rec.t < hitRec.t) { hitRec = rec; closest = o; }
    }
    // a hit nearer than the next cell boundary ends the walk; leaving the grid is a miss
    if (txn < tyn && txn < tzn) {
      if (hitRec.t < txn) { if (hitobject) *hitobject = closest; return true; }
      txn += dtx; ix += ixs;
      if (ix == ixe) return false;
    } else if (tyn < tzn) {
      if (hitRec.t < tyn) { if (hitobject) *hitobject = closest; return true; }
      tyn += dty; iy += iys;
      if (iy == iye) return false;
    } else {
      if (hitRec.t < tzn) { if (hitobject) *hitobject = closest; return true; }
      tzn += dtz; iz += izs;
      if (iz == ize) return false;
    }
  }
}

bool Grid::Traverse(Ray& ray) const {  // grid.cpp:309-358
  const double len = ray.direction.length();
  ray.direction.normalize();
  if (cell_start.empty()) return true;
  int ix, iy, iz, ixs, iys, izs, ixe, iye, ize;
  double txn, tyn, tzn, dtx, dty, dtz;
  // a shadow ray that misses the grid box counts as shadowed (grid.cpp:323-324)
  if (!Init_Traverse(ray, ix, iy, iz, dtx, dty, dtz, txn, tyn, tzn, ixs, iys, izs, ixe, iye, ize)) return true;
  while (true) {
    const int64_t cidx = (int64_t)ix + (int64_t)nx * iy + (int64_t)nx * ny * iz;
    for (int64_t q = cell_start[(size_t)cidx]; q < cell_start[(size_t)cidx + 1]; q++) {
      const HitRecord rec = objects[(size_t)cell_objs[(size_t)q]]->hit(ray);
      if (rec.isHit && (double)rec.t < len) return true;
    }
    if (txn < tyn && txn < tzn) {
      txn += dtx; ix += ixs;
      if (ix == ixe) return false;
    } else if (tyn < tzn) {
      tyn += dty; iy += iys;
      if (iy == iye) return false;
    } else {
      tzn += dtz; iz += izs;
      if (iz == ize) return false;
    }
  }
}

}  // namespace drt

extern "C" int drt_set_image_decoder(drt_image_decoder fn, void* user) {
  std::lock_guard<std::mutex> lk(drt::g_decoder_mu);
  drt::g_decoder = fn;
  drt::g_decoder_user = user;
  return DRT_OK;
}
