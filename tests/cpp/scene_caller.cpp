// scene_caller.cpp — a reference-style C++ caller of include/drt_scene.hpp (test program).
//
// It is written the way the reference's main.cpp drives its scene: Scene::
// load_p3f, Scene::GetCamera / getObject / GetSkyboxColor, Camera::PrimaryRay, Light::
// getAreaLightPoint, Object::hit, AABB::hit / isInside, Vector / Color arithmetic, BVH / Grid
// Build + Traverse with Object** / HitRecord — and for frames drt::upload_scene +
// drt::render_scene on a drt_ctx.  tests/test_cpp_api.py compiles it against include/ and
// libdrt.so and checks its outputs against the reference-produced goldens (tests/golden/), the
// oracle and the Python binding.
//
// I/O is raw little-endian arrays (numpy .tofile / fromfile).  Modes:
//   aabb   BOXES_RAYS.f32 OUT        n x {box min xyz, max xyz, ray o xyz, d xyz} -> per ray
//                                    {hit, inside} u8 pairs then t f32
//   vec    AB.f32 OUT                n x {a xyz, b xyz} -> normalize xyz, length, cross xyz, dot
//   color  C.f32 OUT                 n x rgb -> clamp rgb, exp_ rgb, and (c*2 + c) * c - c
//   light  Q.f32 S.f32 OUT           quad {pos, v1, v2}, n x xyz samples -> getAreaLightPoint
//   camera P.f64 S.f32 OUT           {eye, at, up, fov, hither, resx, resy, aperture, focal},
//                                    n x {px, py, lx, ly} -> pinhole rays then thin-lens rays
//   trace  SCENE.p3f RAYS.f32 OUT    BVH / Grid / NONE from the scene's accel: closest {t, n xyz,
//                                    object} f32 x 4 + i32 per ray, then shadow occluded u8
//   build  SCENE.p3f ACCEL OUT       bvh: n_nodes i32, nodes {box 6 f32, leaf, index, nobjs u32},
//                                    order i32; grid: dims 3 i32, box 6 f32, n_refs i64,
//                                    cell_start i64, cell_objs i32
//   sky    SCENE.p3f DIRS.f32 OUT    GetSkyboxColor (skybox from the scene's `env`, LoadSkybox)
//   hit    SCENE.p3f RAYS.f32 OUT    Object::hit of every object for every ray: {isHit, t, n xyz}
//   render SCENE.p3f SEED OUT        GPU frame through drt::upload_scene / drt::render_scene
//   group  SCENE.p3f SEED NDEV OUT   the same frame tile-sharded over NDEV GPUs (drt_group_*:
//                                    RCCL all-gather, reassembly on device 0), no Python
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "drt_scene.hpp"

using namespace drt;

template <class T>
static std::vector<T> read_all(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::vector<T> v(b.size() / sizeof(T));
  memcpy(v.data(), b.data(), v.size() * sizeof(T));
  return v;
}

struct Out {
  FILE* f;
  explicit Out(const char* p) : f(fopen(p, "wb")) {
    if (!f) { perror(p); exit(2); }
  }
  ~Out() { fclose(f); }
  template <class T>
  void put(const T& v) { fwrite(&v, sizeof(T), 1, f); }
  void vec(const Vector& v) { put(v.x); put(v.y); put(v.z); }
  void col(const Color& c) { put(c.r()); put(c.g()); put(c.b()); }
};

static int load(Scene& s, const char* p3f) {
  if (!s.load_p3f(p3f)) { fprintf(stderr, "cannot load %s\n", p3f); return 2; }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: scene_caller MODE ARGS... OUT\n"); return 2; }
  const std::string mode = argv[1];
  if (mode == "aabb") {
    auto in = read_all<float>(argv[2]);
    const size_t n = in.size() / 12;
    Out o(argv[3]);
    std::vector<float> ts(n);
    for (size_t i = 0; i < n; i++) {
      const float* q = &in[12 * i];
      AABB box(Vector(q[0], q[1], q[2]), Vector(q[3], q[4], q[5]));
      Ray r(Vector(q[6], q[7], q[8]), Vector(q[9], q[10], q[11]));
      float t = 0.f;
      const uint8_t h = box.hit(r, t) ? 1 : 0, ins = box.isInside(r.origin) ? 1 : 0;
      o.put(h); o.put(ins);
      ts[i] = t;
    }
    for (float t : ts) o.put(t);
  } else if (mode == "vec") {
    auto in = read_all<float>(argv[2]);
    Out o(argv[3]);
    for (size_t i = 0; i + 6 <= in.size(); i += 6) {
      Vector a(in[i], in[i + 1], in[i + 2]), b(in[i + 3], in[i + 4], in[i + 5]);
      Vector nrm = a;
      nrm.normalize();
      o.vec(nrm); o.put(a.length()); o.vec(a % b); o.put(a * b);
    }
  } else if (mode == "color") {
    auto in = read_all<float>(argv[2]);
    Out o(argv[3]);
    for (size_t i = 0; i + 3 <= in.size(); i += 3) {
      Color c(in[i], in[i + 1], in[i + 2]);
      o.col(c.clamp()); o.col(c.exp_());
      Color d = c * 2.0f;
      d += c;
      d *= c;
      o.col(d - c);
    }
  } else if (mode == "light") {
    auto q = read_all<float>(argv[2]);
    auto s = read_all<float>(argv[3]);
    Light L(Vector(q[0], q[1], q[2]), Color(1, 1, 1), Vector(q[3], q[4], q[5]), Vector(q[6], q[7], q[8]), 16);
    Out o(argv[4]);
    for (size_t i = 0; i + 3 <= s.size(); i += 3) o.vec(L.getAreaLightPoint(Vector(s[i], s[i + 1], s[i + 2])));
  } else if (mode == "camera") {
    auto p = read_all<double>(argv[2]);
    auto s = read_all<float>(argv[3]);
    Camera cam(Vector((float)p[0], (float)p[1], (float)p[2]), Vector((float)p[3], (float)p[4], (float)p[5]),
               Vector((float)p[6], (float)p[7], (float)p[8]), (float)p[9], (float)p[10], (float)(1000.0 * (float)p[10]),
               (int)p[11], (int)p[12], (float)p[13], (float)p[14]);
    Out o(argv[4]);
    for (int dof = 0; dof < 2; dof++)
      for (size_t i = 0; i + 4 <= s.size(); i += 4) {
        const Vector ps(s[i], s[i + 1], 0.f), lens(s[i + 2], s[i + 3], 0.f);
        const Ray r = dof ? cam.PrimaryRay(lens, ps) : cam.PrimaryRay(ps);
        o.vec(r.origin); o.vec(r.direction);
      }
  } else if (mode == "trace") {
    Scene scene;
    if (int rc = load(scene, argv[2])) return rc;
    auto rays = read_all<float>(argv[3]);
    const size_t n = rays.size() / 6;
    BVH bvh;
    Grid grid;
    std::vector<Object*> objs = scene.objectList();
    if (scene.GetAccelStruct() == BVH_ACC) bvh.Build(objs);
    else if (scene.GetAccelStruct() == GRID_ACC) grid.Build(objs);
    Out o(argv[4]);
    std::vector<uint8_t> occ(n);
    for (size_t i = 0; i < n; i++) {
      const float* q = &rays[6 * i];
      Ray ray(Vector(q[0], q[1], q[2]), Vector(q[3], q[4], q[5]));
      Object* hitObj = nullptr;
      HitRecord rec;
      bool hit = false;
      if (scene.GetAccelStruct() == BVH_ACC) hit = bvh.Traverse(ray, &hitObj, rec);
      else if (scene.GetAccelStruct() == GRID_ACC) hit = grid.Traverse(ray, &hitObj, rec);
      else {  // main.cpp:315-326
        for (int k = 0; k < scene.getNumObjects(); k++) {
          HitRecord h = scene.getObject(k)->hit(ray);
          if (h.isHit && h.t < rec.t) { rec = h; hitObj = scene.getObject(k); hit = true; }
        }
      }
      o.put(hit ? rec.t : FLT_MAX);
      o.vec(hit ? rec.normal : Vector(0.f, 0.f, 0.f));
      o.put((int32_t)(hit && hitObj ? hitObj->scene_index : -1));
      Ray shadow(Vector(q[0], q[1], q[2]), Vector(q[3], q[4], q[5]));
      if (scene.GetAccelStruct() == BVH_ACC) occ[i] = bvh.Traverse(shadow);
      else if (scene.GetAccelStruct() == GRID_ACC) occ[i] = grid.Traverse(shadow);
    }
    for (uint8_t v : occ) o.put(v);
  } else if (mode == "build") {
    Scene scene;
    if (int rc = load(scene, argv[2])) return rc;
    std::vector<Object*> objs = scene.objectList();
    Out o(argv[4]);
    if (std::string(argv[3]) == "bvh") {
      BVH bvh;
      bvh.Build(objs);
      o.put((int32_t)bvh.nodeList().size());
      for (const auto& nd : bvh.nodeList()) {
        o.vec(nd.bbox.min); o.vec(nd.bbox.max);
        o.put((uint32_t)nd.leaf); o.put(nd.index); o.put(nd.leaf ? nd.n_objs : 0u);
      }
      for (Object* ob : bvh.objectOrder()) o.put((int32_t)ob->scene_index);
    } else {
      Grid grid;
      grid.Build(objs);
      o.put((int32_t)grid.nx); o.put((int32_t)grid.ny); o.put((int32_t)grid.nz);
      o.vec(grid.bbox.min); o.vec(grid.bbox.max);
      o.put((int64_t)grid.cell_objs.size());
      for (int64_t v : grid.cell_start) o.put(v);
      for (int32_t v : grid.cell_objs) o.put((int32_t)grid.getObject((unsigned)v)->scene_index);
    }
  } else if (mode == "sky") {
    Scene scene;
    if (int rc = load(scene, argv[2])) return rc;
    if (!scene.GetSkyBoxFlg() || !scene.SkyboxComplete()) { fprintf(stderr, "skybox not loaded\n"); return 3; }
    auto d = read_all<float>(argv[3]);
    Out o(argv[4]);
    for (size_t i = 0; i + 3 <= d.size(); i += 3)
      o.col(scene.GetSkyboxColor(Ray(Vector(0.f, 0.f, 0.f), Vector(d[i], d[i + 1], d[i + 2]))));
  } else if (mode == "hit") {
    Scene scene;
    if (int rc = load(scene, argv[2])) return rc;
    auto rays = read_all<float>(argv[3]);
    Out o(argv[4]);
    for (int k = 0; k < scene.getNumObjects(); k++)
      for (size_t i = 0; i + 6 <= rays.size(); i += 6) {
        Ray r(Vector(rays[i], rays[i + 1], rays[i + 2]), Vector(rays[i + 3], rays[i + 4], rays[i + 5]));
        HitRecord h = scene.getObject(k)->hit(r);
        o.put((float)h.isHit); o.put(h.t); o.vec(h.normal);
      }
  } else if (mode == "group") {
    Scene scene;
    if (int rc = load(scene, argv[2])) return rc;
    BVH bvh;
    Grid grid;
    std::vector<Object*> objs = scene.objectList();
    if (scene.GetAccelStruct() == BVH_ACC) bvh.Build(objs);
    else if (scene.GetAccelStruct() == GRID_ACC) grid.Build(objs);
    drt_group* group = nullptr;
    if (int rc = drt_group_create(&group, atoi(argv[4]), nullptr)) { fprintf(stderr, "drt_group_create: %d\n", rc); return 4; }
    if (int rc = upload_scene(group, scene, &bvh, &grid)) { fprintf(stderr, "upload_scene: %d\n", rc); return 4; }
    drt_frame_params p{};
    p.seed = (uint32_t)strtoul(argv[3], nullptr, 10);
    p.max_depth = 4;
    const Camera* cam = scene.GetCamera();
    std::vector<float> colors((size_t)cam->GetResX() * cam->GetResY() * 3);
    if (int rc = render_scene(group, p, colors.data())) {
      fprintf(stderr, "render_scene: %d %s\n", rc, drt_group_last_error(group));
      return 4;
    }
    drt_group_destroy(group);
    Out o(argv[5]);
    fwrite(colors.data(), sizeof(float), colors.size(), o.f);
  } else if (mode == "render") {
    Scene scene;
    if (int rc = load(scene, argv[2])) return rc;
    BVH bvh;
    Grid grid;
    std::vector<Object*> objs = scene.objectList();
    if (scene.GetAccelStruct() == BVH_ACC) bvh.Build(objs);
    else if (scene.GetAccelStruct() == GRID_ACC) grid.Build(objs);
    drt_ctx* ctx = nullptr;
    drt_options opt{};
    if (int rc = drt_create(&ctx, &opt)) { fprintf(stderr, "drt_create: %d\n", rc); return 4; }
    if (int rc = upload_scene(ctx, scene, &bvh, &grid)) {
      fprintf(stderr, "upload_scene: %d %s\n", rc, drt_last_error(ctx));
      return 4;
    }
    drt_frame_params p{};
    p.seed = (uint32_t)strtoul(argv[3], nullptr, 10);
    p.max_depth = 4;  // MAX_DEPTH (main.cpp:34)
    p.n_shards = 1;
    const Camera* cam = scene.GetCamera();
    std::vector<float> colors((size_t)cam->GetResX() * cam->GetResY() * 3);
    if (int rc = render_scene(ctx, p, colors.data())) {
      fprintf(stderr, "render_scene: %d %s\n", rc, drt_last_error(ctx));
      return 4;
    }
    drt_destroy(ctx);
    Out o(argv[4]);
    fwrite(colors.data(), sizeof(float), colors.size(), o.f);
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  return 0;
}
