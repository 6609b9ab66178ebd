// drt_scene.cpp — host scene model: objects, camera frame, P3F loader, GPU packing.
#include "../../../include/drt_scene.hpp"

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>

namespace drt {

static constexpr double kEps = 0.001;                       // macros.h:1
static constexpr float kPI = 3.141592653589793238462f;       // maths.h:8

// ---------------------------------------------------------------- objects
Triangle::Triangle(const Vector& P0, const Vector& P1, const Vector& P2) {  // scene.cpp:10-35
  points[0] = P0; points[1] = P1; points[2] = P2;
  Min = Vector(+FLT_MAX, +FLT_MAX, +FLT_MAX);
  Max = Vector(-FLT_MAX, -FLT_MAX, -FLT_MAX);
  for (const Vector& p : points) {
    if (p.x < Min.x) Min.x = p.x;
    if (p.x > Max.x) Max.x = p.x;
    if (p.y < Min.y) Min.y = p.y;
    if (p.y > Max.y) Max.y = p.y;
    if (p.z < Min.z) Min.z = p.z;
    if (p.z > Max.z) Max.z = p.z;
  }
  const float e = (float)kEps;  // Vector::operator-=(const float), vector.cpp:78-82
  Min.x -= e; Min.y -= e; Min.z -= e;
  Max.x += e; Max.y += e; Max.z += e;
}

static int mat_index(const Material* m) { return m ? m->index : -1; }

drt_prim Triangle::pack() const {
  drt_prim p{};
  p.type = DRT_PRIM_TRIANGLE;
  p.material = mat_index(m_Material);
  const Vector* v[3] = {&points[0], &points[1], &points[2]};
  float* dst[3] = {p.a, p.b, p.c};
  for (int i = 0; i < 3; i++) { dst[i][0] = v[i]->x; dst[i][1] = v[i]->y; dst[i][2] = v[i]->z; }
  return p;
}

drt_prim Sphere::pack() const {
  drt_prim p{};
  p.type = DRT_PRIM_SPHERE;
  p.material = mat_index(m_Material);
  p.a[0] = center.x; p.a[1] = center.y; p.a[2] = center.z;
  p.r = radius;
  return p;
}

Plane::Plane(const Vector& P0, const Vector& P1, const Vector& P2) {  // scene.cpp:100-114
  PN = (P1 - P0) % (P2 - P0);
  if (PN.length() == 0.0) {
    std::cerr << "DEGENERATED PLANE!\n";
    D = 0.0f;  // left uninitialised upstream
  } else {
    PN.normalize();
    D = -(PN * P0);
  }
}

drt_prim Plane::pack() const {
  drt_prim p{};
  p.type = DRT_PRIM_PLANE;
  p.material = mat_index(m_Material);
  p.a[0] = PN.x; p.a[1] = PN.y; p.a[2] = PN.z;
  p.r = D;
  return p;
}

drt_prim aaBox::pack() const {
  drt_prim p{};
  p.type = DRT_PRIM_BOX;
  p.material = mat_index(m_Material);
  p.a[0] = min.x; p.a[1] = min.y; p.a[2] = min.z;
  p.b[0] = max.x; p.b[1] = max.y; p.b[2] = max.z;
  return p;
}

// ---------------------------------------------------------------- camera (camera.h:32-72)
Camera::Camera(Vector from, Vector At, Vector Up, float angle, float hither, float yon, int ResX, int ResY,
               float Aperture_ratio, float Focal_ratio)
    : eye(from), at(At), up(Up), fovy(angle), vnear(hither), vfar(yon), focal_ratio(Focal_ratio), res_x(ResX),
      res_y(ResY) {
  n = eye - at;
  plane_dist = n.length();
  n = n / plane_dist;
  u = up % n;
  u = u / u.length();
  v = n % u;
  h = 2 * plane_dist * std::tan((kPI * angle / 180) / 2.0f);
  w = ((float)res_x / res_y) * h;
  aperture = Aperture_ratio * (w / res_x);
}

void Camera::SetEye(Vector from) {
  eye = from;
  n = eye - at;
  plane_dist = n.length();
  n = n / plane_dist;
  u = up % n;
  u = u / u.length();
  v = n % u;
}

drt_camera Camera::frame() const {
  drt_camera c{};
  const Vector* src[4] = {&eye, &u, &v, &n};
  float* dst[4] = {c.eye, c.u, c.v, c.n};
  for (int i = 0; i < 4; i++) { dst[i][0] = src[i]->x; dst[i][1] = src[i]->y; dst[i][2] = src[i]->z; }
  c.w = w; c.h = h; c.plane_dist = plane_dist; c.focal_ratio = focal_ratio; c.aperture = aperture;
  c.res_x = res_x; c.res_y = res_y;
  return c;
}

// ---------------------------------------------------------------- scene
Scene::Scene() = default;
Scene::~Scene() {
  for (Object* o : owned) delete o;
  for (Light* l : lights) delete l;
}

void Scene::addObject(Object* o) {
  o->scene_index = (int32_t)objects.size();
  objects.push_back(o);
  owned.push_back(o);
}

Material* Scene::addMaterial(const Material& m) {
  materials.push_back(std::make_unique<Material>(m));
  materials.back()->index = (int)materials.size() - 1;
  return materials.back().get();
}

void Scene::addTriangles(const float* v, size_t n, Material* m) {
  if (!n) return;
  auto pool = std::make_unique<std::vector<Triangle>>();
  pool->reserve(n);  // no reallocation afterwards: object pointers stay valid
  for (size_t i = 0; i < n; i++) {
    const float* q = v + 9 * i;
    pool->emplace_back(Vector(q[0], q[1], q[2]), Vector(q[3], q[4], q[5]), Vector(q[6], q[7], q[8]));
    Triangle& t = pool->back();
    t.SetMaterial(m);
    t.scene_index = (int32_t)objects.size();
    objects.push_back(&t);
  }
  tri_pools.push_back(std::move(pool));
}

void Scene::SetSkyboxFace(int face, int w, int h, int bpp, const uint8_t* px) {
  if (face < 0 || face > 5) return;
  SkyboxFace& f = skybox_img[face];
  f.resX = w; f.resY = h; f.BPP = bpp;
  f.img.assign(px, px + (size_t)w * h * bpp);
}

bool Scene::SkyboxComplete() const {
  for (const auto& f : skybox_img)
    if (f.img.empty()) return false;
  return true;
}

void Scene::describe(drt_scene_desc& d, std::vector<drt_prim>& prims, std::vector<drt_light>& ls,
                     std::vector<drt_material>& ms) const {
  memset(&d, 0, sizeof(d));
  if (camera) d.camera = camera->frame();
  prims.resize(objects.size());
  for (size_t i = 0; i < objects.size(); i++) prims[i] = objects[i]->pack();
  ls.clear();
  for (const Light* l : lights) {
    drt_light q{};
    q.type = l->type == QUAD ? DRT_LIGHT_QUAD : DRT_LIGHT_POINT;
    q.pos[0] = l->position.x; q.pos[1] = l->position.y; q.pos[2] = l->position.z;
    q.e1[0] = l->e1.x; q.e1[1] = l->e1.y; q.e1[2] = l->e1.z;
    q.e2[0] = l->e2.x; q.e2[1] = l->e2.y; q.e2[2] = l->e2.z;
    q.grid_res = l->gridRes;
    ls.push_back(q);
  }
  ms.clear();
  for (const auto& m : materials) {
    drt_material q{};
    Color c = m->GetDiffColor(), s = m->GetSpecColor();
    q.diff[0] = c.r(); q.diff[1] = c.g(); q.diff[2] = c.b();
    q.spec[0] = s.r(); q.spec[1] = s.g(); q.spec[2] = s.b();
    q.kd = m->GetDiffuse(); q.ks = m->GetSpecular(); q.shine = m->GetShine(); q.refl = m->GetReflection();
    q.trans = m->GetTransmittance(); q.ior = m->GetRefrIndex();
    ms.push_back(q);
  }
  d.materials = ms.data();
  d.n_materials = (int32_t)ms.size();
  d.prims = prims.data();
  d.n_prims = (int32_t)prims.size();
  d.lights = ls.data();
  d.n_lights = (int32_t)ls.size();
  d.background[0] = bgColor.r(); d.background[1] = bgColor.g(); d.background[2] = bgColor.b();
  d.accel = accel_struc_type == BVH_ACC ? DRT_ACCEL_BVH : (accel_struc_type == GRID_ACC ? DRT_ACCEL_GRID : DRT_ACCEL_NONE);
  d.spp = samples_per_pixel;
  d.has_skybox = SkyBoxFlg ? 1 : 0;
  for (int f = 0; f < 6; f++) {
    d.skybox[f] = skybox_img[f].img.empty() ? nullptr : skybox_img[f].img.data();
    d.sky_w[f] = skybox_img[f].resX; d.sky_h[f] = skybox_img[f].resY; d.sky_bpp[f] = skybox_img[f].BPP;
  }
}

// ---------------------------------------------------------------- P3F loader (scene.cpp:466-740)
namespace {

// Whitespace tokenizer with the conversions libstdc++'s istream uses (strtof for float,
// strtod for double, strtoul for unsigned), so every number is bit-identical to `file >> x`.
class Tokens {
 public:
  explicit Tokens(std::string s) : buf(std::move(s)) {}
  bool next(std::string& tok) {
    if (failed) return false;
    skip_ws();
    if (pos >= buf.size()) { failed = true; return false; }
    size_t b = pos;
    while (pos < buf.size() && !isspace((unsigned char)buf[pos])) pos++;
    tok.assign(buf, b, pos - b);
    return true;
  }
  float f() { return num<float>([](const char* s, char** e) { return strtof(s, e); }); }
  double d() { return num<double>([](const char* s, char** e) { return strtod(s, e); }); }
  unsigned u() { return num<unsigned>([](const char* s, char** e) { return (unsigned)strtoul(s, e, 10); }); }
  int i() { return num<int>([](const char* s, char** e) { return (int)strtol(s, e, 10); }); }
  Vector vec() { float a = f(), b = f(), c = f(); return Vector(a, b, c); }
  Color col() { float a = f(), b = f(), c = f(); return Color(a, b, c); }
  void ignore_line() {  // file.ignore(1024, '\n')
    size_t n = 0;
    while (pos < buf.size() && n < 1024) {
      char c = buf[pos++];
      n++;
      if (c == '\n') break;
    }
  }
  bool failed = false;

 private:
  void skip_ws() { while (pos < buf.size() && isspace((unsigned char)buf[pos])) pos++; }
  template <class T, class F>
  T num(F conv) {
    if (failed) return T(0);
    skip_ws();
    if (pos >= buf.size()) { failed = true; return T(0); }
    const char* s = buf.c_str() + pos;
    char* e = nullptr;
    errno = 0;
    T v = conv(s, &e);
    if (e == s) { failed = true; return T(0); }
    pos += (size_t)(e - s);
    return v;
  }
  std::string buf;
  size_t pos = 0;
};

}  // namespace

bool Scene::load_p3f(const char* name) {
  std::ifstream file(name, std::ios::in | std::ios::binary);
  if (!file) return false;
  std::stringstream ss;
  ss << file.rdbuf();
  Tokens tk(ss.str());
  Material* material = nullptr;
  SkyBoxFlg = false;
  std::string cmd, tok;
  auto expect = [&](const char* nm) {
    tk.next(tok);
    if (tok != nm) std::cerr << "'" << nm << "' expected.\n";
  };
  if (!tk.next(cmd)) return true;
  while (true) {
    if (cmd == "accel") {
      tk.next(tok);
      if (tok == "none") accel_struc_type = NONE;
      else if (tok == "grid") accel_struc_type = GRID_ACC;
      else if (tok == "bvh") accel_struc_type = BVH_ACC;
      else { printf("Unsupported acceleration type\n"); break; }
    } else if (cmd == "spp") {
      samples_per_pixel = tk.u();
    } else if (cmd == "mat") {
      Color cd = tk.col();
      double Kd = tk.d();
      Color cs = tk.col();
      double Ks = tk.d(), Shine = tk.d(), T = tk.d(), ior = tk.d();
      material = addMaterial(Material(cd, (float)Kd, cs, (float)Ks, (float)Shine, (float)T, (float)ior));
    } else if (cmd == "s") {
      Vector c = tk.vec();
      float r = tk.f();
      Sphere* s = new Sphere(c, r);
      if (material) s->SetMaterial(material);
      addObject(s);
    } else if (cmd == "box") {
      Vector a = tk.vec(), b = tk.vec();
      aaBox* bx = new aaBox(a, b);
      if (material) bx->SetMaterial(material);
      addObject(bx);
    } else if (cmd == "p") {
      unsigned tv = tk.u();
      if (tv == 3) {
        Vector a = tk.vec(), b = tk.vec(), c = tk.vec();
        Triangle* t = new Triangle(a, b, c);
        if (material) t->SetMaterial(material);
        addObject(t);
      } else {
        std::cerr << "Unsupported number of vertices.\n";
        break;
      }
    } else if (cmd == "mesh") {
      unsigned tv = tk.u(), tf = tk.u();
      std::vector<float> verts((size_t)tv * 3);
      for (unsigned i = 0; i < tv; i++) { verts[3 * i] = tk.f(); verts[3 * i + 1] = tk.f(); verts[3 * i + 2] = tk.f(); }
      std::vector<float> tris;
      tris.reserve((size_t)tf * 9);
      bool bad = false;
      for (unsigned i = 0; i < tf; i++) {
        unsigned P0 = tk.u(), P1 = tk.u(), P2 = tk.u();
        if (P0 > 0) { P0 -= 1; P1 -= 1; P2 -= 1; }
        else { P0 += tv; P1 += tv; P2 += tv; }
        if (P0 >= tv || P1 >= tv || P2 >= tv) { std::cerr << "mesh index out of range\n"; bad = true; break; }
        for (unsigned q : {P0, P1, P2}) tris.insert(tris.end(), &verts[3 * (size_t)q], &verts[3 * (size_t)q] + 3);
      }
      addTriangles(tris.data(), tris.size() / 9, material);
      if (bad) break;
    } else if (cmd == "npl") {
      Vector nn = tk.vec();
      float dd = tk.f();
      Plane* p = new Plane(nn, dd);
      if (material) p->SetMaterial(material);
      addObject(p);
    } else if (cmd == "pl") {
      Vector a = tk.vec(), b = tk.vec(), c = tk.vec();
      Plane* p = new Plane(a, b, c);
      if (material) p->SetMaterial(material);
      addObject(p);
    } else if (cmd == "light") {
      tk.next(tok);
      if (tok == "punctual") {
        Vector pos = tk.vec();
        Color col = tk.col();
        addLight(new Light(pos, col));
      } else if (tok == "quad") {
        Vector pos = tk.vec();
        Color col = tk.col();
        Vector v1 = tk.vec(), v2 = tk.vec();
        unsigned g = tk.u();
        addLight(new Light(pos, col, v1, v2, g));
      } else {
        std::cerr << "Unsupported light type.\n";
        break;
      }
    } else if (cmd == "camera") {
      expect("eye"); Vector from = tk.vec();
      expect("at"); Vector at = tk.vec();
      expect("up"); Vector up = tk.vec();
      expect("angle"); float fov = tk.f();
      expect("hither"); float hither = tk.f();
      expect("resolution"); int xres = tk.i(); int yres = tk.i();
      expect("aperture"); float ar = tk.f();
      expect("focal"); float fr = tk.f();
      SetCamera(new Camera(from, at, up, fov, hither, (float)(1000.0 * hither), xres, yres, ar, fr));
    } else if (cmd == "bclr") {
      bgColor = tk.col();
    } else if (cmd == "env") {  // scene.cpp:687-692: LoadSkybox(token) + SetSkyBoxFlg(true)
      tk.next(tok);
      env_dir = tok;
      SkyBoxFlg = true;
      if (!LoadSkybox(tok.c_str())) {  // the reference resolves <dir> from the working directory
        std::string p(name);
        const size_t cut = p.find_last_of('/');
        const std::string dir = cut == std::string::npos ? std::string(".") : p.substr(0, cut);
        LoadSkybox((dir + "/../" + tok).c_str());  // else next to P3D_Scenes/
      }
    } else if (!cmd.empty() && cmd[0] == '#') {
      tk.ignore_line();
    } else {
      std::cerr << "unknown command '" << cmd << "'.\n";
      break;
    }
    if (!tk.next(cmd)) break;
  }
  return true;
}

}  // namespace drt
