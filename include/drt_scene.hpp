// drt_scene.hpp — the reference's C++ scene API on top of libdrt.so (C++17, host side).
//
// rita-mota/DistributionRayTracer's hot path is driven through the class API of
// DistributionRayTracer/scene.h, camera.h, rayAccelerator.h, vector.h, color.h, ray.h and
// boundingBox.h.  This header keeps those classes, their method names and their
// meaning, so a main.cpp written against the reference keeps compiling against it:
//
//   Vector, Color, Ray, AABB, HitRecord     vector.h, color.h:11-75, ray.h, boundingBox.h:5-20,
//                                           scene.h:24-31
//   Material, Light, Object + Triangle /    scene.h:34-180 (Object::hit is the CPU intersection,
//   Sphere / Plane / aaBox                  scene.cpp:44-278)
//   Camera                                  camera.h:12-101 (PrimaryRay pinhole / thin lens)
//   Scene                                   scene.h:183-231: load_p3f (scene.cpp:474-740),
//                                           LoadSkybox / GetSkyboxColor (scene.cpp:329-458)
//   BVH, Grid                               rayAccelerator.h:12-94: Build (tree-identical,
//                                           bvh.cpp:27-227, grid.cpp:30-97), scalar Traverse on
//                                           the CPU (bvh.cpp:231-391, grid.cpp:100-358), the
//                                           Grid object list (grid.cpp:7-27)
//   renderScene()                           drt::upload_scene + drt::render_scene over a drt_ctx
//                                           (include/drt.h): the frame is rendered on the GPU
//
// Everything is in namespace drt (a `using namespace drt;` after the include gives the
// reference's spelling).  The scalar Traverse / hit / GetSkyboxColor calls are the host path
// "for CPU use and tests" (SURVEY.md §8b): one ray at a time, no device involved; bulk queries go
// to the GPU through drt_trace_closest / drt_trace_shadow / drt_trace_device (include/drt.h).
//
// Numerics: the library is compiled with -ffp-contract=off and keeps the reference's operand
// order and float/double promotions, so builds, camera frames and CPU hits are bit-identical to
// the reference's (tests/test_cpp_api.py, tests/golden/).
//
// Skyboxes: the reference decodes the six JPEG faces with DevIL (scene.cpp:329-378).  LoadSkybox
// reads each face through the decoder registered with drt_set_image_decoder (include/drt_host.h;
// a caller with DevIL, stb_image or libjpeg plugs it in there), and without one reads binary PPM
// (P6) files <dir>/<face>.ppm.  Faces decoded elsewhere can be attached with SetSkyboxFace.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <istream>
#include <memory>
#include <ostream>
#include <string>
#include <vector>

#include "drt.h"

namespace drt {

// ---------------------------------------------------------------- Vector (vector.h, vector.cpp)
class Vector {
 public:
  float x = 0.f, y = 0.f, z = 0.f;
  Vector() = default;
  Vector(float a, float b, float c) : x(a), y(b), z(c) {}
  explicit Vector(float a) : x(a), y(a), z(a) {}
  float length() const { return std::sqrt(x * x + y * y + z * z); }
  float getAxisValue(int axis) const { return axis == 0 ? x : (axis == 1 ? y : z); }
  Vector& normalize() {  // vector.cpp:68-73: the scale is 1.0 / length in double, then float
    float l = (float)(1.0 / (double)length());
    x *= l; y *= l; z *= l;
    return *this;
  }
  Vector operator+(const Vector& v) const { return Vector(x + v.x, y + v.y, z + v.z); }
  Vector operator-(const Vector& v) const { return Vector(x - v.x, y - v.y, z - v.z); }
  Vector operator-() const { return Vector(-x, -y, -z); }
  Vector operator*(float f) const { return Vector(x * f, y * f, z * f); }
  float operator*(const Vector& v) const { return x * v.x + y * v.y + z * v.z; }  // inner product
  Vector operator/(float f) const { return Vector(x / f, y / f, z / f); }
  Vector operator%(const Vector& v) const {  // external product (vector.cpp:87-101)
    return Vector(y * v.z - z * v.y, z * v.x - x * v.z, x * v.y - y * v.x);
  }
  Vector& operator-=(const Vector& v) { x -= v.x; y -= v.y; z -= v.z; return *this; }
  Vector& operator-=(float v) { x -= v; y -= v; z -= v; return *this; }
  Vector& operator+=(float v) { x += v; y += v; z += v; return *this; }
  Vector& operator*=(float v) { x *= v; y *= v; z *= v; return *this; }
  // vector.cpp:60-66, as written: != holds only when all three components differ
  bool operator!=(const Vector& v) const { return x != v.x && y != v.y && z != v.z; }
  bool operator==(const Vector& v) const { return x == v.x && y == v.y && z == v.z; }
  friend std::istream& operator>>(std::istream& s, Vector& v) { return s >> v.x >> v.y >> v.z; }
  friend std::ostream& operator<<(std::ostream& os, const Vector& v) {
    return os << "(" << v.x << ", " << v.y << ", " << v.z << ")";
  }
};

// ---------------------------------------------------------------- Color (color.h:11-75)
class Color {
 public:
  Color() = default;
  Color(float r, float g, float b) : R(r), G(g), B(b) {}
  float r() const { return R; }
  float r(float v) { return R = v; }
  float g() const { return G; }
  float g(float v) { return G = v; }
  float b() const { return B; }
  float b(float v) { return B = v; }
  // CLAMP(0.0, x, 1.0) of color.h:9 compares in double: NaN stays NaN, -0 stays -0
  Color clamp() const { return Color(clamp01(R), clamp01(G), clamp01(B)); }
  Color exp_() const { return Color(std::exp(R), std::exp(G), std::exp(B)); }
  Color operator*(float c) const { return Color(R * c, G * c, B * c); }
  Color operator*=(float c) { R *= c; G *= c; B *= c; return *this; }
  Color operator+(const Color& c) const { return Color(R + c.R, G + c.G, B + c.B); }
  Color operator-(const Color& c) const { return Color(R - c.R, G - c.G, B - c.B); }
  Color operator*(const Color& c) const { return Color(R * c.R, G * c.G, B * c.B); }
  Color operator+=(const Color& c) { R += c.R; G += c.G; B += c.B; return *this; }
  Color operator*=(const Color& c) { R *= c.R; G *= c.G; B *= c.B; return *this; }
  friend std::istream& operator>>(std::istream& s, Color& c) { return s >> c.R >> c.G >> c.B; }

 private:
  static float clamp01(float v) { return (float)(((double)v < 0.0) ? 0.0 : (((double)v > 1.0) ? 1.0 : (double)v)); }
  float R = 0.f, G = 0.f, B = 0.f;
};

// ---------------------------------------------------------------- Ray (ray.h)
struct Ray {
  Ray() = default;
  Ray(const Vector& o, const Vector& d, float t = 0.0f) : origin(o), direction(d), time(t) {}
  Vector origin, direction;
  float time = 0.f;  // motion blur (unused by the reference's renderer)
};

// ---------------------------------------------------------------- AABB (boundingBox.h/.cpp)
class AABB {
 public:
  Vector min{-1.f, -1.f, -1.f}, max{1.f, 1.f, 1.f};  // default box: boundingBox.cpp:8-12
  AABB() = default;
  AABB(const Vector& a, const Vector& b) : min(a), max(b) {}
  Vector centroid() const { return (min + max) / 2.0f; }
  void extend(const AABB& b) {  // boundingBox.cpp:52-62
    if (min.x > b.min.x) min.x = b.min.x;
    if (min.y > b.min.y) min.y = b.min.y;
    if (min.z > b.min.z) min.z = b.min.z;
    if (max.x < b.max.x) max.x = b.max.x;
    if (max.y < b.max.y) max.y = b.max.y;
    if (max.z < b.max.z) max.z = b.max.z;
  }
  bool isInside(const Vector& p) const;      // boundingBox.cpp:41-44 (strict)
  bool hit(const Ray& r, float& t) const;    // boundingBox.cpp:64-124 (slabs, 1.0/d in double)
};

struct HitRecord {  // scene.h:24-31
  bool isHit = false;
  Vector normal;
  float t = FLT_MAX;
};

typedef enum { PUNCTUAL, QUAD } lightType;                   // scene.h:16
typedef enum { RIGHT, LEFT, TOP, BOTTOM, FRONT, BACK } CubeMap;  // scene.h:19
typedef enum { NONE, GRID_ACC, BVH_ACC } accelerator;        // scene.h:22

// ---------------------------------------------------------------- Material (scene.h:34-66)
class Material {
 public:
  Material() = default;
  Material(const Color& c, float Kd, const Color& cs, float Ks, float Shine, float T, float ior)
      : diff_(c), spec_(cs), refl_(Ks), T_(T), kd_(Kd), shine_(Shine), ks_(Ks), ior_(ior) {}
  Color GetDiffColor() const { return diff_; }
  Color GetSpecColor() const { return spec_; }
  float GetDiffuse() const { return kd_; }
  float GetSpecular() const { return ks_; }
  float GetShine() const { return shine_; }
  float GetReflection() const { return refl_; }
  float GetTransmittance() const { return T_; }
  float GetRefrIndex() const { return ior_; }
  void SetDiffColor(const Color& c) { diff_ = c; }
  void SetSpecColor(const Color& c) { spec_ = c; }
  void SetDiffuse(float v) { kd_ = v; }
  void SetSpecular(float v) { ks_ = v; }
  void SetShine(float v) { shine_ = v; }
  void SetReflection(float r) { refl_ = r; }
  void SetTransmittance(float v) { T_ = v; }
  void SetRefrIndex(float v) { ior_ = v; }
  int index = -1;  // position in the scene's material table

 private:
  Color diff_{0.2f, 0.2f, 0.2f}, spec_{1.f, 1.f, 1.f};
  float refl_ = 1.0f, T_ = 0.0f, kd_ = 0.2f, shine_ = 20.f, ks_ = 0.8f, ior_ = 1.0f;
};

// ---------------------------------------------------------------- Light (scene.h:68-107)
class Light {
 public:
  Light(const Vector& pos, const Color& col, const Vector& v1, const Vector& v2, unsigned grid_res)
      : position(pos), emission(col), type(QUAD), gridRes(grid_res), e1(v1 - pos), e2(v2 - pos) {}
  Light(const Vector& pos, const Color& col) : position(pos), emission(col), type(PUNCTUAL) {}
  Vector getAreaLightPoint(const Vector& sample) const {  // scene.h:103-106: spans from pos
    return position + e1 * sample.x + e2 * sample.y;
  }
  Vector position;
  Color emission;
  lightType type;
  unsigned gridRes = 0;
  Vector e1, e2;  // quad frame (scene.h:90-91)
};

// ---------------------------------------------------------------- Objects (scene.h:109-180)
class Object {
 public:
  virtual ~Object() = default;
  Material* GetMaterial() const { return m_Material; }
  void SetMaterial(Material* m) { m_Material = m; }
  virtual HitRecord hit(const Ray& r) const = 0;                   // CPU intersection
  virtual AABB GetBoundingBox() const { return AABB(); }  // planes keep [-1,1]^3 (scene.h:116)
  Vector getCentroid() const { return GetBoundingBox().centroid(); }
  virtual drt_prim pack() const = 0;  // the device record (drt_upload_scene)
  bool motion_blur_enabled = false;   // scene.h:118 (never set by the reference)
  int32_t scene_index = -1;           // position in the owning Scene

 protected:
  Material* m_Material = nullptr;
};

class Triangle : public Object {
 public:
  Triangle(const Vector& P0, const Vector& P1, const Vector& P2);  // scene.cpp:10-35 (box +-EPSILON)
  AABB GetBoundingBox() const override { return AABB(Min, Max); }
  HitRecord hit(const Ray& r) const override;  // Moller-Trumbore, scene.cpp:44-92
  drt_prim pack() const override;
  Vector points[3];

 private:
  Vector Min, Max;
};

class Sphere : public Object {
 public:
  Sphere(const Vector& c, float r) : center(c), radius(r) {}
  AABB GetBoundingBox() const override {
    return AABB(center - Vector(radius, radius, radius), center + Vector(radius, radius, radius));
  }
  HitRecord hit(const Ray& r) const override;  // scene.cpp:152-197
  drt_prim pack() const override;
  Vector center;
  float radius;
  Vector velocity{0.f, 0.f, 0.f};  // motion vector (dead upstream)
};

class Plane : public Object {
 public:
  Plane(const Vector& PN, float D) : PN(PN), D(D) {}
  Plane(const Vector& P0, const Vector& P1, const Vector& P2);  // scene.cpp:100-114
  HitRecord hit(const Ray& r) const override;                    // scene.cpp:118-149
  drt_prim pack() const override;
  Vector PN;
  float D = 0.f;
};

class aaBox : public Object {
 public:
  aaBox(const Vector& mn, const Vector& mx) : min(mn), max(mx) {}
  AABB GetBoundingBox() const override { return AABB(min, max); }
  HitRecord hit(const Ray& r) const override;  // slabs, scene.cpp:218-278
  drt_prim pack() const override;
  Vector min, max;
};

// ---------------------------------------------------------------- Camera (camera.h)
class Camera {
 public:
  Camera(Vector from, Vector At, Vector Up, float angle, float hither, float yon, int ResX, int ResY,
         float Aperture_ratio, float Focal_ratio);  // camera.h:32-61
  void SetEye(Vector from);                         // camera.h:63-72
  Ray PrimaryRay(const Vector& pixel_sample) const;                            // camera.h:74-83
  Ray PrimaryRay(const Vector& lens_sample, const Vector& pixel_sample) const;  // camera.h:86-101
  Vector GetEye() const { return eye; }
  int GetResX() const { return res_x; }
  int GetResY() const { return res_y; }
  float GetFov() const { return fovy; }
  float GetPlaneDist() const { return plane_dist; }
  float GetFar() const { return vfar; }
  float GetAperture() const { return aperture; }
  drt_camera frame() const;  // what the GPU consumes

 private:
  Vector eye, at, up;
  float fovy, vnear, vfar, plane_dist, focal_ratio, aperture;
  float w, h;
  int res_x, res_y;
  Vector u, v, n;
};

// ---------------------------------------------------------------- Scene (scene.h:183-231)
struct SkyboxFace {
  std::vector<uint8_t> img;  // rows bottom-up (IL_ORIGIN_LOWER_LEFT, scene.cpp:345)
  int resX = 0, resY = 0, BPP = 3;
};

class Scene {
 public:
  Scene();
  virtual ~Scene();
  Scene(const Scene&) = delete;
  Scene& operator=(const Scene&) = delete;
  Camera* GetCamera() { return camera.get(); }
  const Camera* GetCamera() const { return camera.get(); }
  Color GetBackgroundColor() const { return bgColor; }
  bool GetSkyBoxFlg() const { return SkyBoxFlg; }
  Color GetSkyboxColor(const Ray& r) const;  // cube-map lookup, scene.cpp:380-458
  unsigned GetSamplesPerPixel() const { return samples_per_pixel; }
  accelerator GetAccelStruct() const { return accel_struc_type; }
  void SetBackgroundColor(const Color& c) { bgColor = c; }
  void SetSkyBoxFlg(bool f) { SkyBoxFlg = f; }
  // scene.cpp:329-378: the faces <dir>/{right,left,top,bottom,front,back}, rows bottom-up.
  // Returns false (faces left empty) where the reference exit()s.
  bool LoadSkybox(const char* sky_dir);
  void SetCamera(Camera* c) { camera.reset(c); }  // takes ownership
  void SetAccelStruct(accelerator a) { accel_struc_type = a; }
  void SetSamplesPerPixel(unsigned spp) { samples_per_pixel = spp; }
  int getNumObjects() const { return (int)objects.size(); }
  void addObject(Object* o);  // takes ownership
  Object* getObject(unsigned i) const { return i < objects.size() ? objects[i] : nullptr; }
  int getNumLights() const { return (int)lights.size(); }
  void addLight(Light* l) { lights.push_back(l); }  // takes ownership
  Light* getLight(unsigned i) const { return i < lights.size() ? lights[i] : nullptr; }
  Material* addMaterial(const Material& m);
  int getNumMaterials() const { return (int)materials.size(); }
  // scene.cpp:474-740.  `env <dir>` loads the skybox from <dir> relative to the working
  // directory (the reference's rule), else relative to the scene file's parent directory's
  // parent (P3D_Scenes/../<dir>); if neither decodes, the flag is set and the faces stay empty.
  bool load_p3f(const char* name);
  const std::string& GetSkyboxDir() const { return env_dir; }
  void SetSkyboxFace(int face, int w, int h, int bpp, const uint8_t* bottom_up);
  bool SkyboxComplete() const;
  // Bulk triangle insertion (the mesh fast path): n triangles, 9 floats each.
  void addTriangles(const float* verts, size_t n, Material* m);
  // Pack everything the GPU needs (camera, lights, materials, primitives, skybox).
  void describe(drt_scene_desc& d, std::vector<drt_prim>& prims, std::vector<drt_light>& ls,
                std::vector<drt_material>& ms) const;
  std::vector<Object*>& objectList() { return objects; }
  const std::vector<Object*>& objectList() const { return objects; }

 private:
  std::vector<Object*> objects;
  std::vector<Light*> lights;
  std::vector<std::unique_ptr<Material>> materials;
  std::vector<std::unique_ptr<std::vector<Triangle>>> tri_pools;  // bulk-inserted triangles
  std::vector<Object*> owned;                         // individually allocated objects
  std::unique_ptr<Camera> camera;
  Color bgColor;
  unsigned samples_per_pixel = 0;
  accelerator accel_struc_type = NONE;
  bool SkyBoxFlg = false;
  std::string env_dir;
  SkyboxFace skybox_img[6];
};

// ---------------------------------------------------------------- accelerators (rayAccelerator.h)
class BVH {
 public:
  struct Node {  // BVHNode (rayAccelerator.h:50-67)
    AABB bbox;
    bool leaf = false;
    uint32_t n_objs = 0;
    uint32_t index = 0;  // inner: left child (right = index + 1); leaf: first object
  };
  BVH() = default;
  int getNumObjects() const { return (int)objects.size(); }
  void Build(std::vector<Object*>& objs);  // bvh.cpp:27-227, tree-identical (threaded)
  // Scalar queries on the CPU (bvh.cpp:231-314 closest, :316-391 shadow: normalises `ray`,
  // occluded if a hit lies within |d| + EPSILON)
  bool Traverse(Ray& ray, Object** hit_obj, HitRecord& hitRec) const;
  bool Traverse(Ray& ray) const;
  const std::vector<Node>& nodeList() const { return nodes; }
  const std::vector<Object*>& objectOrder() const { return objects; }
  int upload(drt_ctx* ctx) const;  // drt_upload_bvh
  double build_ms = 0.0;

 private:
  std::vector<Object*> objects;
  std::vector<Node> nodes;
  std::vector<AABB> boxes_;    // per input position
  std::vector<Vector> cents_;  // centroid per input position
  std::vector<int> order_;     // permutation being sorted (positions into boxes_/cents_)
};

class Grid {
 public:
  Grid() = default;
  int getNumObjects() const { return (int)objects.size(); }
  void addObject(Object* o) { objects.push_back(o); }   // grid.cpp:17-20
  Object* getObject(unsigned index) const { return index < objects.size() ? objects[index] : nullptr; }
  void setAABB(const AABB& b) { bbox = b; }
  void Build(std::vector<Object*>& objs);  // grid.cpp:30-97 (appends objs to the object list)
  // Scalar queries on the CPU (grid.cpp:247-306 closest, :309-358 shadow: range |d|, and a
  // ray that misses the grid box counts as shadowed)
  bool Traverse(Ray& ray, Object** hitobject, HitRecord& hitRec) const;
  bool Traverse(Ray& ray) const;
  int upload(drt_ctx* ctx) const;  // drt_upload_grid
  int nx = 0, ny = 0, nz = 0;
  AABB bbox;
  std::vector<int64_t> cell_start;  // CSR over cells x + nx*(y + ny*z); insertion order kept
  std::vector<int32_t> cell_objs;   // positions in the object list
  double build_ms = 0.0;

 private:
  bool Init_Traverse(const Ray& ray, int& ix, int& iy, int& iz, double& dtx, double& dty, double& dtz,
                     double& tx_next, double& ty_next, double& tz_next, int& ix_step, int& iy_step, int& iz_step,
                     int& ix_stop, int& iy_stop, int& iz_stop) const;  // grid.cpp:100-244
  std::vector<Object*> objects;
  float m = 2.0f;
};

// renderScene() replacement (main.cpp:525-738): upload the scene and its accelerator into a
// context (include/drt.h), then render whole frames into `colors` (RES_Y*RES_X*3 floats, row 0 =
// bottom) on the GPU.  Return drt_status codes.
int upload_scene(drt_ctx* ctx, const Scene& scene, const BVH* bvh, const Grid* grid);
int render_scene(drt_ctx* ctx, const drt_frame_params& params, float* colors);
// The per-frame camera of the interactive renderer (main.cpp:530-533: SetEye, then renderScene):
// the camera's current frame replaces the context's (drt_set_camera); the scene stays resident.
int set_camera(drt_ctx* ctx, const Camera& camera);
int set_camera(drt_group* group, const Camera& camera);
// The same over several GPUs (include/drt.h, drt_group_*): the scene on every device, each frame
// tile-sharded, all-gathered over RCCL and reassembled on device 0.
int upload_scene(drt_group* group, const Scene& scene, const BVH* bvh, const Grid* grid);
int render_scene(drt_group* group, const drt_frame_params& params, float* colors);

}  // namespace drt
