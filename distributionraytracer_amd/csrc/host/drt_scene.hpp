// drt_scene.hpp — host C++ API mirroring the reference's scene.h / camera.h / rayAccelerator.h
// (rita-mota/DistributionRayTracer, DistributionRayTracer/), so a main.cpp written against the
// reference keeps compiling: Scene::load_p3f, Scene getters, Camera, Light, Material,
// Object/Triangle/Sphere/Plane/aaBox, BVH::Build/Traverse, Grid::Build/Traverse.
//
// What changed: there is no CPU intersection code.  Object has no hit(); BVH::Traverse and
// Grid::Traverse run on the GPU through the C ABI (include/drt.h) against the context the
// structure was bound to, and renderScene() becomes drt::render_scene().  The host keeps
// what must stay on the host: parsing, the accelerator BUILD (tree-identical to
// bvh.cpp:27-227 and grid.cpp:30-97) and packing for upload.
//
// Numerics: compiled with -ffp-contract=off; every expression that feeds a value the GPU
// consumes (camera frame, triangle boxes, BVH boxes and split decisions) keeps the
// reference's operand order and float/double promotions.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/drt.h"

namespace drt {

// ---------------------------------------------------------------- Vector (vector.h)
class Vector {
 public:
  float x = 0.f, y = 0.f, z = 0.f;
  Vector() = default;
  Vector(float a, float b, float c) : x(a), y(b), z(c) {}
  explicit Vector(float a) : x(a), y(a), z(a) {}
  float length() const { return std::sqrt(x * x + y * y + z * z); }
  float getAxisValue(int axis) const { return axis == 0 ? x : (axis == 1 ? y : z); }
  Vector& normalize() {
    float l = (float)(1.0 / (double)length());
    x *= l; y *= l; z *= l;
    return *this;
  }
  Vector operator+(const Vector& v) const { return Vector(x + v.x, y + v.y, z + v.z); }
  Vector operator-(const Vector& v) const { return Vector(x - v.x, y - v.y, z - v.z); }
  Vector operator-() const { return Vector(-x, -y, -z); }
  Vector operator*(float f) const { return Vector(x * f, y * f, z * f); }
  float operator*(const Vector& v) const { return x * v.x + y * v.y + z * v.z; }
  Vector operator/(float f) const { return Vector(x / f, y / f, z / f); }
  Vector operator%(const Vector& v) const {
    return Vector(y * v.z - z * v.y, z * v.x - x * v.z, x * v.y - y * v.x);
  }
};

// ---------------------------------------------------------------- Color (color.h)
class Color {
 public:
  Color() = default;
  Color(float r, float g, float b) : R(r), G(g), B(b) {}
  float r() const { return R; }
  float g() const { return G; }
  float b() const { return B; }

 private:
  float R = 0.f, G = 0.f, B = 0.f;
};

struct Ray {  // ray.h
  Ray() = default;
  Ray(const Vector& o, const Vector& d, float t = 0.0f) : origin(o), direction(d), time(t) {}
  Vector origin, direction;
  float time = 0.f;
};

// ---------------------------------------------------------------- AABB (boundingBox.h)
class AABB {
 public:
  Vector min{-1.f, -1.f, -1.f}, max{1.f, 1.f, 1.f};  // default box: boundingBox.cpp:8-12
  AABB() = default;
  AABB(const Vector& a, const Vector& b) : min(a), max(b) {}
  Vector centroid() const { return (min + max) / 2.0f; }
  void extend(const AABB& b) {
    if (min.x > b.min.x) min.x = b.min.x;
    if (min.y > b.min.y) min.y = b.min.y;
    if (min.z > b.min.z) min.z = b.min.z;
    if (max.x < b.max.x) max.x = b.max.x;
    if (max.y < b.max.y) max.y = b.max.y;
    if (max.z < b.max.z) max.z = b.max.z;
  }
};

struct HitRecord {  // scene.h:24-31
  bool isHit = false;
  Vector normal;
  float t = FLT_MAX;
};

typedef enum { PUNCTUAL, QUAD } lightType;
typedef enum { RIGHT, LEFT, TOP, BOTTOM, FRONT, BACK } CubeMap;
typedef enum { NONE, GRID_ACC, BVH_ACC } accelerator;

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
  void SetReflection(float r) { refl_ = r; }
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
  virtual AABB GetBoundingBox() const { return AABB(); }  // planes keep [-1,1]^3 (scene.h:116)
  Vector getCentroid() const { return GetBoundingBox().centroid(); }
  virtual drt_prim pack() const = 0;
  int32_t scene_index = -1;

 protected:
  Material* m_Material = nullptr;
};

class Triangle : public Object {
 public:
  Triangle(const Vector& P0, const Vector& P1, const Vector& P2);
  AABB GetBoundingBox() const override { return AABB(Min, Max); }
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
  drt_prim pack() const override;
  Vector center;
  float radius;
};

class Plane : public Object {
 public:
  Plane(const Vector& PN, float D) : PN(PN), D(D) {}
  Plane(const Vector& P0, const Vector& P1, const Vector& P2);
  drt_prim pack() const override;
  Vector PN;
  float D = 0.f;
};

class aaBox : public Object {
 public:
  aaBox(const Vector& mn, const Vector& mx) : min(mn), max(mx) {}
  AABB GetBoundingBox() const override { return AABB(min, max); }
  drt_prim pack() const override;
  Vector min, max;
};

// ---------------------------------------------------------------- Camera (camera.h)
class Camera {
 public:
  Camera(Vector from, Vector At, Vector Up, float angle, float hither, float yon, int ResX, int ResY,
         float Aperture_ratio, float Focal_ratio);
  void SetEye(Vector from);  // camera.h:63-72
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
  std::vector<uint8_t> img;  // bottom-up rows
  int resX = 0, resY = 0, BPP = 3;
};

class Scene {
 public:
  Scene();
  ~Scene();
  Camera* GetCamera() { return camera.get(); }
  Color GetBackgroundColor() const { return bgColor; }
  bool GetSkyBoxFlg() const { return SkyBoxFlg; }
  unsigned GetSamplesPerPixel() const { return samples_per_pixel; }
  accelerator GetAccelStruct() const { return accel_struc_type; }
  void SetBackgroundColor(const Color& c) { bgColor = c; }
  void SetSkyBoxFlg(bool f) { SkyBoxFlg = f; }
  void SetCamera(Camera* c) { camera.reset(c); }
  void SetAccelStruct(accelerator a) { accel_struc_type = a; }
  void SetSamplesPerPixel(unsigned spp) { samples_per_pixel = spp; }
  int getNumObjects() const { return (int)objects.size(); }
  void addObject(Object* o);  // takes ownership
  Object* getObject(unsigned i) const { return i < objects.size() ? objects[i] : nullptr; }
  int getNumLights() const { return (int)lights.size(); }
  void addLight(Light* l) { lights.push_back(l); }
  Light* getLight(unsigned i) const { return i < lights.size() ? lights[i] : nullptr; }
  Material* addMaterial(const Material& m);
  bool load_p3f(const char* name);  // scene.cpp:474-740
  // Skybox: `env <dir>` is recorded; the faces (decoded elsewhere, e.g. by PIL) are attached
  // with SetSkyboxFace (LoadSkybox's DevIL decode, scene.cpp:329-378, is not linked here).
  const std::string& GetSkyboxDir() const { return env_dir; }
  void SetSkyboxFace(int face, int w, int h, int bpp, const uint8_t* bottom_up);
  bool SkyboxComplete() const;
  // Bulk triangle insertion (the mesh fast path): n triangles, 9 floats each.
  void addTriangles(const float* verts, size_t n, Material* m);
  // Pack everything the GPU needs (camera, lights, materials, primitives, skybox).
  void describe(drt_scene_desc& d, std::vector<drt_prim>& prims, std::vector<drt_light>& ls,
                std::vector<drt_material>& ms) const;
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
    uint32_t index = 0;
  };
  BVH() = default;
  int getNumObjects() const { return (int)objects.size(); }
  void Build(std::vector<Object*>& objs);  // bvh.cpp:27-44 (tree-identical)
  // GPU-backed queries (bvh.cpp:231-391) against the context this BVH was uploaded to.
  bool Traverse(Ray& ray, Object** hit_obj, HitRecord& hitRec);
  bool Traverse(Ray& ray);
  void bind(drt_ctx* ctx, const Scene* s) { ctx_ = ctx; scene_ = s; }
  const std::vector<Node>& nodeList() const { return nodes; }
  const std::vector<Object*>& objectOrder() const { return objects; }
  int upload(drt_ctx* ctx) const;
  double build_ms = 0.0;

 private:
  void build_range(int left_index, int right_index, int node);
  std::vector<Object*> objects;
  std::vector<Node> nodes;
  std::vector<AABB> boxes_;     // per input position
  std::vector<Vector> cents_;   // centroid per input position
  std::vector<int> order_;      // permutation being sorted (positions into boxes_/cents_)
  drt_ctx* ctx_ = nullptr;
  const Scene* scene_ = nullptr;
};

class Grid {
 public:
  Grid() = default;
  void Build(std::vector<Object*>& objs);  // grid.cpp:30-97
  bool Traverse(Ray& ray, Object** hitobject, HitRecord& hitRec);
  bool Traverse(Ray& ray);
  void bind(drt_ctx* ctx, const Scene* s) { ctx_ = ctx; scene_ = s; }
  int upload(drt_ctx* ctx) const;
  int nx = 0, ny = 0, nz = 0;
  AABB bbox;
  std::vector<int64_t> cell_start;
  std::vector<int32_t> cell_objs;  // scene indices
  double build_ms = 0.0;

 private:
  float m = 2.0f;
  drt_ctx* ctx_ = nullptr;
  const Scene* scene_ = nullptr;
};

// renderScene() replacement (main.cpp:525-738): uploads scene + accelerator once per bind and
// renders whole frames into `colors` (RES_Y*RES_X*3 floats, row 0 = bottom).
int upload_scene(drt_ctx* ctx, const Scene& scene, const BVH* bvh, const Grid* grid);
int render_scene(drt_ctx* ctx, const drt_frame_params& params, float* colors);

}  // namespace drt
