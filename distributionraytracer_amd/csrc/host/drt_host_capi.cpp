// drt_host_capi.cpp — C entry points (include/drt_host.h) over the C++ host scene API.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../../include/drt_host.h"
#include "../../../include/drt_scene.hpp"

using namespace drt;

struct drt_scene {
  Scene scene;
  BVH bvh;
  Grid grid;
  // a triangle Grid scene's BVH for its shadow tree (drt_upload_grid_shadow_bvh; DRT_GRID_SHADOW_TREE=0: none)
  BVH gv_bvh;
  bool has_gv_bvh = false;
  Material* current = nullptr;
  bool built = false;
};

static Vector v3(const float* p) { return Vector(p[0], p[1], p[2]); }

extern "C" {

drt_scene* drt_scene_new(void) { return new drt_scene(); }

drt_scene* drt_scene_load_p3f(const char* path) {
  if (!path) return nullptr;
  drt_scene* s = new drt_scene();
  if (!s->scene.load_p3f(path)) {
    delete s;
    return nullptr;
  }
  return s;
}

void drt_scene_free(drt_scene* s) { delete s; }

int drt_scene_info(const drt_scene* s, drt_scene_info_t* o) {
  if (!s || !o) return DRT_E_INVALID;
  memset(o, 0, sizeof(*o));
  Scene& sc = const_cast<Scene&>(s->scene);
  if (Camera* c = sc.GetCamera()) {
    o->res_x = c->GetResX();
    o->res_y = c->GetResY();
    o->aperture = c->GetAperture();
  }
  o->spp = sc.GetSamplesPerPixel();
  o->accel = sc.GetAccelStruct() == BVH_ACC ? DRT_ACCEL_BVH : (sc.GetAccelStruct() == GRID_ACC ? DRT_ACCEL_GRID : DRT_ACCEL_NONE);
  o->n_objects = sc.getNumObjects();
  o->n_lights = sc.getNumLights();
  o->n_materials = sc.getNumMaterials();  // (not describe(): that packs every primitive)
  o->has_env = sc.GetSkyBoxFlg() ? 1 : 0;
  o->skybox_loaded = sc.SkyboxComplete() ? 1 : 0;
  o->bvh_nodes = (int32_t)s->bvh.nodeList().size();
  o->build_ms = o->accel == DRT_ACCEL_GRID ? s->grid.build_ms : s->bvh.build_ms;
  return DRT_OK;
}

const char* drt_scene_env(const drt_scene* s) { return s ? s->scene.GetSkyboxDir().c_str() : ""; }

int drt_scene_set_skybox_face(drt_scene* s, int face, int w, int h, int bpp, const uint8_t* px) {
  if (!s || !px || face < 0 || face > 5 || w <= 0 || h <= 0 || (bpp != 3 && bpp != 4)) return DRT_E_INVALID;
  s->scene.SetSkyboxFace(face, w, h, bpp, px);
  return DRT_OK;
}

int drt_scene_set_camera(drt_scene* s, const float eye[3], const float at[3], const float up[3], float fovy,
                         float hither, int rx, int ry, float ap, float fr) {
  if (!s || rx <= 0 || ry <= 0) return DRT_E_INVALID;
  s->scene.SetCamera(new Camera(v3(eye), v3(at), v3(up), fovy, hither, (float)(1000.0 * hither), rx, ry, ap, fr));
  return DRT_OK;
}

int drt_scene_set_background(drt_scene* s, const float rgb[3]) {
  if (!s) return DRT_E_INVALID;
  s->scene.SetBackgroundColor(Color(rgb[0], rgb[1], rgb[2]));
  return DRT_OK;
}

int drt_scene_set_accel(drt_scene* s, int a) {
  if (!s || a < 0 || a > 2) return DRT_E_INVALID;
  s->scene.SetAccelStruct(a == DRT_ACCEL_BVH ? BVH_ACC : (a == DRT_ACCEL_GRID ? GRID_ACC : NONE));
  s->built = false;
  return DRT_OK;
}

int drt_scene_set_spp(drt_scene* s, uint32_t spp) {
  if (!s) return DRT_E_INVALID;
  s->scene.SetSamplesPerPixel(spp);
  return DRT_OK;
}

int drt_scene_add_material(drt_scene* s, const float d[3], double kd, const float sp[3], double ks, double shine,
                           double t, double ior) {
  if (!s) return DRT_E_INVALID;
  s->current = s->scene.addMaterial(
      Material(Color(d[0], d[1], d[2]), (float)kd, Color(sp[0], sp[1], sp[2]), (float)ks, (float)shine, (float)t, (float)ior));
  return s->current->index;
}

int drt_scene_use_material(drt_scene* s, int m) {
  (void)s; (void)m;
  return DRT_E_UNSUPPORTED;  // materials apply to the objects that follow them, as in P3F
}

static int add(drt_scene* s, Object* o) {
  if (s->current) o->SetMaterial(s->current);
  s->scene.addObject(o);
  s->built = false;
  return s->scene.getNumObjects() - 1;
}

int drt_scene_add_sphere(drt_scene* s, const float c[3], float r) { return s ? add(s, new Sphere(v3(c), r)) : DRT_E_INVALID; }
int drt_scene_add_plane_pts(drt_scene* s, const float a[3], const float b[3], const float c[3]) {
  return s ? add(s, new Plane(v3(a), v3(b), v3(c))) : DRT_E_INVALID;
}
int drt_scene_add_plane_nd(drt_scene* s, const float n[3], float d) { return s ? add(s, new Plane(v3(n), d)) : DRT_E_INVALID; }
int drt_scene_add_box(drt_scene* s, const float a[3], const float b[3]) { return s ? add(s, new aaBox(v3(a), v3(b))) : DRT_E_INVALID; }
int drt_scene_add_triangles(drt_scene* s, const float* v, int64_t n) {
  if (!s || n < 0 || (n && !v)) return DRT_E_INVALID;
  s->scene.addTriangles(v, (size_t)n, s->current);
  s->built = false;
  return s->scene.getNumObjects() - 1;
}
int drt_scene_add_light_point(drt_scene* s, const float p[3], const float c[3]) {
  if (!s) return DRT_E_INVALID;
  s->scene.addLight(new Light(v3(p), Color(c[0], c[1], c[2])));
  return s->scene.getNumLights() - 1;
}
int drt_scene_add_light_quad(drt_scene* s, const float p[3], const float c[3], const float a[3], const float b[3],
                             uint32_t g) {
  if (!s) return DRT_E_INVALID;
  s->scene.addLight(new Light(v3(p), Color(c[0], c[1], c[2]), v3(a), v3(b), g));
  return s->scene.getNumLights() - 1;
}

int drt_scene_build(drt_scene* s) {  // main.cpp:1023-1049
  if (!s) return DRT_E_INVALID;
  std::vector<Object*> objs = s->scene.objectList();
  if (s->scene.GetAccelStruct() == BVH_ACC) {
    s->bvh = BVH();
    s->bvh.Build(objs);
  } else if (s->scene.GetAccelStruct() == GRID_ACC) {
    s->grid = Grid();  // Grid::Build appends to the grid's object list (grid.cpp:45)
    s->grid.Build(objs);
    // the Grid frame's shadow queries walk a tree of the same objects (triangle scenes, round 6)
    const char* e = getenv("DRT_GRID_SHADOW_TREE");
    bool tri = !objs.empty() && !(e && atoi(e) == 0);
    for (Object* o : objs)
      if (!dynamic_cast<Triangle*>(o)) { tri = false; break; }
    s->gv_bvh = BVH();
    s->has_gv_bvh = tri;
    if (tri) s->gv_bvh.Build(objs);
  } else {
    s->has_gv_bvh = false;
  }
  s->built = true;
  return DRT_OK;
}

int drt_scene_bvh_export(const drt_scene* s, float* boxes, uint32_t* leaf, uint32_t* index, uint32_t* nobjs,
                         int32_t* order) {
  if (!s) return DRT_E_INVALID;
  const auto& nd = s->bvh.nodeList();
  for (size_t i = 0; i < nd.size(); i++) {
    const AABB& b = nd[i].bbox;
    float* o = boxes + 6 * i;
    o[0] = b.min.x; o[1] = b.min.y; o[2] = b.min.z; o[3] = b.max.x; o[4] = b.max.y; o[5] = b.max.z;
    leaf[i] = nd[i].leaf;
    index[i] = nd[i].index;
    nobjs[i] = nd[i].leaf ? nd[i].n_objs : 0;
  }
  const auto& ob = s->bvh.objectOrder();
  for (size_t i = 0; i < ob.size(); i++) order[i] = ob[i]->scene_index;
  return DRT_OK;
}

int drt_scene_grid_export_dims(const drt_scene* s, int32_t dims[3], float bmin[3], float bmax[3], int64_t* n_refs) {
  if (!s) return DRT_E_INVALID;
  const Grid& g = s->grid;
  dims[0] = g.nx; dims[1] = g.ny; dims[2] = g.nz;
  bmin[0] = g.bbox.min.x; bmin[1] = g.bbox.min.y; bmin[2] = g.bbox.min.z;
  bmax[0] = g.bbox.max.x; bmax[1] = g.bbox.max.y; bmax[2] = g.bbox.max.z;
  *n_refs = (int64_t)g.cell_objs.size();
  return DRT_OK;
}

int drt_scene_grid_export(const drt_scene* s, int64_t* cs, int32_t* co) {
  if (!s) return DRT_E_INVALID;
  memcpy(cs, s->grid.cell_start.data(), sizeof(int64_t) * s->grid.cell_start.size());
  memcpy(co, s->grid.cell_objs.data(), sizeof(int32_t) * s->grid.cell_objs.size());
  return DRT_OK;
}

int drt_scene_camera_frame(const drt_scene* s, drt_camera* out) {
  if (!s || !out) return DRT_E_INVALID;
  Camera* c = const_cast<Scene&>(s->scene).GetCamera();
  if (!c) return DRT_E_STATE;
  *out = c->frame();
  return DRT_OK;
}

int drt_scene_set_eye(drt_scene* s, const float eye[3]) {
  if (!s || !eye) return DRT_E_INVALID;
  Camera* c = s->scene.GetCamera();
  if (!c) return DRT_E_STATE;
  c->SetEye(Vector(eye[0], eye[1], eye[2]));
  return DRT_OK;
}

int drt_scene_upload_camera(drt_ctx* ctx, const drt_scene* s) {
  if (!ctx || !s) return DRT_E_INVALID;
  const Camera* c = s->scene.GetCamera();
  if (!c) return DRT_E_STATE;
  return set_camera(ctx, *c);
}

int drt_group_scene_upload_camera(drt_group* g, const drt_scene* s) {
  if (!g || !s) return DRT_E_INVALID;
  const Camera* c = s->scene.GetCamera();
  if (!c) return DRT_E_STATE;
  return set_camera(g, *c);
}

int drt_scene_upload(drt_ctx* ctx, drt_scene* s) {
  if (!ctx || !s) return DRT_E_INVALID;
  if (!s->scene.GetCamera()) return DRT_E_STATE;
  if (s->scene.GetSkyBoxFlg() && !s->scene.SkyboxComplete()) return DRT_E_STATE;
  if (!s->built) drt_scene_build(s);
  const int rc = upload_scene(ctx, s->scene, &s->bvh, &s->grid);
  if (rc || !s->has_gv_bvh || s->scene.GetAccelStruct() != GRID_ACC) return rc;
  const auto& nd = s->gv_bvh.nodeList();
  std::vector<drt_bvh_node> n(nd.size());
  for (size_t i = 0; i < nd.size(); i++) {
    const AABB& b = nd[i].bbox;
    n[i].bmin[0] = b.min.x; n[i].bmin[1] = b.min.y; n[i].bmin[2] = b.min.z;
    n[i].bmax[0] = b.max.x; n[i].bmax[1] = b.max.y; n[i].bmax[2] = b.max.z;
    n[i].leaf = nd[i].leaf ? 1u : 0u;
    n[i].index = nd[i].index;
    n[i].n_objs = nd[i].leaf ? nd[i].n_objs : 0u;
  }
  const auto& ob = s->gv_bvh.objectOrder();
  std::vector<uint32_t> ord(ob.size());
  for (size_t i = 0; i < ob.size(); i++) ord[i] = (uint32_t)ob[i]->scene_index;
  // without a tree the Grid walk answers every query: a tree the device cannot take is no error
  const int g = drt_upload_grid_shadow_bvh(ctx, n.data(), (uint32_t)n.size(), ord.data(), (uint32_t)ord.size());
  return g == DRT_E_UNSUPPORTED ? DRT_OK : g;
}

int drt_group_scene_upload(drt_group* g, drt_scene* s) {
  if (!g || !s) return DRT_E_INVALID;
  const int n = drt_group_size(g);
  for (int r = 0; r < n; r++) {  // the scene is replicated on every device
    const int rc = drt_scene_upload(drt_group_ctx(g, r), s);
    if (rc) return rc;
  }
  return DRT_OK;
}

int drt_scene_load_skybox(drt_scene* s, const char* dir) {
  if (!s || !dir) return DRT_E_INVALID;
  if (!s->scene.LoadSkybox(dir)) return DRT_E_INVALID;
  s->scene.SetSkyBoxFlg(true);
  return DRT_OK;
}

int drt_scene_trace_cpu(const drt_scene* s, int shadow, const float* rays, int64_t n, float* t, float* normal,
                        int32_t* object, uint8_t* occluded) {
  if (!s || n < 0 || (n && !rays)) return DRT_E_INVALID;
  if (shadow ? (n && !occluded) : (n && (!t || !normal || !object))) return DRT_E_INVALID;
  if (!s->built) return DRT_E_STATE;
  const Scene& sc = s->scene;
  const accelerator acc = sc.GetAccelStruct();
  for (int64_t i = 0; i < n; i++) {
    const float* r = rays + 6 * i;
    Ray ray(Vector(r[0], r[1], r[2]), Vector(r[3], r[4], r[5]));
    if (shadow) {
      bool occ = false;
      if (acc == BVH_ACC) occ = s->bvh.Traverse(ray);
      else if (acc == GRID_ACC) occ = s->grid.Traverse(ray);
      else {  // the NONE loop of main.cpp:432-439 without its self-skip (a raw query has no hit
              // object): a hit with t in (1e-4, |d|) along d occludes
        const float len = ray.direction.length();
        for (int k = 0; k < sc.getNumObjects() && !occ; k++) {
          const HitRecord h = sc.getObject((unsigned)k)->hit(ray);
          occ = h.isHit && h.t > 1e-4f && h.t < len;
        }
      }
      occluded[i] = occ ? 1 : 0;
      continue;
    }
    HitRecord rec;
    Object* hit_obj = nullptr;
    bool hit = false;
    if (acc == BVH_ACC) hit = s->bvh.Traverse(ray, &hit_obj, rec);
    else if (acc == GRID_ACC) hit = s->grid.Traverse(ray, &hit_obj, rec);
    else {  // main.cpp:315-326: linear scan, strict <, first object wins ties
      for (int k = 0; k < sc.getNumObjects(); k++) {
        Object* o = sc.getObject((unsigned)k);
        const HitRecord h = o->hit(ray);
        if (h.isHit && h.t < rec.t) { rec = h; hit_obj = o; hit = true; }
      }
    }
    t[i] = hit ? rec.t : FLT_MAX;
    normal[3 * i] = hit ? rec.normal.x : 0.f;
    normal[3 * i + 1] = hit ? rec.normal.y : 0.f;
    normal[3 * i + 2] = hit ? rec.normal.z : 0.f;
    object[i] = hit && hit_obj ? hit_obj->scene_index : -1;
  }
  return DRT_OK;
}

int drt_scene_skybox_color_cpu(const drt_scene* s, const float* dirs, int64_t n, float* rgb) {
  if (!s || n < 0 || (n && (!dirs || !rgb))) return DRT_E_INVALID;
  for (int64_t i = 0; i < n; i++) {
    const Color c = s->scene.GetSkyboxColor(Ray(Vector(0.f, 0.f, 0.f), Vector(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2])));
    rgb[3 * i] = c.r(); rgb[3 * i + 1] = c.g(); rgb[3 * i + 2] = c.b();
  }
  return DRT_OK;
}

}  // extern "C"
