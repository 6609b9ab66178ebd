// drt_accel.cpp — host-side accelerator builds (tree-identical to the reference) + upload glue.
//
// BVH::Build reproduces bvh.cpp:27-227 exactly: binned SAH over 12 buckets spanning the NODE
// box, leaf at <= 2 objects, cost 1 + (nL*AL + nR*AR)/A, fallback leaf when no split beats
// n, std::sort by centroid on each axis (the same libstdc++ introsort over the same key
// sequence, so ties land in the same order), children appended pairwise in recursion order.
// It runs on flat arrays (boxes/centroids computed once) instead of virtual calls per
// comparison; sibling subtrees are independent and built on separate threads, then the
// node array is renumbered into the reference's DFS numbering.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <future>
#include <thread>

#include "../../../include/drt_scene.hpp"

namespace drt {

static constexpr double kEps = 0.001;

static inline float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
static inline float smax(float a, float b) { return (a < b) ? b : a; }  // std::max

namespace {

// A subtree built independently: nodes numbered locally (0 = subtree root), children of an
// inner node at local index and index+1, exactly as build_recursive appends them.
struct SubTree {
  std::vector<BVH::Node> nodes;
  // children whose subtree was built by another task: local node index -> task result
  std::vector<std::pair<int, std::shared_ptr<SubTree>>> deferred;
};

struct Builder {
  std::vector<AABB>& boxes;
  std::vector<Vector>& cents;
  std::vector<int>& order;
  int par_threshold;

  void sort_axis(int l, int r, int axis) {
    // std::sort over (key, position) pairs compared on the key only performs exactly the
    // comparisons — and therefore the moves — of std::sort over Object* with BVH::Comparator.
    std::vector<std::pair<float, int>> kv((size_t)(r - l));
    for (int i = l; i < r; i++) kv[(size_t)(i - l)] = {cents[order[i]].getAxisValue(axis), order[i]};
    std::sort(kv.begin(), kv.end(),
              [](const std::pair<float, int>& a, const std::pair<float, int>& b) { return a.first < b.first; });
    for (int i = l; i < r; i++) order[i] = kv[(size_t)(i - l)].second;
  }

  // bvh.cpp:62-227 on node `node` of `st`; returns nothing, fills st.
  void build(int left_index, int right_index, SubTree& st, int node, std::vector<std::future<void>>& tasks) {
    const int BUCKET_COUNT = 12;
    const float TRAVERSAL_COST = 1.0f, INTERSECTION_COST = 1.0f;
    const int n_objects = right_index - left_index;
    if (n_objects <= 2) {
      st.nodes[node].leaf = true; st.nodes[node].index = left_index; st.nodes[node].n_objs = n_objects;
      return;
    }
    const AABB box = st.nodes[node].bbox;
    const Vector ext = box.max - box.min;
    const float psa = 2.0f * (ext.x * ext.y + ext.x * ext.z + ext.y * ext.z);
    int best_axis = 0;
    float best_cost = FLT_MAX;
    int best_split = left_index;
    for (int axis = 0; axis < 3; axis++) {
      sort_axis(left_index, right_index, axis);
      int cnt[BUCKET_COUNT] = {0};
      Vector bmn[BUCKET_COUNT], bmx[BUCKET_COUNT];
      for (int b = 0; b < BUCKET_COUNT; b++) {
        bmn[b] = Vector(FLT_MAX, FLT_MAX, FLT_MAX);
        bmx[b] = Vector(-FLT_MAX, -FLT_MAX, -FLT_MAX);
      }
      const float min_bound = box.min.getAxisValue(axis), max_bound = box.max.getAxisValue(axis);
      const float scale = (max_bound - min_bound) > 0.0f ? BUCKET_COUNT / (max_bound - min_bound) : 0.0f;
      for (int i = left_index; i < right_index; i++) {
        const int o = order[i];
        const float c = cents[o].getAxisValue(axis);
        const int bi = std::min(BUCKET_COUNT - 1, (int)((c - min_bound) * scale));
        cnt[bi]++;
        const AABB& ob = boxes[o];
        bmn[bi] = Vector(smin(bmn[bi].x, ob.min.x), smin(bmn[bi].y, ob.min.y), smin(bmn[bi].z, ob.min.z));
        bmx[bi] = Vector(smax(bmx[bi].x, ob.max.x), smax(bmx[bi].y, ob.max.y), smax(bmx[bi].z, ob.max.z));
      }
      for (int i = 1; i < BUCKET_COUNT; i++) {
        Vector lmn(FLT_MAX, FLT_MAX, FLT_MAX), lmx(-FLT_MAX, -FLT_MAX, -FLT_MAX);
        Vector rmn(FLT_MAX, FLT_MAX, FLT_MAX), rmx(-FLT_MAX, -FLT_MAX, -FLT_MAX);
        int lc = 0, rc = 0;
        for (int j = 0; j < i; j++) {
          lmn = Vector(smin(lmn.x, bmn[j].x), smin(lmn.y, bmn[j].y), smin(lmn.z, bmn[j].z));
          lmx = Vector(smax(lmx.x, bmx[j].x), smax(lmx.y, bmx[j].y), smax(lmx.z, bmx[j].z));
          lc += cnt[j];
        }
        for (int j = i; j < BUCKET_COUNT; j++) {
          rmn = Vector(smin(rmn.x, bmn[j].x), smin(rmn.y, bmn[j].y), smin(rmn.z, bmn[j].z));
          rmx = Vector(smax(rmx.x, bmx[j].x), smax(rmx.y, bmx[j].y), smax(rmx.z, bmx[j].z));
          rc += cnt[j];
        }
        const Vector le = lmx - lmn, re = rmx - rmn;
        const float la = 2.0f * (le.x * le.y + le.x * le.z + le.y * le.z);
        const float ra = 2.0f * (re.x * re.y + re.x * re.z + re.y * re.z);
        const float cost = TRAVERSAL_COST + (lc * la + rc * ra) * INTERSECTION_COST / psa;
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = axis;
          best_split = left_index + lc;
        }
      }
    }
    if (best_split <= left_index || best_split >= right_index || best_cost >= n_objects * INTERSECTION_COST) {
      st.nodes[node].leaf = true; st.nodes[node].index = left_index; st.nodes[node].n_objs = n_objects;
      return;
    }
    sort_axis(left_index, right_index, best_axis);
    AABB lb(Vector(FLT_MAX, FLT_MAX, FLT_MAX), Vector(-FLT_MAX, -FLT_MAX, -FLT_MAX)), rb = lb;
    for (int i = left_index; i < best_split; i++) lb.extend(boxes[order[i]]);
    for (int i = best_split; i < right_index; i++) rb.extend(boxes[order[i]]);
    const int li = (int)st.nodes.size();
    st.nodes[node].leaf = false;
    st.nodes[node].index = (uint32_t)li;
    BVH::Node ln, rn;
    ln.bbox = lb;
    rn.bbox = rb;
    st.nodes.push_back(ln);
    st.nodes.push_back(rn);
    // Large left subtree: hand it to a task with its own local numbering (spliced back later).
    if (best_split - left_index >= par_threshold && right_index - best_split >= par_threshold) {
      auto sub = std::make_shared<SubTree>();
      sub->nodes.push_back(ln);
      st.deferred.push_back({li, sub});
      const int l0 = left_index, l1 = best_split;
      tasks.push_back(std::async(std::launch::async, [this, sub, l0, l1]() {
        std::vector<std::future<void>> inner;
        build(l0, l1, *sub, 0, inner);
        for (auto& f : inner) f.get();
      }));
    } else {
      build(left_index, best_split, st, li, tasks);
    }
    build(best_split, right_index, st, li + 1, tasks);
  }
};

// Renumber a forest of local subtrees into the reference's global DFS numbering
// (build_recursive: visit node, append its 2 children, recurse left then right).
void splice(const SubTree& st, int local, uint32_t global, std::vector<BVH::Node>& out) {
  // iterative DFS mirroring the recursion order
  struct Item { const SubTree* t; int local; uint32_t global; };
  std::vector<Item> stack;
  stack.push_back({&st, local, global});
  while (!stack.empty()) {
    Item it = stack.back();
    stack.pop_back();
    const SubTree* t = it.t;
    int loc = it.local;
    // redirect to a deferred subtree root if this local node was handed to a task
    for (const auto& d : t->deferred)
      if (d.first == loc) { t = d.second.get(); loc = 0; break; }
    const BVH::Node& n = t->nodes[loc];
    BVH::Node g = n;
    if (!n.leaf) {
      const uint32_t li = (uint32_t)out.size();
      BVH::Node lc = t->nodes[n.index], rc = t->nodes[n.index + 1];
      out.push_back(lc);
      out.push_back(rc);
      g.index = li;
      // recursion order: left subtree fully before right -> push right first
      stack.push_back({t, (int)n.index + 1, li + 1});
      stack.push_back({t, (int)n.index, li});
    }
    out[it.global] = g;
  }
}

}  // namespace

void BVH::Build(std::vector<Object*>& objs) {  // bvh.cpp:27-44
  auto t0 = std::chrono::steady_clock::now();
  const size_t n = objs.size();
  objects.assign(objs.begin(), objs.end());
  boxes_.resize(n);
  cents_.resize(n);
  order_.resize(n);
  AABB world(Vector(FLT_MAX, FLT_MAX, FLT_MAX), Vector(-FLT_MAX, -FLT_MAX, -FLT_MAX));
  for (size_t i = 0; i < n; i++) {
    boxes_[i] = objs[i]->GetBoundingBox();
    cents_[i] = boxes_[i].centroid();
    world.extend(boxes_[i]);
    order_[i] = (int)i;
  }
  world.min.x = (float)((double)world.min.x - kEps); world.min.y = (float)((double)world.min.y - kEps);
  world.min.z = (float)((double)world.min.z - kEps);
  world.max.x = (float)((double)world.max.x + kEps); world.max.y = (float)((double)world.max.y + kEps);
  world.max.z = (float)((double)world.max.z + kEps);
  SubTree root;
  Node r;
  r.bbox = world;
  root.nodes.push_back(r);
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  Builder b{boxes_, cents_, order_, (int)std::max<size_t>(20000, n / (4 * hw) + 1)};
  std::vector<std::future<void>> tasks;
  b.build(0, (int)n, root, 0, tasks);
  for (auto& f : tasks) f.get();
  nodes.clear();
  nodes.reserve(2 * n + 1);
  nodes.push_back(Node());
  splice(root, 0, 0, nodes);
  std::vector<Object*> perm(n);
  for (size_t i = 0; i < n; i++) perm[i] = objs[(size_t)order_[i]];
  objects.swap(perm);
  build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int BVH::upload(drt_ctx* ctx) const {
  std::vector<drt_bvh_node> nd(nodes.size());
  for (size_t i = 0; i < nodes.size(); i++) {
    const Node& s = nodes[i];
    nd[i].bmin[0] = s.bbox.min.x; nd[i].bmin[1] = s.bbox.min.y; nd[i].bmin[2] = s.bbox.min.z;
    nd[i].bmax[0] = s.bbox.max.x; nd[i].bmax[1] = s.bbox.max.y; nd[i].bmax[2] = s.bbox.max.z;
    nd[i].leaf = s.leaf ? 1u : 0u;
    nd[i].index = s.index;
    nd[i].n_objs = s.leaf ? s.n_objs : 0u;
  }
  std::vector<uint32_t> ord(objects.size());
  for (size_t i = 0; i < objects.size(); i++) ord[i] = (uint32_t)objects[i]->scene_index;
  return drt_upload_bvh(ctx, nd.data(), (uint32_t)nd.size(), ord.data(), (uint32_t)ord.size());
}

static inline double dclamp(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

void Grid::Build(std::vector<Object*>& objs) {  // grid.cpp:30-97
  auto t0 = std::chrono::steady_clock::now();
  AABB gb(Vector(FLT_MAX, FLT_MAX, FLT_MAX), Vector(-FLT_MAX, -FLT_MAX, -FLT_MAX));
  std::vector<AABB> bx(objs.size());
  const size_t base = objects.size();  // positions of these objects in the grid's list
  for (size_t i = 0; i < objs.size(); i++) {
    bx[i] = objs[i]->GetBoundingBox();
    gb.extend(bx[i]);
    addObject(objs[i]);
  }
  gb.min.x = (float)((double)gb.min.x - kEps); gb.min.y = (float)((double)gb.min.y - kEps);
  gb.min.z = (float)((double)gb.min.z - kEps);
  gb.max.x = (float)((double)gb.max.x + kEps); gb.max.y = (float)((double)gb.max.y + kEps);
  gb.max.z = (float)((double)gb.max.z + kEps);
  bbox = gb;
  const double wx = bbox.max.x - bbox.min.x, wy = bbox.max.y - bbox.min.y, wz = bbox.max.z - bbox.min.z;
  const double s = std::pow((int)objs.size() / (wx * wy * wz), 0.3333333);
  nx = (int)(m * wx * s + 1);
  ny = (int)(m * wy * s + 1);
  nz = (int)(m * wz * s + 1);
  const int64_t cells = (int64_t)nx * ny * nz;
  // two passes (count, fill) over the same cell ranges -> CSR in insertion order
  auto range = [&](const AABB& ob, int r[6]) {
    r[0] = (int)dclamp((ob.min.x - bbox.min.x) * nx / (bbox.max.x - bbox.min.x), 0, nx - 1);
    r[1] = (int)dclamp((ob.min.y - bbox.min.y) * ny / (bbox.max.y - bbox.min.y), 0, ny - 1);
    r[2] = (int)dclamp((ob.min.z - bbox.min.z) * nz / (bbox.max.z - bbox.min.z), 0, nz - 1);
    r[3] = (int)dclamp((ob.max.x - bbox.min.x) * nx / (bbox.max.x - bbox.min.x), 0, nx - 1);
    r[4] = (int)dclamp((ob.max.y - bbox.min.y) * ny / (bbox.max.y - bbox.min.y), 0, ny - 1);
    r[5] = (int)dclamp((ob.max.z - bbox.min.z) * nz / (bbox.max.z - bbox.min.z), 0, nz - 1);
  };
  cell_start.assign((size_t)cells + 1, 0);
  for (size_t i = 0; i < objs.size(); i++) {
    int r[6];
    range(bx[i], r);
    for (int iz = r[2]; iz <= r[5]; iz++)
      for (int iy = r[1]; iy <= r[4]; iy++)
        for (int ix = r[0]; ix <= r[3]; ix++) cell_start[(size_t)(ix + nx * iy + nx * ny * iz) + 1]++;
  }
  for (int64_t c = 0; c < cells; c++) cell_start[c + 1] += cell_start[c];
  cell_objs.assign((size_t)cell_start[cells], 0);
  std::vector<int64_t> fill(cell_start.begin(), cell_start.end() - 1);
  for (size_t i = 0; i < objs.size(); i++) {
    int r[6];
    range(bx[i], r);
    for (int iz = r[2]; iz <= r[5]; iz++)
      for (int iy = r[1]; iy <= r[4]; iy++)
        for (int ix = r[0]; ix <= r[3]; ix++) cell_objs[(size_t)fill[(size_t)(ix + nx * iy + nx * ny * iz)]++] = (int32_t)(base + i);
  }
  build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int Grid::upload(drt_ctx* ctx) const {
  const int32_t dims[3] = {nx, ny, nz};
  const float mn[3] = {bbox.min.x, bbox.min.y, bbox.min.z}, mx[3] = {bbox.max.x, bbox.max.y, bbox.max.z};
  // the device indexes scene-order primitive records: list positions -> scene indices
  std::vector<int32_t> scene_ids(cell_objs.size());
  for (size_t i = 0; i < cell_objs.size(); i++) scene_ids[i] = objects[(size_t)cell_objs[i]]->scene_index;
  return drt_upload_grid(ctx, dims, mn, mx, cell_start.data(), scene_ids.data(), (int64_t)scene_ids.size());
}

int upload_scene(drt_ctx* ctx, const Scene& scene, const BVH* bvh, const Grid* grid) {
  drt_scene_desc d;
  std::vector<drt_prim> prims;
  std::vector<drt_light> ls;
  std::vector<drt_material> ms;
  scene.describe(d, prims, ls, ms);
  int rc = drt_upload_scene(ctx, &d);
  if (rc) return rc;
  if (d.accel == DRT_ACCEL_BVH) return bvh ? bvh->upload(ctx) : DRT_E_STATE;
  if (d.accel == DRT_ACCEL_GRID) return grid ? grid->upload(ctx) : DRT_E_STATE;
  return DRT_OK;
}

int render_scene(drt_ctx* ctx, const drt_frame_params& p, float* colors) { return drt_render(ctx, &p, colors); }

int set_camera(drt_ctx* ctx, const Camera& camera) {
  const drt_camera k = camera.frame();
  return drt_set_camera(ctx, &k);
}

int set_camera(drt_group* g, const Camera& camera) {
  const drt_camera k = camera.frame();
  return drt_group_set_camera(g, &k);
}

int upload_scene(drt_group* g, const Scene& scene, const BVH* bvh, const Grid* grid) {
  const int n = drt_group_size(g);
  if (n <= 0) return DRT_E_INVALID;
  for (int r = 0; r < n; r++) {
    const int rc = upload_scene(drt_group_ctx(g, r), scene, bvh, grid);
    if (rc) return rc;
  }
  return DRT_OK;
}

int render_scene(drt_group* g, const drt_frame_params& p, float* colors) { return drt_group_render(g, &p, colors); }

}  // namespace drt
