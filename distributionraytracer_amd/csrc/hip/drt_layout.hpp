// drt_layout.hpp — HBM data layout shared by the host packer and the gfx950 kernels.
//
// Primitive record: 48 B = 3 x float4 (one 16-B load each, coalesced per lane):
//   q0 = (A.x, A.y, A.z, bits: type | material << 2)
//   q1 = (B.x, B.y, B.z, bits: original object index)
//   q2 = (C.x, C.y, C.z, 0)
//   triangle: A = P0, B = P1 - P0 (edge1), C = P2 - P0 (edge2)  — the exact float differences
//             Triangle::hit computes (scene.cpp:59-60), so pre-subtracting changes no bit
//   sphere:   A = centre, B.x = radius
//   plane:    A = PN,     B.x = D
//   box:      A = min,    B = max
// In BVH mode records are stored in the BVH's object order, so every leaf is one contiguous
// run of records; NONE / GRID modes keep scene order.
//
// BVH inner-node record: 64 B = 4 x float4 holding BOTH children's boxes (the reference's
// traversal always tests the two siblings together, bvh.cpp:252-253):
//   a = (L.min.x, L.min.y, L.min.z, L.max.x)
//   b = (L.max.y, L.max.z, R.min.x, R.min.y)
//   c = (R.min.z, R.max.x, R.max.y, R.max.z)
//   d = (L.desc, R.desc, 0, 0)
// A child descriptor (uint32) is either an inner record index (bit 31 clear) or a leaf
// (bit 31 set): bits 0..25 = first primitive, bits 26..30 = object count (< 31); count 31
// marks an oversized leaf whose (first, count) pair lives in the big-leaf table at bits 0..25.
#pragma once
#include <stdint.h>
#include <string.h>

namespace drt {

enum : uint32_t { PRIM_TRIANGLE = 0, PRIM_SPHERE = 1, PRIM_PLANE = 2, PRIM_BOX = 3 };

constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kFirstMask = (1u << 26) - 1u;
constexpr uint32_t kCountShift = 26;
constexpr uint32_t kBigLeaf = 31u;

__host__ __device__ inline uint32_t leaf_desc(uint32_t first, uint32_t count) {
  return kLeafBit | (count << kCountShift) | (first & kFirstMask);
}
__host__ __device__ inline bool desc_is_leaf(uint32_t d) { return (d & kLeafBit) != 0u; }
__host__ __device__ inline uint32_t desc_first(uint32_t d) { return d & kFirstMask; }
__host__ __device__ inline uint32_t desc_count(uint32_t d) { return (d >> kCountShift) & 31u; }

#if defined(__HIPCC__)
__host__ __device__ inline uint32_t f2u(float f) { return __float_as_uint(f); }
__device__ inline uint32_t prim_type(const float4& q0) { return __float_as_uint(q0.w) & 3u; }
__device__ inline uint32_t prim_material(const float4& q0) { return __float_as_uint(q0.w) >> 2; }
__device__ inline uint32_t prim_object(const float4& q1) { return __float_as_uint(q1.w); }
#endif

// Host-side packing helpers (plain structs; no HIP types).
struct PrimRecord {
  float q[12];
};
struct NodeRecord {
  float box[12];
  uint32_t desc[4];
};
static_assert(sizeof(PrimRecord) == 48, "prim record is 48 B");
static_assert(sizeof(NodeRecord) == 64, "node record is 64 B");

inline float bits_as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

}  // namespace drt
