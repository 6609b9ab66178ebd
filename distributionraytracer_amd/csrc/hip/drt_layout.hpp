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
//
// Shadow tree (round 4): BVH::Traverse(Ray&) (bvh.cpp:316-391) answers "is any primitive of a
// leaf whose box the ray hits within range" — an any-hit boolean whose value does not depend on
// the visit order.  Shadow queries of finite rays therefore walk a 4-ary tree collapsed from the
// reference's binary tree (same leaves), 64 B per node = the four 16-B slots the node step loads:
//   s0 = (p.x, p.y, p.z, bits: E.x | E.y << 8 | E.z << 16)   anchor and biased exponents
//   s1 = (lo.x, hi.x, lo.y, hi.y)   s2 = (lo.z, hi.z, 0, 0)   one byte per child per dword
//   s3 = (desc[0], desc[1], desc[2], desc[3])                 inner wide index or leaf descriptor
// Child k's box on axis a is [p.a + lo.a[k] * 2^(E.a-127), p.a + hi.a[k] * 2^(E.a-127)]: p.a is a
// multiple of the scale, so every decoded plane is an exact float (one FMA, no rounding) and the
// box contains the child's reference box.  An unused child slot has lo = 255, hi = 0: an inverted
// box that no ray hits.  A primitive hit within range is accepted only after the exact box of its
// reference leaf (wide leaf-box array, 32 B per primitive: (min.xyz, max.x), (max.yz, 0, 0)) is
// hit too, so the accepted set is exactly the reference's ("shadow tree").
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
// Children per shadow-tree node: 4 (64-B records), or 8 with -DDRT_WIDE8 (A/B, round 6): a 128-B record —
//   s0 = (p, ebits), s1 = lo.x[8], hi.x[8] (two words each), s2 = y, s3 = z, s4 / s5 = desc[0..3] / [4..7],
//   s6, s7 unused — one 128-B line per visit, six slot loads, half the tree levels.
#ifdef DRT_WIDE8
constexpr int kWideK = 8;
#else
constexpr int kWideK = 4;
#endif
constexpr int kWideW = kWideK / 4;  // words per plane (one byte per child)
struct WideNodeRecord4 {
  float p[3];
  uint32_t ebits;
  uint32_t q[6];  // lo.x, hi.x, lo.y, hi.y, lo.z, hi.z (byte k = child k)
  uint32_t pad[2];
  uint32_t desc[4];
};
struct WideNodeRecord8 {
  float p[3];
  uint32_t ebits;
  uint32_t q[12];  // per plane (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z) two words: byte k & 3 of word k >> 2
  uint32_t desc[8];
  uint32_t pad[8];
};
#ifdef DRT_WIDE8
#define WideNodeRecord WideNodeRecord8
#else
#define WideNodeRecord WideNodeRecord4
#endif
struct LeafBoxRecord {
  float box[6];
  uint32_t pad[2];
};
static_assert(sizeof(PrimRecord) == 48, "prim record is 48 B");
static_assert(sizeof(NodeRecord) == 64, "node record is 64 B");
static_assert(sizeof(WideNodeRecord4) == 64, "4-ary wide node record is 64 B");
static_assert(sizeof(WideNodeRecord8) == 128, "8-ary wide node record is 128 B");
static_assert(sizeof(LeafBoxRecord) == 32, "leaf box record is 32 B");

inline float bits_as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

}  // namespace drt
