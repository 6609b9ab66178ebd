// gather_ceiling.hip — the vector-memory ceiling for the BVH kernel's access shape on one MI355X.
//
// The persistent path kernel's node step is a per-lane gather: every traversing lane loads one
// 64-B record (4 x 16-B slots, global_load_dwordx4) whose address depends on the previous
// record, with one record in flight per lane, at 6 waves per SIMD.  This program
// runs exactly that shape with nothing else — a dependent chain of random 64-B records per lane —
// over tables of several sizes (L1-, L2-, Infinity-Cache- and HBM-resident), and reports the
// record bytes served per second.  The fastest table is the ceiling the path kernel cannot
// exceed however much locality its rays have; bench.py's roofline.frac divides the kernel's
// algorithmic record bytes per second by it (roofline.bound "vmem_gather").
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/gather_ceiling tools/gather_ceiling.hip
//   tools/bin/gather_ceiling [chains]      -> one JSON line per table size
//   (chains 0: the quad-cooperative fetch, gather_coop)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int kBlock = 256;
constexpr int kWaves = 6;  // waves per SIMD, the path kernel's occupancy

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float sum16(const float4& a, const float4& b, const float4& d, const float4& e) {
  return ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w)) + ((d.x + d.y) + (d.z + d.w)) +
         ((e.x + e.y) + (e.z + e.w));
}

// CHAINS independent dependent chains per lane (1 = the node step: one record in flight).
template <int CHAINS>
__global__ void __launch_bounds__(kBlock, kWaves) gather(const float4* __restrict__ table, uint32_t mask,
                                                          uint32_t iters, float* __restrict__ out) {
  const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
  uint32_t idx[CHAINS];
  for (int c = 0; c < CHAINS; c++) idx[c] = mix(tid * 0x9E3779B9u + c) & mask;
  float acc = 0.0f;
  for (uint32_t it = 0; it < iters; it++) {
    for (int c = 0; c < CHAINS; c++) {
      const float4* r = table + 4 * (size_t)idx[c];
      const float4 a = r[0], b = r[1], d = r[2], e = r[3];
      acc += sum16(a, b, d, e);  // every dword is consumed, as a node test consumes its record
      // the next record depends on this one (a BVH child descriptor does the same): slot 3's w is
      // 0 in every record (set on the host, unknown to the compiler), so the address is a fresh
      // uniform draw per (lane, step) that still waits for this load.  (Round 1-2's walk fed the
      // record's data back into the hash: a random function of the index, whose chains merge onto
      // cycles of ~sqrt(records) — after a few thousand steps the 128 MiB and 1 GiB tables were
      // read from a few thousand L2-resident records.)
      idx[c] = (mix((tid * 0x9E3779B9u) ^ mix(it * 2u + (uint32_t)c + 1u)) ^ __float_as_uint(e.w)) & mask;
    }
  }
  out[tid] = acc;
}

// The same dependent chains, fetched cooperatively by the 4 lanes of a quad: in round r the quad
// loads the 64-B record of its lane r, lane l taking 16-B slot l, so one load instruction touches
// one 64-B segment per quad instead of one line per lane; then a 4x4 transpose of float4s inside
// the quad (two DPP butterfly stages, quad_perm [1,0,3,2] and [2,3,0,1]) gives each lane its own
// record's four slots.  Same records, same dependent chain per lane, 4 load instructions per
// record as above — only the lane -> address assignment differs.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float4 dpp4(const float4& v) {
  return make_float4(dpp_f<CTRL>(v.x), dpp_f<CTRL>(v.y), dpp_f<CTRL>(v.z), dpp_f<CTRL>(v.w));
}
__device__ __forceinline__ float4 sel4(bool c, const float4& a, const float4& b) {
  return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}
constexpr int kQuadSwap1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kQuadSwap2 = 0x4E;  // quad_perm [2,3,0,1]

// X[r] = slot (lane & 3) of lane r's record  ->  Y[j] = slot j of this lane's record
__device__ __forceinline__ void quad_transpose(float4 X[4], float4 Y[4]) {
  const uint32_t l = threadIdx.x & 3u;
  const bool b0 = (l & 1u) != 0u, b1 = (l & 2u) != 0u;
  const float4 rA = dpp4<kQuadSwap1>(sel4(b0, X[0], X[1]));
  const float4 rB = dpp4<kQuadSwap1>(sel4(b0, X[2], X[3]));
  const float4 T0 = sel4(b0, rA, X[0]), T1 = sel4(b0, X[1], rA);
  const float4 T2 = sel4(b0, rB, X[2]), T3 = sel4(b0, X[3], rB);
  const float4 rC = dpp4<kQuadSwap2>(sel4(b1, T0, T2));
  const float4 rD = dpp4<kQuadSwap2>(sel4(b1, T1, T3));
  Y[0] = sel4(b1, rC, T0);
  Y[1] = sel4(b1, rD, T1);
  Y[2] = sel4(b1, T2, rC);
  Y[3] = sel4(b1, T3, rD);
}

__global__ void __launch_bounds__(kBlock, kWaves) gather_coop(const float4* __restrict__ table, uint32_t mask,
                                                               uint32_t iters, float* __restrict__ out) {
  const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t l = threadIdx.x & 3u;
  uint32_t idx = mix(tid * 0x9E3779B9u) & mask;
  float acc = 0.0f;
  for (uint32_t it = 0; it < iters; it++) {
    float4 X[4], Y[4];
    const uint32_t o0 = dpp_u<0x00>(idx), o1 = dpp_u<0x55>(idx), o2 = dpp_u<0xAA>(idx), o3 = dpp_u<0xFF>(idx);
    X[0] = table[4 * (size_t)o0 + l];
    X[1] = table[4 * (size_t)o1 + l];
    X[2] = table[4 * (size_t)o2 + l];
    X[3] = table[4 * (size_t)o3 + l];
    quad_transpose(X, Y);
    const float4 a = Y[0], b = Y[1], d = Y[2], e = Y[3];
    acc += sum16(a, b, d, e);
    idx = (mix((tid * 0x9E3779B9u) ^ mix(it * 2u + 1u)) ^ __float_as_uint(e.w)) & mask;
  }
  out[tid] = acc;
}

// Dynamic LDS per block (unused) that caps the CU at kWaves blocks of 256 threads, i.e. kWaves
// waves per SIMD: the gather kernel's few registers would otherwise let 8 in.
constexpr size_t kLdsPad = 160 * 1024 / kWaves - 1024;

template <int CHAINS>
static double run(const float4* d_table, uint32_t n_rec, uint32_t iters, int blocks, float* d_out) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  // CHAINS 0: the quad-cooperative fetch (one chain per lane)
  auto launch = [&](uint32_t n_it) {
    if (CHAINS == 0) gather_coop<<<blocks, kBlock, kLdsPad>>>(d_table, n_rec - 1, n_it, d_out);
    else gather<CHAINS ? CHAINS : 1><<<blocks, kBlock, kLdsPad>>>(d_table, n_rec - 1, n_it, d_out);
  };
  launch(4);  // warm caches / code
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(a));
  launch(iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms;
}

int main(int argc, char** argv) {
  const int chains = argc > 1 ? atoi(argv[1]) : 1;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  int per_cu = 0;
  if (chains == 0)
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gather_coop, kBlock, kLdsPad));
  else if (chains == 1)
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gather<1>, kBlock, kLdsPad));
  else
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gather<2>, kBlock, kLdsPad));
  const int blocks = cus * per_cu;
  // table sizes in 64-B records (powers of two): 16 KiB (L1), 2 MiB (L2), 128 MiB (the 1M-triangle
  // scene is 124 MB: Infinity Cache), 1 GiB (HBM)
  const uint32_t sizes[] = {1u << 8, 1u << 15, 1u << 21, 1u << 24};
  const uint32_t max_rec = 1u << 24;
  std::vector<float> h(4 * 4 * (size_t)max_rec);
  uint32_t s = 12345u;
  for (size_t i = 0; i < h.size(); i++) {
    s = s * 1664525u + 1013904223u;
    h[i] = (i % 16 == 15) ? 0.0f : (float)(s >> 8) * (1.0f / 16777216.0f);  // slot 3 .w = 0 (the walk)
  }
  float4* d_table = nullptr;
  float* d_out = nullptr;
  CHECK(hipMalloc(&d_table, h.size() * sizeof(float)));
  CHECK(hipMemcpy(d_table, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&d_out, (size_t)blocks * kBlock * sizeof(float)));
  for (uint32_t n_rec : sizes) {
    const uint32_t iters = n_rec <= (1u << 15) ? 3000 : 2000;
    const double ms = chains == 0   ? run<0>(d_table, n_rec, iters, blocks, d_out)
                      : chains == 1 ? run<1>(d_table, n_rec, iters, blocks, d_out)
                                    : run<2>(d_table, n_rec, iters, blocks, d_out);
    const double recs = (double)blocks * kBlock * iters * (chains ? chains : 1);
    printf("{\"table_bytes\": %llu, \"chains\": %d, \"fetch\": \"%s\", \"blocks\": %d, \"waves_per_simd\": %d, "
           "\"ms\": %.3f, \"records_per_s\": %.4e, \"GB_per_s\": %.1f}\n",
           (unsigned long long)n_rec * 64ull, chains ? chains : 1, chains ? "lane" : "quad_coop", blocks,
           per_cu * kBlock / 64 / 4, ms, recs / (ms * 1e-3),
           recs * 64.0 / (ms * 1e-3) / 1e9);
    fflush(stdout);
  }
  CHECK(hipFree(d_table));
  CHECK(hipFree(d_out));
  return 0;
}
