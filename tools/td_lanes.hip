// td_lanes.hip — what a per-lane gather instruction costs the per-CU vector-memory path as a
// function of its active lanes and its width.
//
// The PMC records (profiles/pmc_traffic.json) put TD_TD_BUSY at 30-33 cycles per vector-memory
// read instruction per CU in every path-kernel configuration, with the kernel's cycles equal to
// (instructions x that) / CUs.  Whether that cost scales with the instruction's active lanes
// (then compaction buys nothing on the memory path) or is paid per instruction (then a half-empty
// wave pays for its idle lanes) decides the next lever.  This program runs dependent random
// gathers from an L1-resident table (16 KiB) with `lanes` of each wave's 64 lanes active and
// per-lane loads of 4, 8 or 16 B, at 6 waves/SIMD, and prints the cycles per load instruction
// per CU (the clock from the device's wall-clock counter rate is not used: cycles are derived from
// a 2.4 GHz nominal clock and reported beside the time).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/td_lanes tools/td_lanes.hip && tools/bin/td_lanes
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
constexpr int kWaves = 6;
constexpr size_t kLdsPad = 160 * 1024 / kWaves - 1024;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// WIDTH 4 / 8 / 16 B per lane; PER 1..4 loads per step (one record of PER x WIDTH bytes);
// lanes < `lanes` of each wave run the chain, the others idle at the loop's branch.
template <int WIDTH, int PER>
__global__ void __launch_bounds__(kBlock, kWaves) gather(const uint4* __restrict__ table, uint32_t mask,
                                                          uint32_t iters, uint32_t lanes, uint32_t spread,
                                                          float* __restrict__ out) {
  const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t acc = 0;
  if (lane < lanes) {
    uint32_t idx = mix(tid * 0x9E3779B9u) & mask, prev = 0;
    for (uint32_t it = 0; it < iters; it++) {
      // records of 64 B; spread 0: all lanes of a wave read the same record (one line)
      const uint32_t rec = spread ? idx : ((mix(blockIdx.x * 977u + (threadIdx.x >> 6) + it * 131u) ^ prev) & mask);
      const char* base = (const char*)(table + 4 * (size_t)rec);
      uint32_t v = 0;
#pragma unroll
      for (int p = 0; p < PER; p++) {
        if (WIDTH == 16) {
          const uint4 q = *(const uint4*)(base + 16 * p);
          v ^= q.x ^ q.y ^ q.z ^ q.w;
        } else if (WIDTH == 8) {
          const uint2 q = *(const uint2*)(base + 16 * p);
          v ^= q.x ^ q.y;
        } else {
          v ^= *(const uint32_t*)(base + 16 * p);
        }
      }
      acc += v;
      prev = v;
      // table words are 0: the next index waits for the load but is a fresh draw
      idx = (mix((tid * 0x9E3779B9u) ^ mix(it + 1u)) ^ v) & mask;
    }
  }
  out[tid] = (float)acc;
}

template <int WIDTH, int PER>
static void run(const uint4* d_table, uint32_t n_rec, int blocks, float* d_out, uint32_t lanes, uint32_t spread) {
  const uint32_t iters = 2000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  gather<WIDTH, PER><<<blocks, kBlock, kLdsPad>>>(d_table, n_rec - 1, 8, lanes, spread, d_out);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(a));
  gather<WIDTH, PER><<<blocks, kBlock, kLdsPad>>>(d_table, n_rec - 1, iters, lanes, spread, d_out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double cus = prop.multiProcessorCount;
  const double waves = (double)blocks * kBlock / 64.0;
  const double instr = waves * iters * PER;  // load instructions (one per wave per load)
  const double lane_loads = instr * lanes;
  const double cyc_per_instr_cu = (ms * 1e-3 * 2.4e9) * cus / instr;
  printf("{\"width_B\": %d, \"loads_per_step\": %d, \"active_lanes\": %u, \"spread\": %u, \"ms\": %.3f, "
         "\"instr_per_s\": %.4e, \"lane_loads_per_s\": %.4e, \"GB_per_s\": %.1f, \"cycles_per_instr_per_cu\": %.2f}\n",
         WIDTH, PER, lanes, spread, ms, instr / (ms * 1e-3), lane_loads / (ms * 1e-3),
         lane_loads * WIDTH / (ms * 1e-3) / 1e9, cyc_per_instr_cu);
  fflush(stdout);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gather<16, 4>, kBlock, kLdsPad));
  const int blocks = prop.multiProcessorCount * per_cu;
  const uint32_t n_rec = 256;  // 16 KiB: L1-resident
  std::vector<uint32_t> h(16 * (size_t)n_rec, 0u);
  uint4* d_table = nullptr;
  float* d_out = nullptr;
  CHECK(hipMalloc(&d_table, h.size() * 4));
  CHECK(hipMemcpy(d_table, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&d_out, (size_t)blocks * kBlock * sizeof(float)));
  const uint32_t lane_set[] = {64, 48, 32, 16, 8, 1};
  for (uint32_t lanes : lane_set) run<16, 4>(d_table, n_rec, blocks, d_out, lanes, 1);
  for (uint32_t lanes : lane_set) run<8, 4>(d_table, n_rec, blocks, d_out, lanes, 1);
  for (uint32_t lanes : lane_set) run<4, 4>(d_table, n_rec, blocks, d_out, lanes, 1);
  run<16, 4>(d_table, n_rec, blocks, d_out, 64, 0);
  run<16, 4>(d_table, n_rec, blocks, d_out, 16, 0);
  run<16, 3>(d_table, n_rec, blocks, d_out, 64, 1);
  run<16, 1>(d_table, n_rec, blocks, d_out, 64, 1);
  CHECK(hipFree(d_table));
  CHECK(hipFree(d_out));
  return 0;
}
