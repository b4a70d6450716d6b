// Microbenchmarks for the roofline peaks bench.py divides by:
//   valu  -- int32 VALU lane-ops/s with the search kernel's fixpoint instruction pair
//            (v_and_b32 + v_bcnt_u32_b32, 16 independent chains per lane, inline asm so
//            the instruction count is exact), every CU busy
//   lds   -- ds_read_b32 bytes/s (conflict-free, lane-contiguous words: the DFS stack's
//            access pattern), every CU busy
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/peak_probe tools/peak_probe.hip
// Prints one JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr int CHAINS = 16;

// MODE 0: v_and_b32 + v_bcnt_u32_b32 pairs (the fixpoint's per-word op pair); 1: v_and_b32
// only; 2: v_bcnt_u32_b32 only; 3: v_add_u32 only
template <int MODE>
__global__ __launch_bounds__(256) void valu_kernel(uint32_t iters, uint32_t seed, uint32_t* out) {
  uint32_t x[CHAINS];
  const uint32_t m = seed * 2654435761u + threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = seed + c * 7919u + threadIdx.x;
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if constexpr (MODE == 0) {
        uint32_t t;
        asm volatile("v_and_b32 %0, %1, %2" : "=v"(t) : "v"(x[c]), "v"(m));
        asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(x[c]) : "v"(t), "v"(x[c]));
      } else if constexpr (MODE == 1) {
        asm volatile("v_and_b32 %0, %1, %2" : "=v"(x[c]) : "v"(x[c]), "v"(m));
        asm volatile("v_and_b32 %0, %1, %2" : "=v"(x[c]) : "v"(m), "v"(x[c]));
      } else if constexpr (MODE == 2) {
        asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(x[c]) : "v"(x[c]), "v"(m));
        asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(x[c]) : "v"(m), "v"(x[c]));
      } else {
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(x[c]) : "v"(x[c]), "v"(m));
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(x[c]) : "v"(m), "v"(x[c]));
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= x[c];
  if (s == 0x12345678u) out[blockIdx.x] = s;  // keeps the chains alive
}

__global__ __launch_bounds__(256) void lds_kernel(uint32_t iters, uint32_t* out) {
  __shared__ uint32_t buf[64 * 64];
  for (uint32_t i = threadIdx.x; i < 64 * 64; i += blockDim.x) buf[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      // word (level k) of this lane: [level][lane] layout, conflict-free ds_read_b32
      const uint32_t idx = ((uint32_t)((k + i + wave) & 63u) << 6) | lane;
      uint32_t v;
      asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(idx * 4u) : "memory");
      acc += v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&out, 1 << 20));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  // VALU: 8 blocks x 256 threads per CU = 32 waves per CU (8 per SIMD)
  const int vblocks = cus * 8;
  const uint32_t viters = 4096;
  auto time_valu = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(vblocks), dim3(256), 0, 0, 16u, 1u, out);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(a));
      hipLaunchKernelGGL(kern, dim3(vblocks), dim3(256), 0, 0, viters, (uint32_t)r + 1, out);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    return (double)vblocks * 256.0 * viters * CHAINS * 2.0 / (best * 1e-3) / 1e12;  // lane-ops/s
  };
  const double v_pair = time_valu(valu_kernel<0>), v_and = time_valu(valu_kernel<1>),
               v_bcnt = time_valu(valu_kernel<2>), v_add = time_valu(valu_kernel<3>);
  // LDS: 8 blocks x 256 threads per CU
  const int lblocks = cus * 8;
  const uint32_t liters = 8192;
  hipLaunchKernelGGL(lds_kernel, dim3(lblocks), dim3(256), 0, 0, 16u, out);
  CHECK(hipDeviceSynchronize());
  float best_l = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(lds_kernel, dim3(lblocks), dim3(256), 0, 0, liters, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best_l) best_l = ms;
  }
  const double lbytes = (double)lblocks * 256.0 * liters * 16.0 * 4.0;
  std::printf(
      "{\"cus\": %d, \"clock_mhz\": %d, \"valu_model_tops\": %.2f, \"valu_and_bcnt_pair_tops\": %.2f, "
      "\"valu_and_tops\": %.2f, \"valu_bcnt_tops\": %.2f, \"valu_add_tops\": %.2f, \"lds_read_b32_tbs\": %.2f}\n",
      cus, p.clockRate / 1000, cus * 4.0 * 32.0 * (p.clockRate * 1e3) / 1e12, v_pair, v_and, v_bcnt, v_add,
      lbytes / (best_l * 1e-3) / 1e12);
  return 0;
}
