// Diagnostics: what do returned atomics of many waves on ONE address (or one 128-byte line)
// cost on this GPU?  2304 single-wave blocks, lane 0 of each does `reps` dependent
// atomicAdd-with-return; variants: one address / 4 words of one line / one line per block % 64
// / plain agent-scope loads of one address.
//   hipcc --offload-arch=gfx950 -O3 -o gpurun_out/atomic_probe tools/atomic_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ void probe(unsigned* ctr, unsigned* sink, int mode, int reps) {
  if (threadIdx.x != 0) return;
  unsigned acc = 0;
  for (int i = 0; i < reps; ++i) {
    unsigned* p;
    if (mode == 0) p = ctr;                                           // one address
    else if (mode == 1) p = ctr + ((i + acc) & 3);                    // 4 words of one line
    else if (mode == 2) p = ctr + (size_t)(blockIdx.x & 63) * 32;     // 64 lines
    else p = ctr + (size_t)blockIdx.x * 32;                           // a line per wave
    if (mode == 4) acc += __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    else if (mode == 5) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // no return
    else acc += atomicAdd(p, 1u);
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

int main() {
  unsigned *ctr, *sink;
  CHECK(hipMalloc(&ctr, 2304 * 128 + 4096));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(ctr, 0, 2304 * 128 + 4096));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"one address, returned", "4 words of one line, returned", "64 lines (block % 64), returned",
                         "one line per wave, returned", "agent-scope load of one address", "one address, no return"};
  for (int blocks : {2304, 256})
    for (int mode = 0; mode < 6; ++mode)
      for (int reps : {1, 4, 16}) {
        float best = 1e9f;
        for (int it = 0; it < 5; ++it) {
          CHECK(hipEventRecord(e0, 0));
          hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, ctr, sink, mode, reps);
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          float ms;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          if (ms < best) best = ms;
        }
        std::printf("{\"blocks\": %d, \"mode\": \"%s\", \"reps\": %d, \"us\": %.1f, \"ns_per_access\": %.2f}\n", blocks, names[mode],
                    reps, best * 1e3, best * 1e6 / ((double)blocks * reps));
      }
  return 0;
}
