// =====================================================================================
//  MI355X (gfx950 / CDNA4) device code for the quorum-intersection hot path.
//
//  search_kernel   iterateMinimalQuorums + checkMinimalQuorums (cpp:252-400) as a
//                  budgeted frontier loop: ONE LANE PER SEARCH NODE.  Each lane walks a
//                  subtree ("unit") depth-first, exclusion branch first, with its pending
//                  inclusion branches on an LDS stack ([level][word][lane], conflict-free
//                  ds_read_b32/ds_write_b32).  The greatest fixpoint (containsQuorum,
//                  cpp:140-177) is a Jacobi iteration over a lane's 32-bit-word masks: the
//                  threshold-node (TN) table is wave-uniform, so its masks arrive by scalar
//                  loads and each TN costs v_and_b32 + v_bcnt_u32_b32 per word.
//                  Quorum leaves (cpp:281-291) are resolved wave-cooperatively: the |D|
//                  single-removal fixpoints of isMinimalQuorum (cpp:179-201) and the
//                  complement check of the visitor (cpp:357-384) of every pending lane are
//                  spread over the 64 lanes (wave prefix sums), so a rare leaf does not
//                  serialise the wave.
//  gfp_batch_kernel containsQuorum over the global TN CSR for arbitrary (nodes, avail)
//                  queries, ONE WAVEFRONT PER CANDIDATE SET: lanes evaluate TNs level by
//                  level into LDS, vertex membership is rebuilt with wave64 __ballot.
//  reduce_kernel   preorder-filtered sums of the per-segment log (exact node counts
//                  under early exit).
// =====================================================================================
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <mutex>
#include <cstdio>
#include <chrono>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "qi_device.h"
#include "qi_jit.h"
#include "../../include/quorum_intersection.h"

// The Makefile compiles this file in parts (-DQI_PART=0..6) so the kernel instantiations
// build in parallel and load separately (a part is a code object, loaded at its first
// launch): part 0 holds everything except the search engines, parts 1-5 one group of
// SearchDeviceImpl instantiations each (make_engine below), part 6 the frontier sort.
// Without QI_PART the file is one translation unit.
#ifndef QI_PART
#define QI_PART -1
#endif

namespace qi {

#define HIP_CHECK(x)                                                                        \
  do {                                                                                      \
    hipError_t e__ = (x);                                                                   \
    if (e__ != hipSuccess)                                                                  \
      throw Error(QI_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e__));          \
  } while (0)

}  // namespace qi

#include "qi_search_kernel.h"
#include "qi_ordered_kernel.h"

namespace qi {
namespace dev {

// Ahead-of-time kernels: one per (vertex words, TN words, stack depth) shape.
// (TIE: findBestNode's tie rule, see search_body)
template <int MW, int TW, int SMAX, bool TIE>
__global__ __launch_bounds__(64) void search_kernel(SearchArgs a) {
  search_body<MW, TW, SMAX, TableEval<MW, TW>, TIE>(a);
}

// Order-exact search for SCCs with threshold-0 quorum sets (qi_ordered_kernel.h).
template <int MW, int TW>
__global__ __launch_bounds__(64) void ordered_kernel(OrdArgs oa) {
  ordered_body<MW, TW>(oa);
}

// ------------------------------------------------------------------------------------
// Batched containsQuorum over the global TN CSR: one wavefront per query.
// ------------------------------------------------------------------------------------
struct GlobalDev {
  uint32_t n, words, T, levels;
  uint32_t nonmonotone;  // any threshold-0 TN: exact ascending Gauss-Seidel
  const uint32_t* level_off;
  const uint32_t* kind;
  const uint32_t* thr;
  const uint32_t* first;
  const uint32_t* vref_off;
  const uint32_t* vref;
  const uint32_t* cref_off;
  const uint32_t* cref;
  const uint32_t* root;
};

// GS = true: the per-query state lives in global memory (`scratch`, `per` bytes per
// query) instead of LDS, for networks whose image exceeds the LDS (a one-wave workgroup
// sees its own global stores in order; __syncthreads() orders them like LDS ones).
template <bool GS>
__global__ __launch_bounds__(64) void gfp_batch_kernel(GlobalDev g, const unsigned long long* nodes,
                                                        const unsigned long long* avail, uint32_t count,
                                                        unsigned long long* out, unsigned long long* rounds_out,
                                                        uint8_t* scratch, size_t per) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  const uint32_t q = blockIdx.x;
  if (q >= count) return;
  unsigned long long* A = GS ? (unsigned long long*)(scratch + (size_t)q * per) : sm;  // [words] available set
  unsigned long long* X = A + g.words;    // [words] current candidates
  uint8_t* sat = (uint8_t*)(X + g.words); // [T]
  const uint32_t lane = threadIdx.x;
  const unsigned long long* qn = nodes + (size_t)q * g.words;
  const unsigned long long* qa = avail + (size_t)q * g.words;
  for (uint32_t w = lane; w < g.words; w += WAVE) {
    const unsigned long long av = qa[w];
    A[w] = av;
    X[w] = qn[w] & av;  // a listed but unavailable vertex fails "no self" (cpp:95)
  }
  __syncthreads();
  uint32_t rounds = 0;
  auto eval_tns = [&]() {
    for (uint32_t l = 0; l < g.levels; ++l) {
      for (uint32_t t = g.level_off[l] + lane; t < g.level_off[l + 1]; t += WAVE) {
        const uint32_t k = g.kind[t];
        bool s = false;
        if (k == TN_FIRST_UNAVAIL) {
          const uint32_t fst = g.first[t];
          const uint32_t idx = fst & 0x7FFFFFFFu;
          const bool avail_first = (fst >> 31) ? (sat[idx] != 0) : ((A[idx >> 6] >> (idx & 63)) & 1ull);
          s = !avail_first;
        } else if (k == TN_NORMAL) {
          uint32_t c = 0;
          for (uint32_t e = g.vref_off[t]; e < g.vref_off[t + 1]; ++e) {
            const uint32_t v = g.vref[e];
            c += (uint32_t)((A[v >> 6] >> (v & 63)) & 1ull);
          }
          for (uint32_t e = g.cref_off[t]; e < g.cref_off[t + 1]; ++e) c += sat[g.cref[e]];
          s = c >= g.thr[t];
        }
        sat[t] = s ? 1 : 0;
      }
      __syncthreads();
    }
  };
  if (g.nonmonotone) {
    // Threshold-0 quorum sets make the slice predicate anti-monotone ("first entry
    // unavailable"), so the fixpoint depends on the sweep order: reproduce the
    // reference's Gauss-Seidel sweep (cpp:148-169) in ascending vertex order exactly.
    // Each step removes the first failing vertex at or after the sweep cursor.
    for (;;) {
      ++rounds;
      bool removed_any = false;
      uint32_t cursor = 0;
      for (;;) {
        eval_tns();
        uint32_t hit = 0xFFFFFFFFu;
        for (uint32_t w = cursor >> 6; w < g.words && hit == 0xFFFFFFFFu; ++w) {
          const uint32_t v = w * 64u + lane;
          const bool fails = v < g.n && v >= cursor && ((X[w] >> lane) & 1ull) && !sat[g.root[v]];
          const unsigned long long b = __ballot(fails);
          if (b) hit = w * 64u + (uint32_t)__builtin_ctzll(b);
        }
        if (hit == 0xFFFFFFFFu) break;
        __syncthreads();
        if (lane == 0) {
          X[hit >> 6] &= ~(1ull << (hit & 63));
          A[hit >> 6] &= ~(1ull << (hit & 63));
        }
        __syncthreads();
        removed_any = true;
        cursor = hit + 1;
        if (cursor >= g.n) break;
      }
      if (!removed_any) break;
    }
    for (uint32_t w = lane; w < g.words; w += WAVE) out[(size_t)q * g.words + w] = X[w];
    if (lane == 0) atomicAdd(rounds_out, (unsigned long long)rounds);
    return;
  }
  for (;;) {
    ++rounds;
    eval_tns();
    bool changed = false;
    for (uint32_t w = 0; w < g.words; ++w) {
      const uint32_t v = w * 64u + lane;
      bool keep = false;
      if (v < g.n) keep = ((X[w] >> lane) & 1ull) && sat[g.root[v]];
      const unsigned long long nw = __ballot(keep);
      const unsigned long long old = X[w];
      changed |= (nw != old);
      __syncthreads();
      if (lane == 0) {
        A[w] &= ~(old & ~nw);  // removed vertices become unavailable (cpp:158-161)
        X[w] = nw;
      }
      __syncthreads();
    }
    if (!changed) break;
  }
  for (uint32_t w = lane; w < g.words; w += WAVE) out[(size_t)q * g.words + w] = X[w];
  if (lane == 0) atomicAdd(rounds_out, (unsigned long long)rounds);
}

}  // namespace dev

#if QI_PART <= 0
// ------------------------------------------------------------------------------------
// Device scratch of the no-allocation entry point (GfpDevice::run_static): one fixed array
// per GPU, held from the first use of the library on that GPU until the process ends.
//   [0, 256)   counters (fixpoint rounds of the last call), cleared by every call
//   [256, ...) per-query state images (available set, candidates, TN satisfaction bytes)
// In host code the array's name is only a handle: the device address is taken once per
// device with hipGetSymbolAddress (static_scratch_ptr) and only that pointer is passed on.
// ------------------------------------------------------------------------------------
namespace dev {
// Clears `n` 64-bit words (a kernel rather than hipMemsetAsync: callers may be capturing
// the stream into a HIP graph).
static __global__ void zero_u64_kernel(unsigned long long* p, uint32_t n) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0ull;
}
}  // namespace dev
constexpr size_t kStaticScratchBytes = QI_STATIC_SCRATCH_BYTES;
constexpr size_t kStaticScratchHeader = 256;
static __device__ __align__(256) unsigned char scratch[kStaticScratchBytes];

namespace {
std::mutex g_scratch_mu;
unsigned char* g_scratch_ptr[64] = {};  // per HIP device: address of that device's copy

// Call with `device` current.  Resolves the array's address on this device (first call per
// device; a set-up step, done when the device image of an FBAS is created).
unsigned char* static_scratch_ptr(int device) {
  if (device < 0 || device >= 64) throw Error(QI_ERR_ARG, "static scratch: device ordinal out of range");
  std::lock_guard<std::mutex> g(g_scratch_mu);
  if (!g_scratch_ptr[device]) {
    unsigned char* p = nullptr;
    HIP_CHECK(hipGetSymbolAddress((void**)&p, HIP_SYMBOL(scratch)));
    if (!p) throw Error(QI_ERR_DEVICE, "static scratch: hipGetSymbolAddress returned null");
    g_scratch_ptr[device] = p;
  }
  return g_scratch_ptr[device];
}
}  // namespace

#endif  // QI_PART <= 0

// =====================================================================================
// Host-side device management
// =====================================================================================
#if QI_PART <= 0
int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int device_cu_count(int device) {
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, device));
  return p.multiProcessorCount;
}

void* device_alloc(int device, size_t bytes) {
  int prev = 0;
  HIP_CHECK(hipGetDevice(&prev));
  HIP_CHECK(hipSetDevice(device));
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) throw Error(QI_ERR_CAPACITY, std::string("hipMalloc: ") + hipGetErrorString(e));
  return p;
}

void device_free(int device, void* p) {
  if (!p) return;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return;
  (void)hipSetDevice(device);
  (void)hipFree(p);
  (void)hipSetDevice(prev);
}

void device_copy(void* dst, int dst_device, const void* src, int src_device, size_t bytes) {
  if (!bytes) return;
  int prev = 0;
  HIP_CHECK(hipGetDevice(&prev));
  HIP_CHECK(hipSetDevice(src_device));
  if (dst_device == src_device) HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice));
  else HIP_CHECK(hipMemcpyPeer(dst, dst_device, src, src_device, bytes));  // xGMI
  HIP_CHECK(hipSetDevice(prev));
}

uint64_t* pinned_word_alloc() {
  void* p = nullptr;
  HIP_CHECK(hipHostMalloc(&p, 64, hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
  *(uint64_t*)p = ~0ull;
  return (uint64_t*)p;
}

void pinned_word_free(uint64_t* p) {
  if (p) (void)hipHostFree((void*)p);
}

bool enable_peer(int a, int b) {
  if (a == b) return true;
  int ab = 0, ba = 0;
  if (hipDeviceCanAccessPeer(&ab, a, b) != hipSuccess || hipDeviceCanAccessPeer(&ba, b, a) != hipSuccess) return false;
  if (!ab || !ba) return false;
  int prev = 0;
  HIP_CHECK(hipGetDevice(&prev));
  for (auto pr : {std::make_pair(a, b), std::make_pair(b, a)}) {
    HIP_CHECK(hipSetDevice(pr.first));
    const hipError_t e = hipDeviceEnablePeerAccess(pr.second, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
      (void)hipSetDevice(prev);
      return false;
    }
    (void)hipGetLastError();  // clear "already enabled"
  }
  HIP_CHECK(hipSetDevice(prev));
  return true;
}
#endif  // QI_PART <= 0

// Small kernels every engine shape uses (reduce, best-key fold, strided deal): defined in ONE
// part of this file and launched through these wrappers.  As per-shape template instances they
// lived in each part's code object, so a search on the run-time specialised kernel that ended
// with a witness loaded a whole part (4-5 ms) just to run its reduce.
void launch_reduce(uint32_t mw, const uint32_t* records, uint64_t n, uint32_t has_key, const uint32_t* key, uint32_t depth,
                   unsigned long long* out, uint32_t blocks, hipStream_t s);
void launch_min_best(unsigned long long* best64, uint32_t* poll_rep, unsigned long long v, hipStream_t s);
void launch_gather_units(uint32_t words, const uint32_t* in, uint64_t offset, uint64_t stride, uint64_t cnt, uint32_t* out,
                         uint32_t blocks, hipStream_t s);
// The frontier sort (radix passes over 32-bit keys with a permutation as values, hipCUB) and
// its helpers: one instance, not one per engine shape (the sort's template instances were
// ~2 MB of every part's code object).
void sort_pairs_u32(void* temp, size_t* temp_bytes, uint32_t* k_in, uint32_t* k_out, uint32_t* v_in, uint32_t* v_out, int n,
                    int end_bit, hipStream_t s);
void launch_iota(uint32_t* p, uint64_t n, uint32_t blocks, hipStream_t s);
void launch_unit_word(const uint32_t* units, uint32_t words, uint32_t off, const uint32_t* perm, uint64_t n, uint32_t* keys,
                      uint32_t blocks, hipStream_t s);
void launch_gather_perm(uint32_t words, const uint32_t* in, const uint32_t* perm, uint64_t n, uint32_t* out, uint32_t blocks,
                        hipStream_t s);
#if QI_PART <= 0
namespace dev {
// Fold a host-known best witness into the device-side one and its polled replicas (1-word keys).
static __global__ void min_best_kernel(unsigned long long* best64, uint32_t* poll_rep, unsigned long long v) {
  if (threadIdx.x == 0) atomicMin(best64, v);
  if (threadIdx.x < POLL_REPS) atomicMin((unsigned long long*)(poll_rep + (size_t)threadIdx.x * 32), v);
}

// A rank's share of a broadcast frontier, dealt in rounds of `stride` units with a rotating
// offset: out[q] = in[q * stride + (offset - q) mod stride].  (A plain stride keeps any
// period of the frontier order that divides it: spilled stacks alternate size classes, and
// stride 8 once gave ranks 10 M vs 19 M nodes.)  `words` per unit, a multiple of 4.
static __global__ void gather_units_kernel(uint32_t words, const uint32_t* in, uint64_t offset, uint64_t stride, uint64_t cnt,
                                           uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t src = i * stride + (offset + stride - i % stride) % stride;
    const uint4* s4 = (const uint4*)(in + src * words);
    uint4* d4 = (uint4*)(out + i * words);
    for (uint32_t q = 0; q < words / 4; ++q) d4[q] = s4[q];
  }
}

// Preorder-filtered sums over a log chunk: segment roots at or before (key, depth); records
// of mw key words + depth, count, evals, minq, zero_fallback (RecLayout).  Wave shuffles, then
// one LDS combine per block and one atomic per value per block (a same-address atomic per
// wave serialised ~65K atomics at the L2: 0.53 ms per reduce).
static __global__ __launch_bounds__(256) void reduce_kernel(uint32_t mw, const uint32_t* records, uint64_t n, uint32_t has_key,
                                                            const uint32_t* key, uint32_t depth, unsigned long long* out) {
  __shared__ unsigned long long part[4][4];
  uint64_t s[4] = {0, 0, 0, 0};
  const uint32_t rw = mw + 5;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t* r = records + i * rw;
    if (has_key) {  // preorder "strictly after": padded path bits, then depth
      bool after = r[mw] > depth;
      for (uint32_t w = mw; w-- > 0;)
        if (r[w] != key[w]) after = r[w] > key[w];
      if (after) continue;
    }
    s[0] += r[mw + 1];
    s[1] += r[mw + 2];
    s[2] += r[mw + 3];
    s[3] += r[mw + 4];
  }
  const uint32_t wv = threadIdx.x >> 6;
  for (int q = 0; q < 4; ++q) {
    uint64_t v = s[q];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63) == 0) part[wv][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long v = 0;
    for (uint32_t w = 0; w < (blockDim.x >> 6); ++w) v += part[w][threadIdx.x];
    if (v) atomicAdd(&out[threadIdx.x], v);
  }
}
}  // namespace dev
void launch_reduce(uint32_t mw, const uint32_t* records, uint64_t n, uint32_t has_key, const uint32_t* key, uint32_t depth,
                   unsigned long long* out, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL(dev::reduce_kernel, dim3(blocks), dim3(256), 0, s, mw, records, n, has_key, key, depth, out);
}
void launch_min_best(unsigned long long* best64, uint32_t* poll_rep, unsigned long long v, hipStream_t s) {
  hipLaunchKernelGGL(dev::min_best_kernel, dim3(1), dim3(64), 0, s, best64, poll_rep, v);
}
void launch_gather_units(uint32_t words, const uint32_t* in, uint64_t offset, uint64_t stride, uint64_t cnt, uint32_t* out,
                         uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL(dev::gather_units_kernel, dim3(blocks), dim3(256), 0, s, words, in, offset, stride, cnt, out);
}
#endif  // QI_PART <= 0
#if QI_PART < 0 || QI_PART == 6  // the frontier sort: a code object of its own, loaded by the first sort
namespace dev {
static __global__ void iota_kernel(uint32_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i;
}
static __global__ void unit_word_kernel(const uint32_t* units, uint32_t words, uint32_t off, const uint32_t* perm, uint64_t n,
                                        uint32_t* keys) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    keys[i] = units[(uint64_t)perm[i] * words + off];
}
static __global__ void gather_perm_kernel(uint32_t words, const uint32_t* in, const uint32_t* perm, uint64_t n, uint32_t* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4* s4 = (const uint4*)(in + (uint64_t)perm[i] * words);
    uint4* d4 = (uint4*)(out + i * words);
    for (uint32_t q = 0; q < words / 4; ++q) d4[q] = s4[q];
  }
}
}  // namespace dev
void sort_pairs_u32(void* temp, size_t* temp_bytes, uint32_t* k_in, uint32_t* k_out, uint32_t* v_in, uint32_t* v_out, int n,
                    int end_bit, hipStream_t s) {
  HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, k_in, k_out, v_in, v_out, n, 0, end_bit, s));
}
void launch_iota(uint32_t* p, uint64_t n, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL(dev::iota_kernel, dim3(blocks), dim3(256), 0, s, p, n);
}
void launch_unit_word(const uint32_t* units, uint32_t words, uint32_t off, const uint32_t* perm, uint64_t n, uint32_t* keys,
                      uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL(dev::unit_word_kernel, dim3(blocks), dim3(256), 0, s, units, words, off, perm, n, keys);
}
void launch_gather_perm(uint32_t words, const uint32_t* in, const uint32_t* perm, uint64_t n, uint32_t* out, uint32_t blocks,
                        hipStream_t s) {
  hipLaunchKernelGGL(dev::gather_perm_kernel, dim3(blocks), dim3(256), 0, s, words, in, perm, n, out);
}
#endif  // frontier sort

// hipStreamCreate costs ~2.4 ms on this stack (measured, QI_TRACE; the first one of a process
// far more): engines and the per-SCC checker take their stream from ONE per-device pool and
// return it, so a solve creates none.  The pool is defined in one part of this file only:
// an instance per part gave every engine shape an empty pool of its own.
hipStream_t acquire_stream(int device);
void release_stream(int device, hipStream_t s);
#if QI_PART <= 0
struct StreamPool {
  std::mutex mu;
  std::vector<std::pair<int, hipStream_t>> free;
};
StreamPool& stream_pool() {
  static StreamPool* p = new StreamPool;  // leaked on purpose: streams outlive static teardown
  return *p;
}
hipStream_t acquire_stream(int device) {
  {
    std::lock_guard<std::mutex> g(stream_pool().mu);
    auto& fr = stream_pool().free;
    for (size_t i = 0; i < fr.size(); ++i)
      if (fr[i].first == device) {
        hipStream_t s = fr[i].second;
        fr.erase(fr.begin() + (long)i);
        return s;
      }
  }
  hipStream_t s = nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (std::getenv("QI_TRACE"))
    std::fprintf(stderr, "[qi]   hipStreamCreate (device %d): %.3f ms\n", device,
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return s;
}
void release_stream(int device, hipStream_t s) {
  if (!s) return;
  (void)hipStreamSynchronize(s);
  std::lock_guard<std::mutex> g(stream_pool().mu);
  stream_pool().free.emplace_back(device, s);
}
// Pinned staging buffers of the per-SCC checker, pooled the same way: the first
// hipHostMalloc of a process beyond a few KB cost 5-6 ms inside the first solve (a
// 512-validator network's 31 KB against 7 KB for 256 validators).  device_prepare creates
// one of kStageMin bytes with the device.
constexpr size_t kStageMin = 256u << 10;
struct StagePool {
  std::mutex mu;
  std::vector<std::pair<unsigned long long*, size_t>> free;  // (buffer, bytes)
};
StagePool& stage_pool() {
  static StagePool* p = new StagePool;  // leaked on purpose, like the streams
  return *p;
}
unsigned long long* acquire_stage(size_t bytes, size_t* cap) {
  {
    std::lock_guard<std::mutex> g(stage_pool().mu);
    auto& fr = stage_pool().free;
    for (size_t i = 0; i < fr.size(); ++i)
      if (fr[i].second >= bytes) {
        unsigned long long* b = fr[i].first;
        *cap = fr[i].second;
        fr.erase(fr.begin() + (long)i);
        return b;
      }
  }
  const size_t want = std::max(bytes, kStageMin);
  unsigned long long* b = nullptr;
  HIP_CHECK(hipHostMalloc((void**)&b, want, hipHostMallocPortable));
  *cap = want;
  return b;
}
void release_stage(unsigned long long* b, size_t cap) {
  if (!b) return;
  std::lock_guard<std::mutex> g(stage_pool().mu);
  stage_pool().free.emplace_back(b, cap);
}
#endif  // QI_PART <= 0

namespace {

// Stack levels of the run-time specialised kernel for a template shape.  |SCC| <= 32: 20
// levels leave LDS for 9 resident waves per CU instead of 8 (17,408 B per wave).  Measured
// on the bench workload: 24 / 22 / 21 / 20 / 19 / 14 levels = 8 / 8 / 8 / 9 / 9 / 12 waves gave
// 2.63 / 2.62 / 2.55 / 2.39 / 2.38 / 2.48 ms; below 19 the extra stack evictions cost more
// than the waves bring.  The engine and jit_precompile must agree (the cache key is the source).
inline int jit_default_smax(int MW, int SMAX) {
  int s = MW == 1 ? 20 : SMAX;
  if (const char* e = std::getenv("QI_JIT_SMAX")) s = std::max(4, std::min(64, std::atoi(e)));  // diagnostics
  return s;
}

template <typename T>
T* dalloc(size_t count) {
  void* p = nullptr;
  if (count == 0) count = 1;
  const hipError_t e = hipMalloc(&p, count * sizeof(T));
  if (e != hipSuccess) {
    (void)hipGetLastError();  // not sticky for later calls
    throw Error(e == hipErrorOutOfMemory ? QI_ERR_CAPACITY : QI_ERR_DEVICE,
                "hipMalloc(" + std::to_string(count * sizeof(T)) + " B): " + hipGetErrorString(e));
  }
  return (T*)p;
}

template <typename T>
T* dupload(const std::vector<T>& v, hipStream_t s) {
  T* p = dalloc<T>(v.size());
  if (!v.empty()) HIP_CHECK(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return p;
}

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int d) {
    HIP_CHECK(hipGetDevice(&prev));
    HIP_CHECK(hipSetDevice(d));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

#if QI_PART <= 0
class GfpDeviceImpl : public GfpDevice {
 public:
  GfpDeviceImpl(int device, const GlobalFlat& g) : device_(device) {
    DeviceGuard dg(device_);
    auto tc0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
      if (!timing::enabled()) return;
      const auto now = std::chrono::steady_clock::now();
      timing::add((std::string("gfp_") + what).c_str(), std::chrono::duration<double, std::milli>(now - tc0).count());
      tc0 = now;
    };
    static_ = static_scratch_ptr(device_);  // set-up: this device's scratch array address
    lap("scratch_symbol");
    // the stream goes back to the per-device pool after set-up and after every run(), so the
    // search engine of the same solve reuses it (a stream costs ~2 ms to create, the first
    // one of a process ~9 ms)
    stream_ = acquire_stream(device_);
    lap("stream");
    HIP_CHECK(hipEventCreate(&e0_));
    HIP_CHECK(hipEventCreate(&e1_));
    lap("events");
    d_.n = g.n;
    d_.words = g.words;
    d_.T = g.T;
    d_.levels = g.levels;
    d_.nonmonotone = g.nonmonotone ? 1u : 0u;
    bufs_.push_back(d_.level_off = dupload(g.level_off, stream_));
    bufs_.push_back(d_.kind = dupload(g.kind, stream_));
    bufs_.push_back(d_.thr = dupload(g.thr, stream_));
    bufs_.push_back(d_.first = dupload(g.first, stream_));
    bufs_.push_back(d_.vref_off = dupload(g.vref_off, stream_));
    bufs_.push_back(d_.vref = dupload(g.vref, stream_));
    bufs_.push_back(d_.cref_off = dupload(g.cref_off, stream_));
    bufs_.push_back(d_.cref = dupload(g.cref, stream_));
    bufs_.push_back(d_.root = dupload(g.root, stream_));
    rounds_ = dalloc<unsigned long long>(1);
    lap("alloc_upload");
    HIP_CHECK(hipStreamSynchronize(stream_));
    release_stream(device_, stream_);
    stream_ = nullptr;
    lap("sync");
  }
  ~GfpDeviceImpl() override {
    DeviceGuard dg(device_);
    for (auto* p : bufs_) (void)hipFree((void*)p);
    (void)hipFree(rounds_);
    (void)hipFree(io_);
    (void)hipFree(scratch_);
    release_stage(hio_, hio_bytes_);
    (void)hipEventDestroy(e0_);
    (void)hipEventDestroy(e1_);
    release_stream(device_, stream_);
  }
  struct StreamLease {  // the engine's stream for the duration of one call
    GfpDeviceImpl& g;
    explicit StreamLease(GfpDeviceImpl& g_) : g(g_) { g.stream_ = acquire_stream(g.device_); }
    ~StreamLease() {
      release_stream(g.device_, g.stream_);
      g.stream_ = nullptr;
    }
  };
  void run(const uint64_t* nodes, const uint64_t* avail, uint32_t count, uint64_t* out) override {
    if (count == 0) return;
    DeviceGuard dg(device_);
    auto tc0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {  // QI_TIMING: where a batch's host time goes
      if (!timing::enabled()) return;
      const auto now = std::chrono::steady_clock::now();
      timing::add((std::string("gfp_run_") + what).c_str(), std::chrono::duration<double, std::milli>(now - tc0).count());
      tc0 = now;
    };
    StreamLease lease(*this);
    lap("stream");
    const size_t per = (size_t)count * d_.words;
    if (io_cap_ < per && 3 * per * 8 > kZeroCopyBytes) {
      (void)hipFree(io_);
      io_ = dalloc<unsigned long long>(3 * per);
      io_cap_ = per;
    }
    if (hio_bytes_ < 3 * per * 8) {
      release_stage(hio_, hio_bytes_);
      hio_ = acquire_stage(3 * per * 8, &hio_bytes_);
      HIP_CHECK(hipHostGetDevicePointer((void**)&hio_dev_, hio_, 0));
    }
    // A small batch (the per-SCC checks of a solve) is read and written by the kernel
    // straight in the pinned buffer: the first hipMemcpyAsync of a process beyond ~16 KB
    // brings up a copy queue (5.6 ms inside the first solve of a 512-validator network).
    const bool zero_copy = 3 * per * 8 <= kZeroCopyBytes;
    lap("buffers");
    unsigned long long* dn = zero_copy ? hio_dev_ : io_;
    unsigned long long* da = dn + per;
    unsigned long long* dout = dn + 2 * per;
    // both inputs through one pinned staging buffer: one DMA each way per batch
    std::memcpy(hio_, nodes, per * 8);
    std::memcpy(hio_ + per, avail, per * 8);
    if (!zero_copy) HIP_CHECK(hipMemcpyAsync(dn, hio_, 2 * per * 8, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemsetAsync(rounds_, 0, 8, stream_));
    const size_t shm = (size_t)d_.words * 16 + ((d_.T + 15) / 16) * 16;
    HIP_CHECK(hipEventRecord(e0_, stream_));
    if (shm <= kLdsImage) {
      hipLaunchKernelGGL(dev::gfp_batch_kernel<false>, dim3(count), dim3(64), shm, stream_, d_, dn, da, count, dout,
                         rounds_, nullptr, (size_t)0);
    } else {  // a network too large for the LDS image: the same kernel on global scratch
      const size_t need = shm * count;
      if (scratch_cap_ < need) {
        (void)hipFree(scratch_);
        scratch_ = dalloc<uint8_t>(need);
        scratch_cap_ = need;
      }
      hipLaunchKernelGGL(dev::gfp_batch_kernel<true>, dim3(count), dim3(64), 0, stream_, d_, dn, da, count, dout, rounds_,
                         scratch_, shm);
    }
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(e1_, stream_));
    if (!zero_copy) HIP_CHECK(hipMemcpyAsync(hio_ + 2 * per, dout, per * 8, hipMemcpyDeviceToHost, stream_));
    lap("enqueue");
    HIP_CHECK(hipStreamSynchronize(stream_));
    lap("sync");
    std::memcpy(out, hio_ + 2 * per, per * 8);
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0_, e1_));
    last_ms_ = ms;
  }
  // No allocation on this path: the tables were uploaded by the constructor, the masks are
  // the caller's device memory and the per-query state lives in this GPU's static scratch
  // array.  Every call on a GPU shares that array (calls that overlap on one GPU race) and
  // finds the previous call's contents in it: the counter header is cleared by a fill
  // kernel, the state images are fully rewritten by the kernel before it reads them.
  void run_static(const uint64_t* d_nodes, const uint64_t* d_avail, uint32_t count, uint64_t* d_out,
                  void* stream) override {
    if (count == 0) return;
    DeviceGuard dg(device_);
    const size_t per = (size_t)d_.words * 16 + ((d_.T + 15) / 16) * 16;  // multiple of 16 B
    const size_t room = kStaticScratchBytes - kStaticScratchHeader;
    if (per > room || (size_t)count > room / per)
      throw Error(QI_ERR_CAPACITY, "qi_gfp_batch_static: " + std::to_string(count) + " queries x " + std::to_string(per) +
                                       " B of state exceed the " + std::to_string(room) + " B static scratch (at most " +
                                       std::to_string(room / per) + " queries per call for this network)");
    for (const void* p : {(const void*)d_nodes, (const void*)d_avail, (const void*)d_out}) {
      hipPointerAttribute_t at{};
      if (hipPointerGetAttributes(&at, p) != hipSuccess ||
          (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged) || at.device != device_) {
        (void)hipGetLastError();
        throw Error(QI_ERR_ARG, "qi_gfp_batch_static: masks must be device memory of HIP device " + std::to_string(device_));
      }
    }
    // no caller stream: HIP's default stream of this device (creating or borrowing a stream
    // of the library's pool could allocate)
    hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t) nullptr;
    unsigned long long* rounds = (unsigned long long*)static_;
    hipLaunchKernelGGL(dev::zero_u64_kernel, dim3(1), dim3(64), 0, s, rounds, (uint32_t)(kStaticScratchHeader / 8));
    hipLaunchKernelGGL(dev::gfp_batch_kernel<true>, dim3(count), dim3(64), 0, s, d_,
                       (const unsigned long long*)d_nodes, (const unsigned long long*)d_avail, count,
                       (unsigned long long*)d_out, rounds, (uint8_t*)(static_ + kStaticScratchHeader), per);
    HIP_CHECK(hipGetLastError());
    if (!stream) HIP_CHECK(hipStreamSynchronize(nullptr));
  }
  double last_kernel_ms() const override { return last_ms_; }

 private:
  int device_;
  unsigned char* static_ = nullptr;  // this device's static scratch array (device address)
  hipStream_t stream_{};
  hipEvent_t e0_{}, e1_{};
  dev::GlobalDev d_{};
  std::vector<const uint32_t*> bufs_;
  unsigned long long* rounds_ = nullptr;
  unsigned long long* io_ = nullptr;
  unsigned long long* hio_ = nullptr;  // pinned staging (pooled): nodes, avail, out
  size_t hio_bytes_ = 0;
  unsigned long long* hio_dev_ = nullptr;  // the same buffer as the device sees it
  static constexpr size_t kZeroCopyBytes = 64u << 10;
  size_t io_cap_ = 0;
  uint8_t* scratch_ = nullptr;  // global-memory query state (networks beyond the LDS image)
  size_t scratch_cap_ = 0;
 public:
  static size_t kLdsImage;      // LDS bytes one query may use (QI_GFP_LDS overrides: tests)
 private:
  double last_ms_ = 0;
};
size_t GfpDeviceImpl::kLdsImage = 160 * 1024;
#endif  // QI_PART <= 0

// ORD = false: search_kernel / the run-time specialised kernel (monotone SCCs);
// ORD = true: ordered_kernel (SCCs with threshold-0 quorum sets), same protocol.
template <int MW, int TW, int SMAX, bool ORD = false>
class SearchDeviceImpl : public SearchDevice {
  using UL = std::conditional_t<ORD, dev::OrdUnitLayout<MW>, dev::UnitLayout<MW>>;
  using RL = dev::RecLayout<MW>;
  using WL = dev::WitLayout<MW>;

 public:
  SearchDeviceImpl(int device, const LocalFlat& f, const SearchConfig& cfg)
      : device_(device), cfg_(cfg), m_(f.m), flat_(f) {
    DeviceGuard dg(device_);
    trace_ = std::getenv("QI_TRACE") != nullptr;
    auto tc0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
      if (!trace_ && !timing::enabled()) return;
      const auto now = std::chrono::steady_clock::now();
      const double ms = std::chrono::duration<double, std::milli>(now - tc0).count();
      if (trace_) std::fprintf(stderr, "[qi]   ctor %-22s %.3f ms\n", what, ms);
      timing::add((std::string("engine_") + what).c_str(), ms);
      tc0 = now;
    };
    // tuning overrides for experiments (profiling only; defaults are the measured best)
    if (const char* e = std::getenv("QI_GRACE")) cfg_.grace = (uint32_t)std::atoi(e);
    if (const char* e = std::getenv("QI_GROW")) cfg_.grow_budget = (uint32_t)std::max(1, std::atoi(e));
    if (const char* e = std::getenv("QI_EVICT")) cfg_.evict_max = (uint32_t)std::atoi(e);
    if (const char* e = std::getenv("QI_RUN_AT")) cfg_.run_at = (uint32_t)std::atoi(e);
    if (const char* e = std::getenv("QI_LOOKAHEAD")) cfg_.lookahead = (uint32_t)std::max(1, std::atoi(e));
    if (const char* e = std::getenv("QI_MAX_FRONTIER_GB")) max_frontier_bytes_ = (uint64_t)std::atoll(e) << 30;
    jit_smax_ = ORD ? SMAX : jit_default_smax(MW, SMAX);
    if (ORD) cfg_.jit = 1;  // no run-time specialisation of the ordered kernel
    if (ORD && cfg_.tiebreak)
      throw Error(QI_ERR_UNSUPPORTED,
                  "QI_TIE_RANDOM: the order-exact kernel (threshold-0 quorum sets, SCCs beyond 256 vertices) only has "
                  "the lowest-index rule");
    stream_ = acquire_stream(device_);
    HIP_CHECK(hipEventCreate(&e0_));
    HIP_CHECK(hipEventCreate(&e1_));
    lap("stream/events");
    // pack one record per TN (TnRec layout), padded to the template's word counts
    using RC = dev::TnRec<MW, TW>;
    const uint32_t T = f.T;
    std::vector<uint32_t> rec((size_t)std::max<uint32_t>(T, 1) * RC::WORDS, 0);
    for (uint32_t t = 0; t < T; ++t) {
      uint32_t* r = &rec[(size_t)t * RC::WORDS];
      for (uint32_t w = 0; w < f.mw; ++w) r[w] = f.vmask[(size_t)t * f.mw + w];
      for (uint32_t w = 0; w < f.tw; ++w) r[MW + w] = f.cmask[(size_t)t * f.tw + w];
      const bool inv = (f.flags[t] & 1u) != 0;
      r[RC::THR0] = inv ? 1u : (uint32_t)f.thr[2 * t];
      r[RC::THR1] = inv ? 1u : (uint32_t)f.thr[2 * t + 1];
      r[RC::INV] = inv ? 1u : 0u;
      r[RC::EXTRA] = (f.flags[t] & 2u) ? 1u : 0u;
    }
    std::vector<uint32_t> extra_src = f.extra_src;
    for (auto& x : extra_src)
      if (x >= f.mw) x = x - f.mw + MW;  // re-base TN-sat words after padding
    auto pad_rows = [&](const std::vector<uint32_t>& v, size_t rows) {
      std::vector<uint32_t> o(rows * MW, 0);
      for (size_t r = 0; r < rows; ++r)
        for (uint32_t w = 0; w < f.mw; ++w) o[r * MW + w] = v[r * f.mw + w];
      return o;
    };
    d_.T = T;
    d_.R = f.R;
    d_.G = f.G;
    d_.m = f.m;
    d_.qmin0 = f.qmin[0];
    d_.qmin1 = f.qmin[1];
    keep(d_.tn = dupload(rec, stream_));
    keep(d_.extra_off = dupload(f.extra_off, stream_));
    keep(d_.extra_src = dupload(extra_src, stream_));
    keep(d_.extra_mask = dupload(f.extra_mask, stream_));
    keep(d_.root_tn = dupload(f.root_tn, stream_));
    keep(d_.root_users = dupload(pad_rows(f.root_users, f.R), stream_));
    keep(d_.grp_members = dupload(pad_rows(f.grp_members, f.G), stream_));
    keep(d_.grp_col = dupload(pad_rows(f.grp_col, f.G), stream_));
    keep(d_.grp_extra_off = dupload(f.grp_extra_off, stream_));
    const size_t ge = f.grp_extra_off.empty() ? 0 : f.grp_extra_off.back();
    keep(d_.grp_extra = dupload(pad_rows(f.grp_extra, ge), stream_));
    lap("tables");
    for (uint32_t w = 0; w < 32; ++w) scc_mask_[w] = 0;
    for (uint32_t v = 0; v < f.m; ++v) scc_mask_[v >> 5] |= 1u << (v & 31);
    for (uint32_t w = 0; w < 32; ++w) d_.scc_mask[w] = scc_mask_[w];
    if (ORD) {  // per-vertex roots, SCC-local adjacency, hash buckets of the global ids
      keep(ord_.vroot = dupload(f.vroot, stream_));
      keep(ord_.adj_off = dupload(f.ladj_off, stream_));
      keep(ord_.adj = dupload(f.ladj, stream_));
      std::vector<uint16_t> bm((size_t)dev::kHashSizes * f.m);
      for (uint32_t r = 0; r < (uint32_t)dev::kHashSizes; ++r)
        for (uint32_t v = 0; v < f.m; ++v) bm[(size_t)r * f.m + v] = (uint16_t)(f.scc[v] % dev::kHashBuckets[r]);
      keep(ord_.bktmod = dupload(bm, stream_));
      ord_.smax = kOrdSmax;
      ord_.depth_max = 32u * MW;
      // monotone (here for its size, or forced): sweep order is immaterial; QI_ORDERED=2
      // keeps the exact sweeps anyway (diagnostics: exercises them on monotone inputs)
      const char* fo = std::getenv("QI_ORDERED");
      ord_.jacobi = (f.nonmonotone || (fo && std::atoi(fo) == 2)) ? 0u : 1u;
      ord_.probe = 2048;
      if (const char* e = std::getenv("QI_PROBE")) ord_.probe = (uint32_t)std::atoi(e);
    }

    cus_ = (uint32_t)device_cu_count(device_);
    max_blocks_ = cfg_.max_blocks ? cfg_.max_blocks : cus_ * 8u;  // refined below once shm_ is known
    ctr_ = dalloc<uint32_t>((size_t)(kMaxBatch + 1) * dev::CTR_WORDS);
    glob_ = dalloc<uint32_t>(2);
    HIP_CHECK(hipMemsetAsync(glob_, 0, 8, stream_));
    // pinned: the launches' published counters, the flag words of a chain's end, a snapshot of
    // the running totals (copied with the flags at every chain end: reading the totals after
    // a search then needs no device round trip) and the root unit
    constexpr size_t kTotBytes = 16 * dev::TOT_SHARDS * sizeof(unsigned long long);
    HIP_CHECK(hipHostMalloc((void**)&hctr_, (size_t)kMaxBatch * dev::HC_WORDS * 4 + 64 + kTotBytes + UL::BYTES,
                            hipHostMallocMapped | hipHostMallocCoherent));
    HIP_CHECK(hipHostGetDevicePointer((void**)&hctr_dev_, (void*)hctr_, 0));
    glob_host_ = hctr_ + (size_t)kMaxBatch * dev::HC_WORDS;
    totals_host_ = (unsigned long long*)(hctr_ + (size_t)kMaxBatch * dev::HC_WORDS + 16);
    root_host_ = (uint32_t*)(totals_host_ + 16 * dev::TOT_SHARDS);
    std::memset((void*)totals_host_, 0, kTotBytes);
    totals_host_valid_ = true;  // totals_ is zeroed below
    lap("counters+pinned");
    for (auto& e : ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDefault));
    lap("chain events");
    totals_ = dalloc<unsigned long long>(16 * dev::TOT_SHARDS);
    best64_ = dalloc<unsigned long long>(1);
    poll_rep_ = dalloc<uint32_t>((size_t)dev::POLL_REPS * 32);
    diag_waves_on_ = std::getenv("QI_DIAG_WAVES") != nullptr;  // diagnostics: per-wave timestamps of every launch
    HIP_CHECK(hipMemsetAsync(poll_rep_, 0xFF, (size_t)dev::POLL_REPS * 128, stream_));
    red_ = dalloc<unsigned long long>(4);
    keydev_ = dalloc<uint32_t>(dev::KEY_WORDS_MAX);
    wit_cap_ = 1u << 16;
    wit_ = dalloc<uint32_t>((size_t)wit_cap_ * WL::WORDS);
    HIP_CHECK(hipMemsetAsync(totals_, 0, 16 * dev::TOT_SHARDS * sizeof(unsigned long long), stream_));
    unsigned long long inf = ~0ull;
    HIP_CHECK(hipMemcpyAsync(best64_, &inf, 8, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    shm_ = ORD ? 0 : (size_t)dev::search_lds_words<MW, SMAX>() * 4;
    shm_ = (shm_ + 15) / 16 * 16;
    // QI_JIT_SMAX (diagnostics): LDS bytes per stack level as in search_lds_words
    jit_shm_ = (size_t)jit_smax_ * (2 * MW + 1) * 64 * 4 + (shm_ - (size_t)SMAX * (2 * MW + 1) * 64 * 4);
    if (!ORD) {  // the specialised kernel's D-order words are sized for this SCC (QI_LDS_OW)
      const size_t ow_full = (dev::UnitLayout<MW>::DMAX + 3) / 4, owl = std::min<size_t>(jit_lds_ow(flat_), ow_full);
      jit_shm_ -= (ow_full - owl) * 64 * 4;
    }
    jit_shm_ = (jit_shm_ + 15) / 16 * 16;
    // The ahead-of-time kernel's attributes and occupancy are looked up when it is first
    // needed (aot_setup): touching it loads its code object (~6 ms), which a search that
    // runs the cached specialised kernel from its first launch never pays.
    if ((cfg_.jit == 0 || cfg_.jit == 4) && jit_eligible(flat_)) {
      // auto / cache-only: a specialised kernel already in the on-disk cache runs from the
      // first launch (hipModuleLoadData, ~1 ms); auto compiles a missing one in the
      // background once the search proves long (step()), cache-only never compiles
      jit_code_ = jit_cached(jit_source(flat_, MW, TW, jit_smax_, false, cfg_.tiebreak != 0));
      if (!jit_code_.empty()) {
        jit_state_.store(2);
        load_jit();
      }
    }
    if ((cfg_.jit == 2 || cfg_.jit == 3) && jit_eligible(flat_)) {
      start_jit();
      if (!wait_jit()) throw Error(QI_ERR_UNSUPPORTED, "specialised kernel failed to build: " + jit_log_);
    }
    lap("jit");
    if (ORD || !jit_fn_) aot_setup();
    lap("aot_kernel");
    reset_root();
    lap("root");
  }

  ~SearchDeviceImpl() override {
    if (jit_thread_.joinable()) jit_thread_.join();
    DeviceGuard dg(device_);
    if (jit_mod_) (void)hipModuleUnload(jit_mod_);
    for (auto* p : bufs_) (void)hipFree(p);
    for (int i = 0; i < 2; ++i) (void)hipFree(units_[i]);
    for (auto& c : log_) (void)hipFree(c.ptr);
    (void)hipFree(ctr_);
    (void)hipFree(glob_);
    (void)hipHostFree((void*)hctr_);
    for (auto& e : ev_) (void)hipEventDestroy(e);
    (void)hipFree(totals_);
    (void)hipFree(best64_);
    (void)hipFree(poll_rep_);
    (void)hipFree(diag_waves_);
    (void)hipFree(red_);
    (void)hipFree(keydev_);
    (void)hipFree(wit_);
    pinned_word_free(xbest_bridge_);
    for (auto* p : {sk_[0], sk_[1], sp_[0], sp_[1]}) (void)hipFree(p);
    (void)hipFree(stemp_);
    (void)hipEventDestroy(e0_);
    (void)hipEventDestroy(e1_);
    release_stream(device_, stream_);
  }

  int device() const override { return device_; }
  uint32_t key_words() const override { return MW; }
  uint32_t unit_bytes() const override { return UL::BYTES; }

  void reset_root() override {
    DeviceGuard dg(device_);
    ensure_cap(0, 1);
    if (!root_ready_) {  // the root unit, kept in pinned memory: later resets only enqueue its copy
      uint32_t* u = root_host_;
      std::memset(u, 0, UL::BYTES);
      if constexpr (ORD) {  // toRemove = scc in ascending order, dontRemove = {} (cpp:393)
        u[UL::TLEN] = m_;
        for (uint32_t v = 0; v < m_; ++v) u[UL::TORD + v / UL::EPW] |= v << (32 / UL::EPW * (v % UL::EPW));
      } else {
        for (int w = 0; w < MW; ++w) u[UL::T_ + w] = scc_mask_[w];  // toRemove = scc, dontRemove = {} (cpp:393)
      }
      root_ready_ = true;
    }
    HIP_CHECK(hipMemcpyAsync(units_[cur_], root_host_, UL::BYTES, hipMemcpyHostToDevice, stream_));
    n_ = 1;
  }

  void clear_frontier() override { n_ = 0; }

  uint64_t frontier_size() const override { return n_; }

  // One step = a chain of up to `batch` launches (see C_* in qi_search_kernel.h).  Every
  // launch reads its input count and log position from the previous launch's counter
  // block on the device, so the host only enqueues.  It keeps `lookahead` launches in
  // flight beyond the one it waits for; the last block of each launch publishes that
  // launch's counters into pinned host memory, so the host sees the frontier run empty
  // (or a capacity stop) without a copy and stops enqueueing: at most `lookahead` empty
  // launches trail a search.  A launch that could exceed the unit or log capacity does
  // nothing, and neither does the rest of the chain; the host grows the buffers and
  // resumes from that launch's input.
  StepInfo step(uint64_t until) override {
    DeviceGuard dg(device_);
    StepInfo si;
    si.frontier_in = n_;
    if (n_ == 0) return si;
    totals_host_valid_ = false;  // until this chain's end has copied the totals again
    // run-time specialised kernel: start compiling once the search proves non-trivial,
    // switch to it at the first step boundary after it is ready
    if (cfg_.jit == 0 && launches_ >= cfg_.jit_after && jit_state_.load() == 0 && jit_eligible(flat_)) start_jit();
    if (jit_state_.load() == 2) load_jit();
    const bool spec = jit_fn_ != nullptr;
    if (!spec) aot_setup();
    const uint32_t smax = ORD ? kOrdSmax : (spec ? (uint32_t)jit_smax_ : (uint32_t)SMAX);
    const uint32_t blocks = max_blocks_;
    const uint32_t K = std::max(1u, std::min(cfg_.batch ? cfg_.batch : (uint32_t)kMaxBatch, (uint32_t)kMaxBatch));
    // growing to a target: no look-ahead, so the chain stops at the first launch past it
    const uint32_t D = until ? 0u : std::max(1u, cfg_.lookahead);
    auto log_need = [&](uint64_t n) { return n; };  // the device's log check: one record per input unit
    auto first_need = [&](uint64_t n) {
      const uint64_t nb = std::min<uint64_t>((n + 63) / 64, blocks);
      return n + nb * 64u * (dev::spill_reserve(smax) + cfg_.evict_max);  // search_body's need_out
    };
    {
      timing::Scope tsc("frontier_alloc");
      const uint64_t need = first_need(n_);
      if (need > 0xFFFFFFF0ull) throw Error(QI_ERR_CAPACITY, "search frontier exceeds 2^32 units");
      ensure_cap(cur_, need, true);
      ensure_cap(1 - cur_, need);
      if (log_.empty() || log_.back().cap - log_.back().used < log_need(n_)) new_log_chunk(2 * log_need(n_));
    }
    if (diag_waves_on_) {  // diagnostics: per-wave timestamps of every launch of this chain
      if (!diag_waves_) diag_waves_ = dalloc<uint32_t>((size_t)kMaxBatch * blocks * 4);
      HIP_CHECK(hipMemsetAsync(diag_waves_, 0, (size_t)kMaxBatch * blocks * 16, stream_));
    }
    LogChunk& lc = log_.back();
    uint32_t seed[dev::CTR_WORDS] = {0};
    seed[dev::C_OUT] = (uint32_t)n_;
    seed[dev::C_LOGN] = (uint32_t)lc.used;
    HIP_CHECK(hipMemcpyAsync(ctr_, seed, sizeof seed, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemsetAsync(ctr_ + dev::CTR_WORDS, 0, (size_t)K * dev::CTR_WORDS * 4, stream_));
    std::memset((void*)hctr_, 0, (size_t)K * dev::HC_WORDS * 4);
    for (uint32_t k = 0; k < K; ++k)  // no best key published yet
      hctr_[(size_t)k * dev::HC_WORDS + dev::HC_BEST] = hctr_[(size_t)k * dev::HC_WORDS + dev::HC_BEST + 1] = 0xFFFFFFFFu;

    dev::SearchArgs a{};
    a.f = d_;
    a.out_cap = (uint32_t)std::min<uint64_t>(cap_[0], cap_[1]);
    a.log_cap = (uint32_t)std::min<uint64_t>(lc.cap, 0xFFFFFFF0ull);
    a.glob = glob_;
    a.records = lc.ptr;
    a.wit = wit_;
    a.wit_cap = wit_cap_;
    a.totals = totals_;
    a.best64 = best64_;
    a.xbest = xbest_dev_ ? xbest_dev_ : best64_;
    a.poll_rep = poll_rep_;
    a.diag_waves = nullptr;
    a.tiebreak = cfg_.tiebreak;
    a.tie_seed = cfg_.tie_seed;
    a.grow_budget = cfg_.grow_budget;
    a.run_budget = cfg_.run_budget;
    a.grace = cfg_.grace;
    a.run_at = cfg_.run_at;
    a.evict_max = cfg_.evict_max;
    a.half_m = m_ / 2;
    {  // cooperative slot: smallest power of two covering |D| + 1 <= half_m + 1 jobs
      uint32_t sl = 1, lg = 0;
      while (sl < a.half_m + 1 && sl < 64) {
        sl <<= 1;
        ++lg;
      }
      a.coop_slot = sl;
      a.coop_slot_log2 = lg;
    }
    a.has_best = has_best_ ? 1u : 0u;
    a.best_depth = best_depth_;
    static_assert(MW <= dev::KEY_WORDS_MAX, "path key wider than the key buffers");
    for (int w = 0; w < dev::KEY_WORDS_MAX; ++w) a.best_key[w] = w < (int)best_key_.size() ? best_key_[w] : 0u;
    if (MW == 1 && has_best_ && best_dirty_) {  // 1-word keys: the device best is exact; fold the host's in
      launch_min_best(best64_, poll_rep_, ((unsigned long long)best_key_[0] << 32) | best_depth_, stream_);
      HIP_CHECK(hipGetLastError());
    }
    best_dirty_ = false;
    HIP_CHECK(hipEventRecord(ev_[0], stream_));
    auto enqueue = [&](uint32_t k) {
      a.units_in = units_[(cur_ + k) & 1];
      a.units_out = units_[(cur_ + k + 1) & 1];
      a.prev = ctr_ + (size_t)k * dev::CTR_WORDS;
      a.counters = ctr_ + (size_t)(k + 1) * dev::CTR_WORDS;
      a.host_ctr = hctr_dev_ + (size_t)k * dev::HC_WORDS;
      if (diag_waves_) a.diag_waves = diag_waves_ + (size_t)k * blocks * 4;
      if (++seq_ == 0xFFFFFFFFu) seq_ = 1;  // (the replicas' reset value is never a sequence number)
      a.seq = seq_;
      if constexpr (ORD) {
        dev::OrdArgs oa = ord_;
        oa.a = a;
        hipLaunchKernelGGL((dev::ordered_kernel<MW, TW>), dim3(blocks), dim3(64), 0, stream_, oa);
      } else if (spec) {
        void* args[] = {&a};
        HIP_CHECK(hipModuleLaunchKernel(jit_fn_, blocks, 1, 1, 64, 1, 1, (unsigned)jit_shm_, stream_, args, nullptr));
      } else {
        if (cfg_.tiebreak) hipLaunchKernelGGL((dev::search_kernel<MW, TW, SMAX, true>), dim3(blocks), dim3(64), shm_, stream_, a);
        else hipLaunchKernelGGL((dev::search_kernel<MW, TW, SMAX, false>), dim3(blocks), dim3(64), shm_, stream_, a);
      }
      HIP_CHECK(hipGetLastError());
      if (trace_) HIP_CHECK(hipEventRecord(ev_[k + 1], stream_));  // per-launch times: diagnostics only
    };
    // Launch k's published flag word in pinned host memory: the host spins on it instead of
    // recording and waiting for an event per launch (an event between two chained launches
    // cost ~10 us of the ~13 us per launch boundary).
    auto wait_flag = [&](uint32_t k) -> uint64_t {
      volatile uint64_t* fp = (volatile uint64_t*)(hctr_ + (size_t)k * dev::HC_WORDS + dev::HC_FLAG);
      for (uint32_t spin = 0;; ++spin) {
        const uint64_t v = __atomic_load_n((const uint64_t*)fp, __ATOMIC_ACQUIRE);
        if (v >> 63) return v;
        if ((spin & 0xFFFu) == 0xFFFu) {  // a fault or a drained stream must not spin for ever
          const hipError_t q = hipStreamQuery(stream_);
          if (q == hipSuccess) {
            const uint64_t v2 = __atomic_load_n((const uint64_t*)fp, __ATOMIC_ACQUIRE);
            if (v2 >> 63) return v2;
            throw Error(QI_ERR_DEVICE, "search launch did not publish its counters");
          }
          if (q != hipErrorNotReady) throw Error(QI_ERR_DEVICE, std::string("search chain: ") + hipGetErrorString(q));
        }
        __builtin_ia32_pause();
      }
    };
    auto hc = [&](uint32_t k) -> const volatile uint32_t* { return hctr_ + (size_t)k * dev::HC_WORDS; };
    auto fold_best = [&](uint32_t k) {  // launch k's best key into the engines' shared word
      if (!xbest_host_ || !hc(k)[dev::HC_DONE] || hc(k)[dev::HC_STOP]) return;
      const uint64_t b = ((uint64_t)hc(k)[dev::HC_BEST + 1] << 32) | hc(k)[dev::HC_BEST];
      uint64_t cur = __atomic_load_n(xbest_host_, __ATOMIC_RELAXED);
      while (b < cur && !__atomic_compare_exchange_n(xbest_host_, &cur, b, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
      }
      if (xbest_bridge_) __atomic_store_n(xbest_bridge_, std::min(cur, b), __ATOMIC_RELAXED);
    };
    uint32_t enq = 0, folded = 0;
    while (enq < K) {
      enqueue(enq++);
      if (enq > D) {  // wait for launch enq-1-D; stop enqueueing once the chain has run out
        const uint32_t j = enq - 1 - D;
        const uint64_t fl = wait_flag(j);
        for (; folded <= j; ++folded) fold_best(folded);
        if (((fl >> 62) & 1u) || (uint32_t)fl == 0u) break;
        if (until && (uint32_t)fl >= until) break;
      }
    }
    if (!trace_) HIP_CHECK(hipEventRecord(ev_[1], stream_));  // the whole chain, first launch to last
    HIP_CHECK(hipMemcpyAsync((void*)glob_host_, glob_, 8, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync((void*)totals_host_, totals_, 16 * dev::TOT_SHARDS * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    totals_host_valid_ = true;
    for (; folded < enq; ++folded) fold_best(folded);
    const uint32_t g_wit = glob_host_[0], g_flags = glob_host_[1];
    if (g_flags & dev::FLAG_OUT_OVERFLOW) throw Error(QI_ERR_CAPACITY, "search frontier buffer overflow");
    if (g_flags & dev::FLAG_WIT_OVERFLOW) throw Error(QI_ERR_CAPACITY, "witness buffer overflow");
    if (g_flags & dev::FLAG_DEPTH)  // zero-fallback steps that keep T (cpp:221, 343): the
      // reference's recursion would not terminate either
      throw Error(QI_ERR_STATE, "search path deeper than the path key (non-terminating recursion)");
    // walk the chain: launches that ran, the first stopped one, the final frontier
    uint32_t ran = 0, k = 0;
    bool stopped = false;
    double ms_sum = 0;
    uint64_t n_next = n_, log_next = lc.used;
    bool halted = false;
    int cur_next = cur_;
    if (trace_) {
      for (uint32_t j = 0; j < enq; ++j) {
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, ev_[j], ev_[j + 1]));
        si.dispatch_ms += ms;
      }
    } else {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
      si.dispatch_ms = ms;
    }
    si.dispatches = enq;
    for (; k < enq; ++k) {
      const volatile uint32_t* c = hc(k);
      if (!c[dev::HC_DONE]) throw Error(QI_ERR_DEVICE, "search launch did not publish its counters");
      if (c[dev::HC_STOP]) {  // frontier = launch k's input
        stopped = true;
        break;
      }
      cur_next = (cur_ + k + 1) & 1;
      n_next = c[dev::HC_OUT];
      halted = c[dev::HC_HALT] != 0;
      log_next = c[dev::HC_LOGN];
      if (c[dev::HC_NIN] == 0) continue;
      ++ran;
      si.processed += c[dev::HC_NIN];
      float ms = 0;
      if (trace_) {
        HIP_CHECK(hipEventElapsedTime(&ms, ev_[k], ev_[k + 1]));
        ms_sum += ms;
      }
      if (trace_) {
        std::fprintf(stderr, "[qi]     launch %u: in %u out %u halt %u, %.1f us", k, c[dev::HC_NIN], c[dev::HC_OUT],
                     c[dev::HC_HALT], ms * 1e3);
        if (c[dev::HC_DIAG + 1])  // a QI_DIAG_LAUNCH build: this launch's nodes and wave iterations
          std::fprintf(stderr, ", nodes %u wave-iters %u", c[dev::HC_DIAG] - (c[dev::HC_DIAG] >= diag_prev_[0] ? diag_prev_[0] : 0u),
                       c[dev::HC_DIAG + 1] - (c[dev::HC_DIAG + 1] >= diag_prev_[1] ? diag_prev_[1] : 0u));
        if (c[dev::HC_DIAG + 1])
          std::fprintf(stderr, " (max %u), wave us avg %.1f max %.1f span %.1f", c[dev::HC_DIAG + 2],
                       c[dev::HC_DIAG + 3] * 0.01 / std::max(1u, std::min((c[dev::HC_NIN] + 63u) / 64u, blocks)),
                       c[dev::HC_DIAG + 4] * 0.01, c[dev::HC_DIAG + 5] * 0.01);
        if (c[dev::HC_DIAG + 6]) {  // waves that went dry and spilled: average phase times
          const double w = 0.01 / c[dev::HC_DIAG + 6];
          std::fprintf(stderr, "; %u dry waves: start %.1f, to dry %.1f, grace %.1f, spill %.1f (slot wait %.1f), end %.1f us",
                       c[dev::HC_DIAG + 6], c[dev::HC_DIAG + 7] * w, c[dev::HC_DIAG + 8] * w, c[dev::HC_DIAG + 9] * w,
                       c[dev::HC_DIAG + 10] * w, c[dev::HC_DIAG + 12] * w, c[dev::HC_DIAG + 11] * w);
        }
        diag_prev_[0] = c[dev::HC_DIAG];
        diag_prev_[1] = c[dev::HC_DIAG + 1];
        std::fprintf(stderr, "\n");
      }
    }
    if (diag_waves_) {  // per launch: waves, and percentiles of wave life, start -> dry, dry -> end (us)
      std::vector<uint32_t> dw((size_t)enq * blocks * 4);
      HIP_CHECK(hipMemcpy(dw.data(), diag_waves_, dw.size() * 4, hipMemcpyDeviceToHost));
      for (uint32_t j = 0; j < enq; ++j) {
        std::vector<double> life, todry, tail, endt;
        uint32_t t_first = 0xFFFFFFFFu;
        for (uint32_t b = 0; b < blocks; ++b) {
          const uint32_t* w = &dw[((size_t)j * blocks + b) * 4];
          if (w[3]) t_first = std::min(t_first, w[0]);
        }
        for (uint32_t b = 0; b < blocks; ++b) {
          const uint32_t* w = &dw[((size_t)j * blocks + b) * 4];
          if (!w[3]) continue;
          life.push_back((w[3] - w[0]) * 0.01);
          endt.push_back((w[3] - t_first) * 0.01);
          if (w[1]) {
            todry.push_back((w[1] - w[0]) * 0.01);
            tail.push_back((w[3] - w[1]) * 0.01);
          }
        }
        if (life.empty()) continue;
        auto pct = [](std::vector<double>& v, double p) {
          if (v.empty()) return 0.0;
          std::sort(v.begin(), v.end());
          return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
        };
        double sum = 0;
        for (double x : life) sum += x;
        std::fprintf(stderr,
                     "[qi]     waves of launch %u: %zu, life avg %.1f p50 %.1f p90 %.1f max %.1f | end after launch start p10 %.1f "
                     "p50 %.1f p90 %.1f max %.1f | start->dry p10 %.1f p50 %.1f p90 %.1f max %.1f | dry->end p50 %.1f p90 %.1f max %.1f us\n",
                     j, life.size(), sum / life.size(), pct(life, .5), pct(life, .9), pct(life, 1), pct(endt, .1), pct(endt, .5),
                     pct(endt, .9), pct(endt, 1), pct(todry, .1), pct(todry, .5), pct(todry, .9), pct(todry, 1), pct(tail, .5),
                     pct(tail, .9), pct(tail, 1));
      }
    }
    if (!trace_) ms_sum = si.dispatch_ms;  // the chain's kernels back to back (<= 2 empty launches at its end)
    n_ = n_next;
    cur_ = cur_next;
    lc.used = log_next;
    if (stopped) {
      timing::Scope tsc("frontier_alloc");
      const uint64_t need = first_need(n_);
      if (need > 0xFFFFFFF0ull) throw Error(QI_ERR_CAPACITY, "search frontier exceeds 2^32 units");
      if (need > std::min(cap_[0], cap_[1])) {  // grow once to the full-grid bound (ramp stops
        // cost a host round trip each)
        const uint64_t full = std::min<uint64_t>(std::max<uint64_t>(4 * need, first_need((uint64_t)blocks * 64u * 16u)),
                                                 0xFFFFFFF0ull);
        ensure_cap(cur_, full, true);
        ensure_cap(1 - cur_, full);
      }
      if (lc.cap - lc.used < log_need(n_)) new_log_chunk(2 * log_need(n_));
      ++stops_;
    }
    if (g_flags & dev::FLAG_POOL) {  // some lane found the eviction pool dry and stopped early:
      // double the frontier buffers (the current frontier is preserved), so the next
      // launches can dig deeper -- up to the frontier memory budget: past it lanes keep
      // spilling and stopping, which the preorder sort after a halt keeps progressing
      const uint64_t c2 = 2 * std::min(cap_[0], cap_[1]);
      if (2 * c2 * (uint64_t)UL::BYTES <= max_frontier_bytes_) {
        ensure_cap(cur_, c2, true);
        ensure_cap(1 - cur_, c2);
      }
      const uint32_t zero = 0;
      HIP_CHECK(hipMemcpyAsync(glob_ + 1, &zero, 4, hipMemcpyHostToDevice, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
      ++pool_growths_;
    }
    // The last launch that ran had to carry units over: its lanes spent their node budgets
    // with units left, so launches no longer cover the frontier.  Serve it in preorder
    // from now on: the preorder-first units (the only ones that can hold the first
    // witness) go to lanes first, and nothing after a found witness starves it.
    if (halted && n_ > 1) {
      sort_frontier();
      ++sorts_;
    }
    // collect new witnesses (the buffer restarts at 0 for the next step)
    if (g_wit > 0) {
      const uint32_t nw = std::min(g_wit, wit_cap_);
      std::vector<uint32_t> wv((size_t)nw * WL::WORDS);
      HIP_CHECK(hipMemcpyAsync(wv.data(), wit_, wv.size() * 4, hipMemcpyDeviceToHost, stream_));
      HIP_CHECK(hipMemsetAsync(glob_, 0, 8, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
      for (uint32_t i = 0; i < nw; ++i) absorb_witness(&wv[(size_t)i * WL::WORDS]);
      si.new_witnesses = nw;
    }
    if (trace_)
      std::fprintf(stderr,
                   "[qi]   step: %u launches enqueued, %u ran, processed %llu, frontier %llu, %s%s%s, wit %u, best %d, "
                   "cap %llu, kernel %.3f ms\n",
                   enq, ran, (unsigned long long)si.processed, (unsigned long long)n_,
                   stopped ? (halted ? "halt+sort" : "capacity stop") : "chain end", (g_flags & dev::FLAG_POOL) ? ", pool dry" : "",
                   "", g_wit, (int)has_best_, (unsigned long long)std::min(cap_[0], cap_[1]), si.dispatch_ms);
    // no-progress guard: a step that ran no unit and did not shrink the frontier (its first
    // launch stopped for capacity, which the host just fixed) may happen once in a row;
    // more means the chain cannot advance, and the caller gets an error instead of a spin
    if (si.processed == 0 && n_ >= si.frontier_in) {
      if (++idle_steps_ > 4) throw Error(QI_ERR_STATE, "search step made no progress (frontier " + std::to_string(n_) + ")");
    } else {
      idle_steps_ = 0;
    }
    si.frontier_out = n_;
    si.budget = cfg_.run_budget;
    si.blocks = blocks;
    si.kernel_ms = ms_sum;
    si.launches = ran;
    si.has_best = has_local_best_ || has_best_;
    si.specialized = spec;
    sum_ms_ += ms_sum;
    launches_ += ran;
    dispatches_ += enq;
    dispatch_ms_ += si.dispatch_ms;
    if (spec) spec_launches_ += ran;
    return si;
  }

  void export_tail(uint64_t count, void* dev_dst) override {
    DeviceGuard dg(device_);
    if (count > n_) throw Error(QI_ERR_ARG, "export: count exceeds frontier");
    HIP_CHECK(hipMemcpyAsync(dev_dst, units_[cur_] + (n_ - count) * UL::WORDS, count * UL::BYTES,
                             hipMemcpyDeviceToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    n_ -= count;
  }

  void import_units(uint64_t count, const void* dev_src) override {
    DeviceGuard dg(device_);
    ensure_cap(cur_, n_ + count, true);
    HIP_CHECK(hipMemcpyAsync(units_[cur_] + n_ * UL::WORDS, dev_src, count * UL::BYTES, hipMemcpyDeviceToDevice,
                             stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    n_ += count;
  }

  void keep_slice(uint64_t begin, uint64_t end) override {
    DeviceGuard dg(device_);
    end = std::min<uint64_t>(end, n_);
    begin = std::min(begin, end);
    if (begin > 0 && end > begin)
      HIP_CHECK(hipMemcpyAsync(units_[cur_], units_[cur_] + begin * UL::WORDS, (end - begin) * UL::BYTES,
                               hipMemcpyDeviceToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    n_ = end - begin;
  }

  void keep_strided(uint64_t offset, uint64_t stride) override {
    DeviceGuard dg(device_);
    if (stride == 0) throw Error(QI_ERR_ARG, "keep_strided: stride 0");
    // round q holds units [q*stride, (q+1)*stride); this rank's unit of round q is at
    // q*stride + (offset - q) mod stride, present while that index is < n_
    uint64_t cnt = n_ / stride;
    if (cnt * stride + (offset + stride - cnt % stride) % stride < n_) ++cnt;
    if (offset >= stride) cnt = 0;
    if (cnt) {
      ensure_cap(1 - cur_, cnt);
      const uint32_t nb = (uint32_t)std::min<uint64_t>((cnt + 255) / 256, 4096);
      launch_gather_units((uint32_t)UL::WORDS, units_[cur_], offset, stride, cnt, units_[1 - cur_], nb, stream_);
      HIP_CHECK(hipGetLastError());
      cur_ = 1 - cur_;
    }
    HIP_CHECK(hipStreamSynchronize(stream_));
    n_ = cnt;
  }

  void set_best(const std::vector<uint32_t>& key, uint32_t depth) override {
    best_key_ = key;
    best_key_.resize(MW, 0);
    best_depth_ = depth;
    has_best_ = true;
    best_dirty_ = true;
  }

  bool best(Witness* w) const override {
    if (!has_local_best_) return false;
    if (w) *w = local_best_;
    return true;
  }

  void share_best(uint64_t* host_word) override {
    DeviceGuard dg(device_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    pinned_word_free(xbest_bridge_);
    xbest_bridge_ = nullptr;
    xbest_host_ = nullptr;
    xbest_dev_ = nullptr;
    if (!host_word) return;
    if (((uintptr_t)host_word & 7u) != 0) throw Error(QI_ERR_ARG, "share_best: the word must be 8-byte aligned");
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, (void*)host_word, 0) != hipSuccess) {
      // Not HIP host memory (a shared-memory page of several processes: the driver does not
      // pin shared file mappings).  The kernels then poll a pinned word of this engine, and
      // the host carries the minimum both ways after every launch (fold_best).
      (void)hipGetLastError();
      xbest_bridge_ = pinned_word_alloc();
      HIP_CHECK(hipHostGetDevicePointer(&dp, (void*)xbest_bridge_, 0));
    }
    xbest_host_ = host_word;
    xbest_dev_ = (const unsigned long long*)dp;
  }

  Totals reduce(bool has_key, const std::vector<uint32_t>& key, uint32_t depth) override {
    // no witness: every segment counts, and the running totals are exactly those sums
    if (!has_key) return running_totals();
    DeviceGuard dg(device_);
    // the whole key (MW words): reduce_kernel compares every word of a record's key
    std::vector<uint32_t> k(dev::KEY_WORDS_MAX, 0);
    for (size_t i = 0; i < key.size() && i < (size_t)dev::KEY_WORDS_MAX; ++i) k[i] = key[i];
    HIP_CHECK(hipMemcpyAsync(keydev_, k.data(), k.size() * 4, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemsetAsync(red_, 0, 32, stream_));
    for (auto& c : log_) {
      if (!c.used) continue;
      const uint32_t nb = (uint32_t)std::min<uint64_t>((c.used + 255) / 256, (uint64_t)cus_ * 4u);
      static_assert(RL::WORDS == MW + 5, "reduce_kernel's record layout");
      launch_reduce((uint32_t)MW, c.ptr, c.used, has_key ? 1u : 0u, keydev_, depth, red_, nb, stream_);
      HIP_CHECK(hipGetLastError());
    }
    unsigned long long r[4];
    HIP_CHECK(hipMemcpyAsync(r, red_, 32, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    Totals t;
    t.nodes = r[0];
    t.evals = r[1];
    t.minq = r[2];
    t.zero_fallback = r[3];
    const Totals rt = running_totals();
    t.rounds = rt.rounds;
    t.units = rt.units;
    t.wave_iters = rt.wave_iters;
    t.coop_phases = rt.coop_phases;
    for (int q = 0; q < 8; ++q) t.dbg[q] = rt.dbg[q];
    return t;
  }

  Totals running_totals() const override {
    std::vector<unsigned long long> sh(16 * dev::TOT_SHARDS);
    if (totals_host_valid_) {  // nothing ran since the last chain end (or the last reset)
      std::memcpy(sh.data(), (const void*)totals_host_, sh.size() * 8);
    } else {
      DeviceGuard dg(device_);
      HIP_CHECK(hipMemcpyAsync(sh.data(), totals_, sh.size() * 8, hipMemcpyDeviceToHost, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
    unsigned long long r[16] = {0};
    for (int q = 0; q < dev::TOT_SHARDS; ++q)
      for (int i = 0; i < 16; ++i) r[i] += sh[(size_t)q * 16 + i];
    Totals t;
    t.nodes = r[0];
    t.evals = r[1];
    t.minq = r[2];
    t.zero_fallback = r[3];
    t.rounds = r[4];
    t.units = r[5];
    t.wave_iters = r[6];
    t.coop_phases = r[7];
    for (int q = 0; q < 8; ++q) t.dbg[q] = r[8 + q];
    return t;
  }

  void drop_log() override {
    for (auto& c : log_) c.used = 0;
    DeviceGuard dg(device_);
    HIP_CHECK(hipMemsetAsync(totals_, 0, 16 * dev::TOT_SHARDS * sizeof(unsigned long long), stream_));
    std::memset((void*)totals_host_, 0, 16 * dev::TOT_SHARDS * sizeof(unsigned long long));
    totals_host_valid_ = true;
    // no-witness best key; stream-ordered before every later launch, no host round trip
    HIP_CHECK(hipMemsetAsync(best64_, 0xFF, 8, stream_));
    HIP_CHECK(hipMemsetAsync(poll_rep_, 0xFF, (size_t)dev::POLL_REPS * 128, stream_));
    if (xbest_bridge_) __atomic_store_n(xbest_bridge_, ~0ull, __ATOMIC_RELAXED);  // a new search: no key yet
    has_best_ = false;
    has_local_best_ = false;
    sum_ms_ = 0;
    launches_ = 0;
    dispatches_ = 0;
    dispatch_ms_ = 0;
    spec_launches_ = 0;
  }

  double sum_kernel_ms() const override { return sum_ms_; }
  uint64_t launches() const override { return launches_; }
  uint64_t dispatches() const override { return dispatches_; }
  double dispatch_ms() const override { return dispatch_ms_; }
  uint64_t specialized_launches() const override { return spec_launches_; }

  bool wait_jit() override {
    if (jit_thread_.joinable()) jit_thread_.join();
    if (jit_state_.load() == 2) load_jit();
    return jit_fn_ != nullptr;
  }

 private:
  struct LogChunk {
    uint32_t* ptr = nullptr;
    uint64_t cap = 0, used = 0;
  };

  void keep(const void* p) { bufs_.push_back((void*)p); }

  // Frontier into preorder: LSD radix passes (stable) over depth, then the path-key words
  // from last to first, i.e. lexicographic (K[0], ..., K[MW-1], depth) = after_key order.
  void sort_frontier() {
    const uint64_t n = n_;
    if (n > 0xFFFFFFFFull) throw Error(QI_ERR_CAPACITY, "frontier sort: too many units");
    if (sort_cap_ < n) {
      for (auto* p : {sk_[0], sk_[1], sp_[0], sp_[1]}) (void)hipFree(p);
      (void)hipFree(stemp_);
      sort_cap_ = std::max<uint64_t>(n, 1u << 16);
      for (int i = 0; i < 2; ++i) {
        sk_[i] = dalloc<uint32_t>(sort_cap_);
        sp_[i] = dalloc<uint32_t>(sort_cap_);
      }
      stemp_bytes_ = 0;
      sort_pairs_u32(nullptr, &stemp_bytes_, sk_[0], sk_[1], sp_[0], sp_[1], (int)sort_cap_, 32, stream_);
      stemp_ = (void*)dalloc<uint8_t>(stemp_bytes_);
    }
    const uint32_t nb = (uint32_t)std::min<uint64_t>((n + 255) / 256, 65535);
    launch_iota(sp_[0], n, nb, stream_);
    for (int pass = 0; pass <= MW; ++pass) {  // pass 0: depth; pass p: K[MW - p]
      const int off = pass == 0 ? UL::DEPTH : UL::K_ + MW - pass;
      launch_unit_word(units_[cur_], (uint32_t)UL::WORDS, (uint32_t)off, sp_[0], n, sk_[0], nb, stream_);
      size_t tb = stemp_bytes_;
      sort_pairs_u32(stemp_, &tb, sk_[0], sk_[1], sp_[0], sp_[1], (int)n, pass == 0 ? 12 : 32, stream_);
      std::swap(sp_[0], sp_[1]);
    }
    ensure_cap(1 - cur_, n);
    launch_gather_perm((uint32_t)UL::WORDS, units_[cur_], sp_[0], n, units_[1 - cur_], nb, stream_);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(stream_));
    cur_ = 1 - cur_;
  }
  uint32_t* sk_[2] = {nullptr, nullptr};
  uint32_t* sp_[2] = {nullptr, nullptr};
  void* stemp_ = nullptr;
  size_t stemp_bytes_ = 0;
  uint64_t sort_cap_ = 0;
  uint64_t sorts_ = 0;
  static constexpr uint32_t kOrdSmax = 16;  // ordered kernel: stack levels per lane
  dev::OrdArgs ord_{};

  void ensure_cap(int which, uint64_t units, bool preserve = false) {
    if (cap_[which] >= units) return;
    uint64_t nc = std::max<uint64_t>(units, cap_[which] * 2);
    nc = std::max<uint64_t>(nc, 1u << 16);
    uint32_t* p = dalloc<uint32_t>(nc * UL::WORDS);
    if (preserve && units_[which] && n_)
      HIP_CHECK(hipMemcpyAsync(p, units_[which], n_ * UL::BYTES, hipMemcpyDeviceToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    (void)hipFree(units_[which]);
    units_[which] = p;
    cap_[which] = nc;
  }

  void new_log_chunk(uint64_t min_cap) {
    LogChunk c;
    c.cap = std::max<uint64_t>(min_cap, 1u << 23);
    c.cap = std::min<uint64_t>(c.cap, 0xFFFFFFF0ull);
    c.ptr = dalloc<uint32_t>(c.cap * RL::WORDS);
    c.used = 0;
    log_.push_back(c);
  }

  static bool key_less(const std::vector<uint32_t>& a, uint32_t da, const std::vector<uint32_t>& b, uint32_t db) {
    for (size_t w = 0; w < a.size(); ++w)
      if (a[w] != b[w]) return a[w] < b[w];
    return da < db;
  }

  void absorb_witness(const uint32_t* wv) {
    Witness w;
    w.key.assign(wv, wv + MW);
    w.depth = wv[MW];
    const uint32_t dl = wv[MW + 1];
    for (uint32_t v = 0; v < m_; ++v)
      if ((wv[MW + 2 + (v >> 5)] >> (v & 31)) & 1u) w.q1_local.push_back(v);
    constexpr uint32_t EPW = 4 / dev::OrdBytes<MW>::VB, EB = 32 / EPW;
    for (uint32_t i = 0; i < dl; ++i) w.q2_local.push_back((wv[2 * MW + 2 + i / EPW] >> (EB * (i % EPW))) & ((1u << EB) - 1u));
    if (!has_local_best_ || key_less(w.key, w.depth, local_best_.key, local_best_.depth)) {
      local_best_ = w;
      has_local_best_ = true;
      if (!has_best_ || key_less(w.key, w.depth, best_key_, best_depth_)) set_best(w.key, w.depth);
    }
  }

  int device_;
  SearchConfig cfg_;
  uint32_t m_;
  hipStream_t stream_{};
  hipEvent_t e0_{}, e1_{};
  dev::LocalDev d_{};
  std::vector<void*> bufs_;
  uint32_t scc_mask_[32];
  uint32_t max_blocks_ = 0;
  uint32_t cus_ = 0;
  uint32_t* units_[2] = {nullptr, nullptr};
  uint64_t cap_[2] = {0, 0};
  int cur_ = 0;
  uint64_t n_ = 0;
  uint32_t idle_steps_ = 0;    // consecutive steps without progress (guard)
  uint64_t max_frontier_bytes_ = 16ull << 30;  // both frontier buffers (QI_MAX_FRONTIER_GB)
  uint64_t pool_growths_ = 0;  // buffer doublings after a dry eviction pool
  static constexpr uint32_t kMaxBatch = 64;
  uint32_t* ctr_ = nullptr;       // [kMaxBatch + 1][CTR_WORDS]: seed block + one per launch
  uint32_t* glob_ = nullptr;      // witness count, flags
  volatile uint32_t* hctr_ = nullptr;  // pinned host: [kMaxBatch][HC_WORDS] published counters, glob mirror
  uint32_t* hctr_dev_ = nullptr;       // device view of hctr_
  volatile uint32_t* glob_host_ = nullptr;
  hipEvent_t ev_[kMaxBatch + 1] = {};
  uint64_t stops_ = 0;
  unsigned long long* totals_ = nullptr;
  unsigned long long* totals_host_ = nullptr;  // pinned snapshot of totals_ (valid: see running_totals)
  bool totals_host_valid_ = false;
  uint32_t* root_host_ = nullptr;              // pinned root unit
  bool root_ready_ = false;
  unsigned long long* best64_ = nullptr;
  uint32_t* poll_rep_ = nullptr;                    // [POLL_REPS][32]: polled best key + dry flag lines
  uint32_t* diag_waves_ = nullptr;                  // QI_DIAG_WAVES: [launches of a chain][blocks][4] timestamps
  bool diag_waves_on_ = false;
  uint32_t seq_ = 0;                                // launch sequence numbers
  uint64_t* xbest_host_ = nullptr;                  // the engines' shared best key (share_best)
  const unsigned long long* xbest_dev_ = nullptr;   // its device view
  uint64_t* xbest_bridge_ = nullptr;                // pinned copy the kernels poll when the shared
                                                    // word itself is not HIP host memory
  unsigned long long* red_ = nullptr;
  uint32_t* keydev_ = nullptr;
  uint32_t* wit_ = nullptr;
  uint32_t wit_cap_ = 0;
  std::vector<LogChunk> log_;
  size_t shm_ = 0, jit_shm_ = 0;
  int jit_smax_ = SMAX;
  bool has_best_ = false;
  std::vector<uint32_t> best_key_;
  uint32_t best_depth_ = 0;
  bool best_dirty_ = false;
  bool trace_ = false;
  uint32_t diag_prev_[2] = {0, 0};
  bool has_local_best_ = false;
  Witness local_best_;
  double sum_ms_ = 0;
  uint64_t launches_ = 0;
  uint64_t spec_launches_ = 0;
  uint64_t dispatches_ = 0;
  double dispatch_ms_ = 0;
  // run-time specialisation (qi_jit.cpp)
  LocalFlat flat_;
  std::thread jit_thread_;
  std::atomic<int> jit_state_{0};  // 0 idle, 1 compiling, 2 code ready, 3 failed, 4 loaded
  std::vector<char> jit_code_;
  std::string jit_log_;
  hipModule_t jit_mod_ = nullptr;
  hipFunction_t jit_fn_ = nullptr;

  void start_jit() {
    jit_state_.store(1);
    std::string src = jit_source(flat_, MW, TW, jit_smax_, cfg_.jit == 3, cfg_.tiebreak != 0);
    jit_thread_ = std::thread([this, src]() {
      std::vector<char> code = jit_compile(src, &jit_log_);
      jit_code_ = std::move(code);
      jit_state_.store(jit_code_.empty() ? 3 : 2);
    });
  }

  // Attributes, occupancy (and the ordered kernel's per-lane stacks) of the ahead-of-time
  // kernel; once, before its first launch.
  void aot_setup() {
    if (aot_ready_) return;
    aot_ready_ = true;
    DeviceGuard dg(device_);
    const void* kfn;
    if constexpr (ORD) kfn = (const void*)dev::ordered_kernel<MW, TW>;
    else kfn = cfg_.tiebreak ? (const void*)dev::search_kernel<MW, TW, SMAX, true> : (const void*)dev::search_kernel<MW, TW, SMAX, false>;
    if (!ORD) HIP_CHECK(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm_));
    if (!cfg_.max_blocks) {  // one resident wave of blocks: no second-wave tail
      int nb = 0;
      HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kfn, 64, shm_));
      if (ORD) nb = std::min(nb, 8);  // scratch-heavy lanes: a few waves per CU hide the latency
      if (nb > 0) aot_blocks_ = cus_ * (uint32_t)nb;
    }
    if (!jit_fn_) max_blocks_ = aot_blocks_ ? aot_blocks_ : max_blocks_;
    if (ORD) {  // one DFS stack (and, beyond 256 vertices, one workspace) per lane of a launch
      keep(ord_.ostack = dalloc<uint32_t>((size_t)max_blocks_ * kOrdSmax * (dev::OrdUnitLayout<MW>::OWT + 3) * 64));
      if (dev::OrdWorkspace<MW>::GLOBAL)
        keep(ord_.ows = dalloc<uint8_t>((size_t)max_blocks_ * 64 * dev::OrdWorkspace<MW>::BYTES));
    }
  }
  bool aot_ready_ = false;
  uint32_t aot_blocks_ = 0;

  void load_jit() {
    if (jit_state_.load() != 2) return;
    if (jit_thread_.joinable()) jit_thread_.join();
    DeviceGuard dg(device_);
    if (hipModuleLoadData(&jit_mod_, jit_code_.data()) != hipSuccess ||
        hipModuleGetFunction(&jit_fn_, jit_mod_, "qi_search_spec") != hipSuccess) {
      jit_fn_ = nullptr;
      jit_state_.store(3);
      return;
    }
    jit_state_.store(4);
    if (!cfg_.max_blocks) {
      int nb = 0;
      if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, jit_fn_, 64, jit_shm_) == hipSuccess && nb > 0) {
        if (const char* e = std::getenv("QI_JIT_WAVES")) nb = std::max(1, std::min(nb, std::atoi(e)));  // diagnostics
        max_blocks_ = cus_ * (uint32_t)nb;
      }
    }
  }
};

}  // namespace

// One search engine shape; explicitly instantiated by the part that owns its group.
template <int MW, int TW, int SMAX, bool ORD>
std::unique_ptr<SearchDevice> make_engine(int device, const LocalFlat& f, const SearchConfig& cfg) {
  return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<MW, TW, SMAX, ORD>(device, f, cfg));
}
// (the one-word shape, the usual one for a real network's searched SCC, has a part -- a code
// object -- of its own: the first run on a network loads only that, ~1 ms instead of 4-6)
#define QI_ENGINES_5(X) X(1, 1, 24, false)
#define QI_ENGINES_1(X) X(1, 2, 24, false) X(1, 4, 24, false) X(2, 2, 16, false) X(2, 4, 16, false)
#define QI_ENGINES_2(X) X(4, 4, 12, false) X(4, 8, 12, false) X(8, 8, 8, false)
#define QI_ENGINES_3(X) X(1, 1, 24, true) X(1, 4, 24, true) X(2, 4, 16, true) X(4, 8, 12, true)
#define QI_ENGINES_4(X) X(8, 8, 8, true) X(16, 16, 8, true) X(32, 32, 8, true)
#define QI_ENGINE_DEF(MW, TW, S, O) \
  template std::unique_ptr<SearchDevice> make_engine<MW, TW, S, O>(int, const LocalFlat&, const SearchConfig&);
#define QI_ENGINE_EXT(MW, TW, S, O) \
  extern template std::unique_ptr<SearchDevice> make_engine<MW, TW, S, O>(int, const LocalFlat&, const SearchConfig&);
#if QI_PART == 0
QI_ENGINES_1(QI_ENGINE_EXT)
QI_ENGINES_2(QI_ENGINE_EXT)
QI_ENGINES_3(QI_ENGINE_EXT)
QI_ENGINES_4(QI_ENGINE_EXT)
QI_ENGINES_5(QI_ENGINE_EXT)
#elif QI_PART == 1
QI_ENGINES_1(QI_ENGINE_DEF)
#elif QI_PART == 2
QI_ENGINES_2(QI_ENGINE_DEF)
#elif QI_PART == 3
QI_ENGINES_3(QI_ENGINE_DEF)
#elif QI_PART == 4
QI_ENGINES_4(QI_ENGINE_DEF)
#elif QI_PART == 5
QI_ENGINES_5(QI_ENGINE_DEF)
#endif

#if QI_PART <= 0
// The ordered kernel's emulation of libstdc++ unordered_set iteration order, run on the
// host (tests compare it with the real container): keys[v] = global index of local
// vertex v; the table is built by inserting seq[0..n_seq) in order (repeats ignored).
uint32_t hash_iteration_order(const uint32_t* keys, uint32_t n_keys, const uint32_t* seq, uint32_t n_seq,
                              uint32_t* out) {
  if (n_keys > 1024) throw Error(QI_ERR_ARG, "hash order: more than 1024 keys");
  auto* hl = new dev::HashList<1024, 1109>;
  hl->clear();
  std::vector<uint8_t> seen(n_keys, 0);
  auto bmod = [&](uint32_t v, int r) -> uint32_t { return keys[v] % dev::kHashBuckets[r]; };
  for (uint32_t i = 0; i < n_seq; ++i) {
    const uint32_t v = seq[i];
    if (v >= n_keys) {
      delete hl;
      throw Error(QI_ERR_ARG, "hash order: vertex out of range");
    }
    if (seen[v]) continue;
    seen[v] = 1;
    hl->insert((uint16_t)v, bmod);
  }
  uint32_t n = 0;
  for (uint16_t v = hl->head; v != dev::HashList<1024, 1109>::NIL; v = hl->nxt[v]) out[n++] = v;
  delete hl;
  return n;
}


void device_prepare(int device) {
  DeviceGuard dg(device);
  // the stream (hardware queue) that the per-SCC checks and the search engine of a solve
  // take in turn is created here, with the device, not inside the first solve
  release_stream(device, acquire_stream(device));
  size_t cap = 0;
  unsigned long long* st = acquire_stage(kStageMin, &cap);  // the per-SCC checker's pinned staging buffer
  release_stage(st, cap);
  (void)static_scratch_ptr(device);
}

std::unique_ptr<GfpDevice> make_gfp_device(int device, const GlobalFlat& g) {
  if (const char* e = std::getenv("QI_GFP_LDS")) GfpDeviceImpl::kLdsImage = (size_t)std::atoll(e);
  return std::unique_ptr<GfpDevice>(new GfpDeviceImpl(device, g));
}

bool jit_precompile(const LocalFlat& f, std::string* log) {
  const uint32_t mw = f.mw, tw = f.tw;
  int MW, TW, SMAX;
  if (mw <= 1 && tw <= 1) { MW = 1; TW = 1; SMAX = 24; }
  else if (mw <= 1 && tw <= 2) { MW = 1; TW = 2; SMAX = 24; }
  else if (mw <= 1 && tw <= 4) { MW = 1; TW = 4; SMAX = 24; }
  else if (mw <= 2 && tw <= 2) { MW = 2; TW = 2; SMAX = 16; }
  else if (mw <= 2 && tw <= 4) { MW = 2; TW = 4; SMAX = 16; }
  else if (mw <= 4 && tw <= 4) { MW = 4; TW = 4; SMAX = 12; }
  else if (mw <= 4 && tw <= 8) { MW = 4; TW = 8; SMAX = 12; }
  else if (mw <= 8 && tw <= 8) { MW = 8; TW = 8; SMAX = 8; }
  else return false;
  if (!jit_eligible(f)) return false;
  return !jit_compile(jit_source(f, MW, TW, jit_default_smax(MW, SMAX), false), log).empty();
}

std::unique_ptr<SearchDevice> make_search_device(int device, const LocalFlat& f, const SearchConfig& cfg) {
  const uint32_t mw = f.mw, tw = f.tw;
  // threshold-0 quorum sets: the order-exact kernel (QI_ORDERED=1 forces it, diagnostics);
  // |SCC| or the TN count beyond 256: the order-exact kernel too (exact for monotone SCCs
  // as well), with 16-bit order lists
  const char* fo = std::getenv("QI_ORDERED");
  const bool ordered = f.nonmonotone || (fo && std::atoi(fo) != 0) || mw > 8 || tw > 8;
  if (ordered) {
    if (mw <= 1 && tw <= 1) return make_engine<1, 1, 24, true>(device, f, cfg);
    if (mw <= 1 && tw <= 4) return make_engine<1, 4, 24, true>(device, f, cfg);
    if (mw <= 2 && tw <= 4) return make_engine<2, 4, 16, true>(device, f, cfg);
    if (mw <= 4 && tw <= 8) return make_engine<4, 8, 12, true>(device, f, cfg);
    if (mw <= 8 && tw <= 8) return make_engine<8, 8, 8, true>(device, f, cfg);
    if (mw <= 16 && tw <= 16) return make_engine<16, 16, 8, true>(device, f, cfg);
    if (mw <= 32 && tw <= 32) return make_engine<32, 32, 8, true>(device, f, cfg);
    throw Error(QI_ERR_UNSUPPORTED, "searched SCC too large for the device kernels (|SCC| > 1024 or > 1024 TNs)");
  }
  if (mw <= 1 && tw <= 1) return make_engine<1, 1, 24, false>(device, f, cfg);
  if (mw <= 1 && tw <= 2) return make_engine<1, 2, 24, false>(device, f, cfg);
  if (mw <= 1 && tw <= 4) return make_engine<1, 4, 24, false>(device, f, cfg);
  if (mw <= 2 && tw <= 2) return make_engine<2, 2, 16, false>(device, f, cfg);
  if (mw <= 2 && tw <= 4) return make_engine<2, 4, 16, false>(device, f, cfg);
  if (mw <= 4 && tw <= 4) return make_engine<4, 4, 12, false>(device, f, cfg);
  if (mw <= 4 && tw <= 8) return make_engine<4, 8, 12, false>(device, f, cfg);
  return make_engine<8, 8, 8, false>(device, f, cfg);
}

#endif  // QI_PART <= 0

}  // namespace qi
