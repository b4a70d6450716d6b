// =====================================================================================
//  qi_search_kernel.h -- device code of the branch-and-bound search (gfx950).
//
//  Self-contained so that the same source is compiled twice:
//   * ahead of time by hipcc (qi_device.hip) with the table-interpreting evaluator
//     TableEval for every FBAS shape, and
//   * at run time by hipRTC (qi_jit.cpp) with an evaluator generated for one flattened
//     FBAS (literal masks and thresholds, no table loads).
//  Frontier units, segment records and witnesses have identical layouts in both, so the
//  engine can switch kernels at any launch boundary.
// =====================================================================================
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <cstdint>
#else
using __hip_internal::int32_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
using __hip_internal::uint8_t;
#endif

namespace qi {
namespace dev {

constexpr int WAVE = 64;

// ------------------------------------------------------------------------------------
// SCC-local TN table (see LocalFlat in qi_internal.h)
// ------------------------------------------------------------------------------------
// One packed record per threshold node, read with a single wide scalar load:
//   [0, MW) validator mask (plane 0) | [MW, MW+TW) child mask (plane 0) |
//   thr (outside unavailable) | thr (outside available) | invert | has-extra-planes
// "invert" encodes threshold 0 ("first entry unavailable"): thr = 1 and the test is
// flipped, so sat = (count >= thr) XOR invert without a branch.
template <int MW, int TW>
struct TnRec {
  static constexpr int RAW = MW + TW + 4;
  static constexpr int WORDS = RAW <= 8 ? 8 : (RAW <= 16 ? 16 : 32);
  static constexpr int THR0 = MW + TW, THR1 = MW + TW + 1, INV = MW + TW + 2, EXTRA = MW + TW + 3;
};

struct LocalDev {
  const uint32_t* tn;          // [T][TnRec::WORDS]
  const uint32_t* extra_off;   // [T+1]
  const uint32_t* extra_src;
  const uint32_t* extra_mask;
  const uint32_t* root_tn;     // [R]
  const uint32_t* root_users;  // [R][MW]
  const uint32_t* grp_members; // [G][MW]
  const uint32_t* grp_col;     // [G][MW]
  const uint32_t* grp_extra_off;  // [G+1]
  const uint32_t* grp_extra;      // [E][MW]
  uint32_t T, R, G, m;
};

// Wave-uniform tables are read through the constant address space so the compiler emits
// scalar loads (s_load into SGPRs, consumed directly by v_and/v_bcnt) instead of vector
// loads with a uniform address (SQ_INSTS_VMEM dominated the first profile, r01).
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* K(const T* p) {
  return (const __attribute__((address_space(4))) T*)p;
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t rank_in(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint32_t bcast0(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

template <int MW, int TW>
__device__ __forceinline__ uint32_t extra_terms(const LocalDev& f, uint32_t t, const uint32_t (&X)[MW],
                                                const uint32_t (&sb)[TW]) {
  uint32_t c = 0;
  const uint32_t e0 = K(f.extra_off)[t], e1 = K(f.extra_off)[t + 1];
  for (uint32_t e = e0; e < e1; ++e) {
    const uint32_t src = K(f.extra_src)[e], msk = K(f.extra_mask)[e];
    uint32_t word = 0;
#pragma unroll
    for (int w = 0; w < MW; ++w) word = (src == (uint32_t)w) ? X[w] : word;
#pragma unroll
    for (int w = 0; w < TW; ++w) word = (src == (uint32_t)(MW + w)) ? sb[w] : word;
    c += __popc(word & msk);
  }
  return c;
}

// containsQuorum (cpp:140-177) as a Jacobi greatest fixpoint on one lane's masks.
// X: in = candidate set (nodes ∩ avail within the SCC), out = survivors.
// POL 0 = vertices outside the SCC unavailable (cpp:281/184/192/301/658),
//     1 = available (visitor, cpp:354/368), 2 = per-lane `pol` (cooperative phase).
// Same set as the reference's Gauss-Seidel sweep for monotone slices (every quorum set
// has threshold >= 1); threshold-0 inputs are flagged nonmonotone by the host.
template <int MW, int TW, int POL>
__device__ __forceinline__ bool gfp(const LocalDev& f, uint32_t (&X)[MW], uint32_t pol, uint32_t& rounds) {
  using R = TnRec<MW, TW>;
  for (;;) {
    uint32_t any = 0;
#pragma unroll
    for (int w = 0; w < MW; ++w) any |= X[w];
    if (!any) return false;
    ++rounds;
    uint32_t sb[TW];
#pragma unroll
    for (int w = 0; w < TW; ++w) sb[w] = 0;
#pragma unroll
    for (int tw = 0; tw < TW; ++tw) {
      const uint32_t tb = (uint32_t)tw * 32u;
      const uint32_t te = min(f.T, tb + 32u);
      const __attribute__((address_space(4))) uint32_t* rec = K(f.tn) + (size_t)tb * R::WORDS;
#pragma unroll 4
      for (uint32_t t = tb; t < te; ++t, rec += R::WORDS) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < MW; ++w) c += __popc(X[w] & rec[w]);
#pragma unroll
        for (int w = 0; w <= tw; ++w) c += __popc(sb[w] & rec[MW + w]);
        if (rec[R::EXTRA]) c += extra_terms<MW, TW>(f, t, X, sb);  // multiplicity > 1 (rare)
        int32_t th;
        if (POL == 0) th = (int32_t)rec[R::THR0];
        else if (POL == 1) th = (int32_t)rec[R::THR1];
        else th = pol ? (int32_t)rec[R::THR1] : (int32_t)rec[R::THR0];
        const uint32_t bit = (((int32_t)c >= th) ? 1u : 0u) ^ rec[R::INV];
        sb[tw] |= bit << (t - tb);
      }
    }
    uint32_t Xn[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) Xn[w] = 0;
    for (uint32_t r = 0; r < f.R; ++r) {
      const uint32_t tn = K(f.root_tn)[r];
      uint32_t word = sb[0];
#pragma unroll
      for (int w = 1; w < TW; ++w) word = ((tn >> 5) == (uint32_t)w) ? sb[w] : word;
      const uint32_t sel = 0u - ((word >> (tn & 31u)) & 1u);
#pragma unroll
      for (int w = 0; w < MW; ++w) Xn[w] |= K(f.root_users)[r * MW + w] & sel;
    }
    bool same = true;
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      Xn[w] &= X[w];
      same &= (Xn[w] == X[w]);
    }
    if (same) return true;
#pragma unroll
    for (int w = 0; w < MW; ++w) X[w] = Xn[w];
  }
}

// findBestNode (cpp:203-250): argmax over w in Q\D of indeg_Q(w) = Σ_{v∈Q} mult(v→w),
// ties -> lowest vertex index (one of the reference's uniformly-random outcomes).
// Vertices with identical in-edge columns form one group (one popcount per group).
template <int MW>
__device__ __forceinline__ uint32_t best_node(const LocalDev& f, const uint32_t (&Q)[MW], const uint32_t (&D)[MW],
                                              uint32_t& zero_fallback) {
  uint32_t bestdeg = 0, bestv = 0xFFFFFFFFu;
  for (uint32_t g = 0; g < f.G; ++g) {
    uint32_t deg = 0, low = 0xFFFFFFFFu;
#pragma unroll
    for (int w = 0; w < MW; ++w) deg += __popc(Q[w] & K(f.grp_col)[g * MW + w]);
    const uint32_t e0 = K(f.grp_extra_off)[g], e1 = K(f.grp_extra_off)[g + 1];
    for (uint32_t e = e0; e < e1; ++e) {
#pragma unroll
      for (int w = 0; w < MW; ++w) deg += __popc(Q[w] & K(f.grp_extra)[e * MW + w]);
    }
#pragma unroll
    for (int w = MW - 1; w >= 0; --w) {
      const uint32_t c = Q[w] & ~D[w] & K(f.grp_members)[g * MW + w];
      low = c ? (uint32_t)w * 32u + (uint32_t)__builtin_ctz(c) : low;
    }
    const bool better = (low != 0xFFFFFFFFu) && (deg > bestdeg || (deg == bestdeg && low < bestv));
    bestdeg = better ? deg : bestdeg;
    bestv = better ? low : bestv;
  }
  zero_fallback += (bestdeg == 0u) ? 1u : 0u;
  return bestv;
}

// The generic evaluator: interprets the packed TN table (any FBAS shape).  A runtime-
// specialised evaluator with the same interface is generated per FBAS (qi_jit.cpp).
template <int MW, int TW>
struct TableEval {
  template <int POL>
  static __device__ __forceinline__ bool gfp(const LocalDev& f, uint32_t (&X)[MW], uint32_t pol, uint32_t& rounds) {
    return dev::gfp<MW, TW, POL>(f, X, pol, rounds);
  }
  static __device__ __forceinline__ uint32_t best(const LocalDev& f, const uint32_t (&Q)[MW], const uint32_t (&D)[MW],
                                                  uint32_t& zero_fallback) {
    return dev::best_node<MW>(f, Q, D, zero_fallback);
  }
};

// ------------------------------------------------------------------------------------
// Frontier unit / log record layouts
// ------------------------------------------------------------------------------------
template <int MW>
struct UnitLayout {
  static constexpr int DMAX = MW * 16 + 1;  // |D| <= m/2 + 1 for every unit
  static constexpr int RAW = MW * 12 + 8 + DMAX;
  static constexpr int BYTES = (RAW + 15) / 16 * 16;
  static constexpr int WORDS = BYTES / 4;
  // word offsets
  static constexpr int T_ = 0, D_ = MW, K_ = 2 * MW, DEPTH = 3 * MW, DLEN = 3 * MW + 1, ORD = 3 * MW + 2;
};
// record: key[MW], depth, count, evals, minq, zero_fallback
template <int MW>
struct RecLayout {
  static constexpr int WORDS = MW + 5;
};
// witness: key[MW], depth, dlen, q1[MW], order bytes
template <int MW>
struct WitLayout {
  static constexpr int ORDW = (UnitLayout<MW>::DMAX + 3) / 4;
  static constexpr int WORDS = 2 * MW + 2 + ORDW;
};

// Per-launch counter block (CTR_WORDS words).  Launches are chained on the device: launch
// k reads its input count, log position and stop state from launch k-1's block (or from a
// host-written seed block), so the host enqueues launches without reading anything back
// in between.  The atomically updated words and the plainly written ones sit on separate
// 128-B lines.  The last block of a launch carries never-claimed input units over and
// publishes the final block to pinned host memory (HC_* words), where the host polls it.
enum : int {
  C_OUT = 0,       // units written to units_out (spills + carried-over units)   [atomic]
  C_HEAD = 1,      // dynamic claims past the statically assigned range           [atomic]
  C_DONE = 2,      // used blocks that finished                                   [atomic]
  C_NIN = 32,      // input units of this launch (the previous block's C_OUT)
  C_LOGB = 33,     // first segment-log record of this launch
  C_STOP = 34,     // 1: capacity would be exceeded; this launch (and the rest of the chain) did nothing
  C_STATIC = 35,   // end of the statically assigned range (64 units per used block)
  CTR_WORDS = 64,
  HC_OUT = 0, HC_NIN = 1, HC_LOGB = 2, HC_STOP = 3, HC_DONE = 4, HC_WORDS = 8
};
constexpr int TOT_SHARDS = 64;  // running totals: [TOT_SHARDS][16] u64, shard = block % 64

struct SearchArgs {
  LocalDev f;
  const uint32_t* units_in;
  uint32_t* units_out;
  uint32_t out_cap;
  uint32_t log_cap;              // records in the current log chunk
  const uint32_t* prev;          // previous launch's counter block (or the seed block)
  uint32_t* counters;            // this launch's counter block
  uint32_t* host_ctr;            // pinned host words HC_* for this launch (device pointer)
  uint32_t* glob;                // [0] witness count [1] flags (whole batch)
  uint32_t* records;             // log chunk base; this launch writes from prev's C_LOGB + C_NIN
  uint32_t* wit;
  uint32_t wit_cap;
  unsigned long long* totals;    // [TOT_SHARDS][16]: nodes, evals, minq, zero_fallback, rounds, units, ...
  unsigned long long* best64;    // device-side best witness, best_pack(): exact when MW == 1,
                                 // the first 64 path bits (conservative pruning) otherwise
  uint32_t grow_budget;          // per-lane node budget while the frontier is below half the lanes
  uint32_t run_budget;
  uint32_t grace;                // extra steps per lane once the unit queue is dry
  uint32_t evict_max;
  uint32_t half_m;
  uint32_t coop_slot;            // lanes per pending owner in the cooperative phase (pow2)
  uint32_t coop_slot_log2;
  uint32_t has_best;             // host-known best key (multiword) for pruning
  uint32_t best_depth;
  uint32_t best_key[8];
  uint32_t scc_mask[8];
};

enum : uint32_t { FLAG_OUT_OVERFLOW = 1u, FLAG_WIT_OVERFLOW = 2u };

// 64-bit preorder summary of a node (path key K, depth d) for the device-side best key:
// MW == 1: (K0, d) -- exact order; MW > 1: (K0, K1) -- "strictly greater" still implies
// "strictly after in preorder", equal values are never pruned.
template <int MW>
__device__ __forceinline__ uint64_t best_pack(const uint32_t (&K)[MW], uint32_t d) {
  if constexpr (MW == 1) return ((uint64_t)K[0] << 32) | d;
  else return ((uint64_t)K[0] << 32) | K[1];
}

// preorder "strictly after" test of (K, d) vs (B, db): padded path bits, then depth.
template <int MW>
__device__ __forceinline__ bool after_key(const uint32_t (&K)[MW], uint32_t d, const uint32_t* B, uint32_t db) {
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    if (K[w] != B[w]) return K[w] > B[w];
  }
  return d > db;
}

template <int MW>
__device__ __forceinline__ void key_prefix_bit(uint32_t (&K)[MW], uint32_t de) {
  // keep path positions < de, then set position de (inclusion branch at depth de)
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    const uint32_t lo = (uint32_t)w * 32u;
    uint32_t keep;
    if (de >= lo + 32u) keep = 0xFFFFFFFFu;
    else if (de <= lo) keep = 0u;
    else keep = 0xFFFFFFFFu << (32u - (de - lo));
    K[w] &= keep;
    if ((de >> 5) == (uint32_t)w) K[w] |= 0x80000000u >> (de & 31u);
  }
}

// Wave-aggregated reservation of n (per lane) slots on a global counter.
__device__ __forceinline__ uint32_t reserve(uint32_t n, uint32_t* counter, uint32_t& total_out) {
  const uint32_t lane = lane_id();
  uint32_t x = n;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if ((int)lane >= d) x += y;
  }
  const uint32_t total = __shfl(x, WAVE - 1);
  uint32_t base = 0;
  if (lane == 0 && total) base = atomicAdd(counter, total);
  base = __shfl(base, 0);
  total_out = total;
  return base + x - n;
}

// Diagnostic build only (QI_STAMPS, run-time specialised kernel with jit=3): per-wave
// s_memtime sums of the loop sections, added into totals[8..15].  The production kernels
// contain no stamps (MI355X guide §7 "In-kernel stamps": read shares, not lengths).
#ifdef QI_STAMPS
#define QI_STAMP(slot)                                                   \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();                  \
    __builtin_amdgcn_sched_barrier(0);                                   \
    stamp_sum[(slot)] += now_ - stamp_prev;                              \
    stamp_prev = now_;                                                   \
  } while (0)
#else
#define QI_STAMP(slot) \
  do {                 \
  } while (0)
#endif

template <int MW, int TW, int SMAX, class EV>
__device__ __forceinline__ void search_body(const SearchArgs& a) {
  using UL = UnitLayout<MW>;
  using RL = RecLayout<MW>;
  using WL = WitLayout<MW>;
  constexpr int DMAX = UL::DMAX;
  constexpr int UW = UL::WORDS;
  constexpr int SE = MW + 1;  // stack entry words: T'[MW], packed(b, depth, dlen)

  constexpr int OW = (DMAX + 3) / 4;  // packed D-order words (4 vertex bytes each)
  (void)OW;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* st = lds;                                          // [SMAX][SE][64]
  uint32_t* co_NE = st + SMAX * SE * WAVE;                      // [MW][64] per pending rank
  uint32_t* co_VIS = co_NE + MW * WAVE;                         // [MW][64] per pending rank
  uint32_t* uring = co_VIS + MW * WAVE;                         // [UW][64] staged units
  uint32_t* dow = uring + UW * WAVE;                            // [OW][64] D in branch order

  const uint32_t lane = threadIdx.x;
  const LocalDev& f = a.f;
  // ---- chained launch prologue: input count, log position, capacity (wave-uniform) ----
  const uint32_t* pc = a.prev;
  uint32_t* cc = a.counters;
  if (pc[C_STOP]) {  // an earlier launch of this chain stopped: the frontier stays where it is
    if (blockIdx.x == 0 && lane == 0) {
      cc[C_STOP] = 1u;
      a.host_ctr[HC_STOP] = 1u;
      a.host_ctr[HC_DONE] = 1u;
    }
    return;
  }
  const uint32_t n_in = pc[C_OUT];
  const uint32_t log_base = pc[C_LOGB] + pc[C_NIN];
  const uint32_t nb_used = min((n_in + (uint32_t)WAVE - 1u) / (uint32_t)WAVE, gridDim.x);
  const uint32_t static_end = min(n_in, nb_used * (uint32_t)WAVE);
  {
    const uint64_t need_out = (uint64_t)n_in + (uint64_t)nb_used * WAVE * (uint64_t)(SMAX + 1 + a.evict_max);
    const bool stop = need_out > (uint64_t)a.out_cap || (uint64_t)log_base + n_in > (uint64_t)a.log_cap;
    if (blockIdx.x == 0 && lane == 0) {
      cc[C_NIN] = n_in;
      cc[C_LOGB] = log_base;
      cc[C_STATIC] = static_end;
      cc[C_STOP] = stop ? 1u : 0u;
      if (stop || nb_used == 0) {  // nothing runs: publish now (else the last block does)
        a.host_ctr[HC_OUT] = 0u;
        a.host_ctr[HC_NIN] = n_in;
        a.host_ctr[HC_LOGB] = log_base;
        a.host_ctr[HC_STOP] = stop ? 1u : 0u;
        a.host_ctr[HC_DONE] = 1u;
      }
    }
    if (stop || blockIdx.x >= nb_used) return;
  }
  uint32_t* const records = a.records + (size_t)log_base * RL::WORDS;
  const uint32_t budget = (n_in >= gridDim.x * (uint32_t)WAVE / 2u) ? a.run_budget : a.grow_budget;
#define ST_(lvl, w) st[((lvl) * SE + (w)) * WAVE + lane]
#define DOW_(w) dow[(w) * WAVE + lane]
#define UR_(w, slot) uring[(w) * WAVE + (slot)]
  // byte i of this lane's D order (ds_write_b8 into the packed word)
  auto set_ord = [&](uint32_t i, uint32_t v) {
    ((uint8_t*)dow)[(((i >> 2) * WAVE + lane) << 2) + (i & 3u)] = (uint8_t)v;
  };

  uint32_t T[MW], D[MW], K[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) T[w] = D[w] = K[w] = 0;
  uint32_t depth = 0, dlen = 0;
  bool has = false, done = false;
  uint32_t nst = 0, sbase = 0;
  uint32_t steps = 0, evictions = 0;
  uint32_t limit = budget;  // per-lane step limit; shrinks to steps+grace when the queue dries
  bool dry = false;
  uint32_t iter = 0;
  // current segment (one per fetched unit)
  bool seg_open = false;
  uint32_t seg_idx = 0, seg_depth = 0, seg_count = 0, seg_evals = 0, seg_minq = 0, seg_zfb = 0;
  uint32_t seg_K[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) seg_K[w] = 0;
  uint64_t tot_nodes = 0, tot_evals = 0, tot_minq = 0, tot_zfb = 0, tot_fetched = 0;
  uint32_t rounds = 0;
  uint32_t wave_iters = 0, coop_phases = 0;  // wave-uniform: occupancy accounting
#ifdef QI_STAMPS
  uint64_t stamp_sum[6] = {0, 0, 0, 0, 0, 0};
  uint64_t stamp_prev = __builtin_amdgcn_s_memtime();
#endif

  // wave-uniform LDS ring of staged units (see (2) below)
  uint32_t ring_src = 0, ring_cnt = 0, ring_next = 0;
  bool ring_dead = false;
  uint64_t best64 = ~0ull;
  auto refill = [&](uint32_t base) {  // convergent: every lane stages one unit
    const uint32_t cnt = min(n_in - base, (uint32_t)WAVE);
    if (lane < cnt) {
      const uint4* src = (const uint4*)(a.units_in + (size_t)(base + lane) * UW);
#pragma unroll
      for (int q = 0; q < UW / 4; ++q) {
        const uint4 v = src[q];
        UR_(4 * q + 0, lane) = v.x;
        UR_(4 * q + 1, lane) = v.y;
        UR_(4 * q + 2, lane) = v.z;
        UR_(4 * q + 3, lane) = v.w;
      }
    }
    __syncthreads();
    ring_src = base;
    ring_cnt = cnt;
    ring_next = 0;
  };
  // the first 64 units of this block's range are statically assigned (no atomic)
  if (blockIdx.x * WAVE < n_in) refill(blockIdx.x * WAVE);
  else ring_dead = true;

  auto close_segment = [&]() {
    uint32_t* r = records + (size_t)seg_idx * RL::WORDS;
#pragma unroll
    for (int w = 0; w < MW; ++w) r[w] = seg_K[w];
    r[MW] = seg_depth;
    r[MW + 1] = seg_count;
    r[MW + 2] = seg_evals;
    r[MW + 3] = seg_minq;
    r[MW + 4] = seg_zfb;
    tot_nodes += seg_count;
    tot_evals += seg_evals;
    tot_minq += seg_minq;
    tot_zfb += seg_zfb;
    seg_open = false;
  };

  auto pruned = [&](const uint32_t (&KK)[MW], uint32_t d) -> bool {
    bool p = false;
    if (a.has_best) p = after_key<MW>(KK, d, a.best_key, a.best_depth);
    p = p || (best_pack<MW>(KK, d) > best64);
    return p;
  };

  // write one unit (T, D given as masks, order = dord[0..ol) + optional extra byte)
  auto write_unit = [&](uint32_t slot, const uint32_t (&UT)[MW], const uint32_t (&UD)[MW], const uint32_t (&UK)[MW],
                        uint32_t udepth, uint32_t ol, int extra_b) {
    if (slot >= a.out_cap) {
      atomicOr(&a.glob[1], FLAG_OUT_OVERFLOW);
      return;
    }
    uint32_t* u = a.units_out + (size_t)slot * UW;
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      u[UL::T_ + w] = UT[w];
      u[UL::D_ + w] = UD[w];
      u[UL::K_ + w] = UK[w];
    }
    const uint32_t ulen = ol + (extra_b >= 0 ? 1u : 0u);
    u[UL::DEPTH] = udepth;
    u[UL::DLEN] = ulen;
    for (uint32_t i = 0; i < (ulen + 3) / 4; ++i) {  // bytes >= ulen are don't-care
      uint32_t word = DOW_(i);
      if (extra_b >= 0 && i == (ol >> 2)) {
        const uint32_t sh = 8u * (ol & 3u);
        word = (word & ~(0xFFu << sh)) | ((uint32_t)extra_b << sh);
      }
      u[UL::ORD + i] = word;
    }
  };

  // write stack entry at circular position pos as a unit
  auto write_entry = [&](uint32_t slot, uint32_t pos) {
    uint32_t UT[MW], UD[MW], UK[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      UT[w] = ST_(pos, w);
      UD[w] = 0;
      UK[w] = K[w];
    }
    const uint32_t pk = ST_(pos, MW);
    const uint32_t b = pk & 255u, de = (pk >> 8) & 511u, dle = pk >> 17;
    for (uint32_t i = 0; i < (dle + 3) / 4; ++i) {
      const uint32_t word = DOW_(i);
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j)
        if (i * 4 + j < dle) {
          const uint32_t v = (word >> (8 * j)) & 255u;
          UD[v >> 5] |= 1u << (v & 31u);
        }
    }
    UD[b >> 5] |= 1u << (b & 31u);
    key_prefix_bit<MW>(UK, de);
    write_unit(slot, UT, UD, UK, de + 1, dle, (int)b);
  };

  for (;;) {
    // ---- (1) continue the current unit from its stack -------------------------------
    if (!done && !has) {
      while (nst > 0) {
        --nst;
        const uint32_t pos = (sbase + nst) & (SMAX - 1);
        const uint32_t pk = ST_(pos, MW);
        const uint32_t b = pk & 255u, de = (pk >> 8) & 511u, dle = pk >> 17;
        uint32_t NK[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) NK[w] = K[w];
        key_prefix_bit<MW>(NK, de);
        if (pruned(NK, de + 1)) {  // deeper entries precede shallower ones: drop all
          nst = 0;
          break;
        }
        for (uint32_t i = dle >> 2; i < (dlen + 3) / 4; ++i) {  // drop inclusions below `de`
          const uint32_t word = DOW_(i);
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t p = i * 4 + j;
            if (p >= dle && p < dlen) {
              const uint32_t v = (word >> (8 * j)) & 255u;
              D[v >> 5] &= ~(1u << (v & 31u));
            }
          }
        }
        D[b >> 5] |= 1u << (b & 31u);
        set_ord(dle, b);
        dlen = dle + 1;
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          T[w] = ST_(pos, w);
          K[w] = NK[w];
        }
        depth = de + 1;
        has = true;
        break;
      }
      if (!has && nst == 0) {
        if (seg_open) close_segment();
        if (steps >= limit) done = true;
      }
    }

    QI_STAMP(0);  // pop / segment close
    // ---- (2) fetch new units from the wave's LDS ring --------------------------------
    // The ring holds up to 64 units staged by one coalesced refill (one atomic on the
    // global head + one unit per lane), so the global-load latency is paid once per 64
    // fetches instead of on every fetch.
    bool need = !done && !has;
    uint64_t nm = __ballot(need);
    while (nm) {
      if (ring_next >= ring_cnt) {
        if (ring_dead) break;
        uint32_t base = 0;
        if (lane == 0) base = static_end + atomicAdd(&cc[C_HEAD], (uint32_t)WAVE);
        base = __shfl(base, 0);
        if (base >= n_in) {
          ring_dead = true;
          break;
        }
        refill(base);
      }
      const uint32_t avail = ring_cnt - ring_next;
      const uint32_t r = rank_in(nm);
      if (need && r < avail) {
        const uint32_t slot = ring_next + r;
        uint32_t UK[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          T[w] = UR_(UL::T_ + w, slot);
          D[w] = UR_(UL::D_ + w, slot);
          UK[w] = UR_(UL::K_ + w, slot);
        }
        const uint32_t ud = UR_(UL::DEPTH, slot);
        dlen = UR_(UL::DLEN, slot);
        for (uint32_t i = 0; i < (dlen + 3) / 4; ++i) DOW_(i) = UR_(UL::ORD + i, slot);
        ++tot_fetched;
        seg_idx = ring_src + slot;
        seg_open = true;
        seg_count = seg_evals = seg_minq = seg_zfb = 0;
#pragma unroll
        for (int w = 0; w < MW; ++w) seg_K[w] = K[w] = UK[w];
        seg_depth = depth = ud;
        nst = 0;
        sbase = 0;
        need = false;
        if (pruned(UK, ud)) close_segment();  // zero record
        else has = true;
      }
      ring_next += min((uint32_t)__popcll(nm), avail);
      nm = __ballot(need);
    }
    if (ring_dead && need) done = true;
    if (!__any(has)) break;

    // Every 32 iterations poll the global head and the device-side best key (one
    // blocking global load pair, kept off the per-iteration path).  Once no unit is left
    // to fetch anywhere, every lane gets a short grace period and then spills: the next
    // launch spreads the remaining subtrees over all lanes instead of letting a few lanes
    // grind through deep subtrees while the rest idle.
    if ((iter++ & 31u) == 0u || (ring_dead && !dry)) {
      uint32_t h = 0;
      uint64_t b = ~0ull;
      if (lane == 0) {
        h = static_end + __hip_atomic_load(&cc[C_HEAD], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b = __hip_atomic_load(a.best64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      h = __shfl(h, 0);
      best64 = __shfl(b, 0);
      if (!dry && (ring_dead || h >= n_in)) {
        dry = true;
        limit = min(limit, steps + a.grace);
      }
    }

    QI_STAMP(1);  // fetch + polls
    // ---- (3) budget exhausted: spill current node + stack to the next frontier --------
    {
      const bool spill = has && (steps >= limit || evictions >= a.evict_max);
      if (__any(spill)) {
        uint32_t total = 0;
        const uint32_t n = spill ? 1u + nst : 0u;
        uint32_t slot = reserve(n, &cc[C_OUT], total);
        if (spill) {
          write_unit(slot++, T, D, K, depth, dlen, -1);
          for (uint32_t i = nst; i > 0; --i) write_entry(slot++, (sbase + i - 1) & (SMAX - 1));
          nst = 0;
          has = false;
          done = true;
          close_segment();
        }
      }
    }

    QI_STAMP(2);  // spill
    // ---- (4) one search node per active lane (cpp:258-345) ---------------------------
    ++wave_iters;
    bool pending = false;
    bool active = has;
    if (has) {
      ++steps;
      ++seg_count;
      uint32_t any = 0;
#pragma unroll
      for (int w = 0; w < MW; ++w) any |= T[w] | D[w];
      if (dlen > a.half_m || !any) {  // currentVisitor prune (cpp:261) / empty (cpp:266)
        active = false;
        has = false;
      }
    }
    uint32_t X[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) X[w] = active ? D[w] : 0u;
    const bool dq = EV::template gfp<0>(f, X, 0u, rounds);  // cpp:281
    if (active) {
      ++seg_evals;
      pending = dq;
    }
    const bool active2 = active && !dq;
#pragma unroll
    for (int w = 0; w < MW; ++w) X[w] = active2 ? (T[w] | D[w]) : 0u;
    const bool qne = EV::template gfp<0>(f, X, 0u, rounds);  // cpp:301
    QI_STAMP(3);  // the two fixpoints
    bool push = false;
    uint32_t pb = 0;
    if (active2) {
      ++seg_evals;
      uint32_t dout = 0, qd = 0;
#pragma unroll
      for (int w = 0; w < MW; ++w) {
        dout |= D[w] & ~X[w];
        qd |= X[w] & ~D[w];
      }
      if (!qne || dout || !qd) {  // cpp:303, 308-314, 325
        has = false;
      } else {
        pb = EV::best(f, X, D, seg_zfb);  // cpp:317
#pragma unroll
        for (int w = 0; w < MW; ++w) X[w] &= ~D[w];
        X[pb >> 5] &= ~(1u << (pb & 31u));  // toRemove' = Q \ D \ {b} (cpp:330-334)
        push = true;
      }
    }
    // push the inclusion branch (cpp:343-345); a full stack evicts its shallowest entry
    // into the next frontier (wave-aggregated slot reservation, convergent).
    {
      const bool evict = push && nst == (uint32_t)SMAX;
      if (__any(evict)) {
        uint32_t total = 0;
        const uint32_t slot = reserve(evict ? 1u : 0u, &cc[C_OUT], total);
        if (evict) {
          write_entry(slot, sbase & (SMAX - 1));
          sbase = (sbase + 1) & (SMAX - 1);
          --nst;
          ++evictions;
        }
      }
      if (push) {
        const uint32_t pos = (sbase + nst) & (SMAX - 1);
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          ST_(pos, w) = X[w];
          T[w] = X[w];
        }
        ST_(pos, MW) = pb | (depth << 8) | (dlen << 17);
        ++nst;
        ++depth;  // continue with the exclusion branch (cpp:336): key bit stays 0
      }
    }

    QI_STAMP(4);  // findBestNode + push
    // ---- (5) quorum leaves: isMinimalQuorum + visitor, wave-cooperative --------------
    // Every pending lane (GFP(D) != ∅, cpp:281) needs |D| single-removal fixpoints
    // (isMinimalQuorum, cpp:188-198) and the complement check of the visitor (cpp:368).
    // Done per lane they would serialise the wave (the first removable vertex sits at a
    // ~uniform position of the D order), so they are spread over the wave in fixed slots
    // of S = a.coop_slot lanes per pending lane: lane l serves owner (l / S) of the
    // current pass, job k = l % S (+ chunk offset when |D|+1 > S).  The owner's D arrives
    // by __shfl, results by one LDS ds_or per successful job; one barrier per pass.
    const uint64_t pm = __ballot(pending);
    if (pm) {
      ++coop_phases;
      const uint32_t npend = (uint32_t)__popcll(pm);
      const uint32_t r = rank_in(pm);
      const uint32_t S = a.coop_slot, lgS = a.coop_slot_log2;
      const uint32_t P = (uint32_t)WAVE >> lgS;  // owners per pass
      if (pending) {
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          co_NE[w * WAVE + r] = 0u;
          co_VIS[w * WAVE + r] = 0u;
        }
      }
      __syncthreads();
      for (uint32_t q0 = 0; q0 < npend; q0 += P) {
        const uint32_t oi = q0 + (lane >> lgS);
        uint64_t mm = pm;
        for (uint32_t c = 0; c < oi && mm; ++c) mm &= mm - 1ull;  // oi-th pending lane
        const uint32_t ol = mm ? (uint32_t)__builtin_ctzll(mm) : 0u;
        uint32_t Dr[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) Dr[w] = __shfl(D[w], (int)ol);
        const uint32_t dl = __shfl(dlen, (int)ol);
        for (uint32_t c0 = 0; c0 <= a.half_m; c0 += S) {  // jobs 0..|D| (|D| <= half_m)
          const uint32_t k = c0 + (lane & (S - 1u));
          const bool act = oi < npend && k <= dl;
          const bool vis = act && k == dl;
          // job k < |D| removes the k-th vertex of the owner's D order (its LDS bytes);
          // NE is indexed by that position, so isMinimal's first hit is one ctz
          uint32_t v = 0;
          if (act && !vis) v = (dow[(k >> 2) * WAVE + ol] >> (8u * (k & 3u))) & 255u;
          uint32_t Y[MW];
#pragma unroll
          for (int w = 0; w < MW; ++w) {
            if (!act) Y[w] = 0u;
            else if (vis) Y[w] = a.scc_mask[w] & ~Dr[w];  // visitor: scc \ Q, outside available
            else Y[w] = Dr[w];
          }
          if (act && !vis) Y[v >> 5] &= ~(1u << (v & 31u));  // isMinimal: D \ {v}
          const bool ne = EV::template gfp<2>(f, Y, vis ? 1u : 0u, rounds);
          if (act && !vis && ne) atomicOr(&co_NE[(k >> 5) * WAVE + oi], 1u << (k & 31u));
          if (vis) {
#pragma unroll
            for (int w = 0; w < MW; ++w) co_VIS[w * WAVE + oi] = Y[w];
          }
          if (c0 + S > a.half_m) break;
        }
      }
      __syncthreads();
      if (pending) {
        uint32_t ne_any = 0, vis_any = 0;
        uint32_t NE[MW], VIS[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          NE[w] = co_NE[w * WAVE + r];
          VIS[w] = co_VIS[w * WAVE + r];
          ne_any |= NE[w];
          vis_any |= VIS[w];
        }
        has = false;
        if (!ne_any) {  // minimal quorum (cpp:283-285)
          seg_evals += 2u + dlen;  // cpp:184, |D| x cpp:192, visitor cpp:368
          ++seg_minq;
          if (vis_any) {  // disjoint quorum: witness, the unit ends here (cpp:369-377)
            const uint32_t slot = atomicAdd(&a.glob[0], 1u);
            if (slot < a.wit_cap) {
              uint32_t* wv = a.wit + (size_t)slot * WL::WORDS;
#pragma unroll
              for (int w = 0; w < MW; ++w) {
                wv[w] = K[w];
                wv[MW + 2 + w] = VIS[w];
              }
              wv[MW] = depth;
              wv[MW + 1] = dlen;
              for (uint32_t i = 0; i < (dlen + 3) / 4; ++i) wv[2 * MW + 2 + i] = DOW_(i);
            } else {
              atomicOr(&a.glob[1], FLAG_WIT_OVERFLOW);
            }
            atomicMin(a.best64, (unsigned long long)best_pack<MW>(K, depth));
            nst = 0;  // everything left in this unit follows the witness in preorder
          }
        } else {  // not minimal: isMinimal stops at the first removable vertex in D order
          uint32_t pos = 0;
#pragma unroll
          for (int w = MW - 1; w >= 0; --w)
            if (NE[w]) pos = (uint32_t)w * 32u + (uint32_t)__builtin_ctz(NE[w]);
          seg_evals += 2u + pos;  // cpp:184 + (pos+1) x cpp:192
        }
      }
      __syncthreads();
    }
    QI_STAMP(5);  // quorum-leaf phase
  }

  // units claimed by this wave's ring but never fetched: carry them over unchanged
  {
    const uint32_t ring_pos = ring_src + ring_next;
    const uint32_t left = (ring_next < ring_cnt) ? ring_cnt - ring_next : 0u;
    if (left) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&cc[C_OUT], left);
      base = __shfl(base, 0);
      for (uint32_t i = lane; i < left; i += WAVE) {
        const uint32_t src = ring_pos + i, dst = base + i;
        uint32_t* r = records + (size_t)src * RL::WORDS;
        for (int w = 0; w < RL::WORDS; ++w) r[w] = 0u;
        if (dst < a.out_cap) {
          const uint4* s4 = (const uint4*)(a.units_in + (size_t)src * UW);
          uint4* d4 = (uint4*)(a.units_out + (size_t)dst * UW);
          for (int q = 0; q < UW / 4; ++q) d4[q] = s4[q];
        } else {
          atomicOr(&a.glob[1], FLAG_OUT_OVERFLOW);
        }
      }
    }
  }

  // wave-reduce the running totals
  auto wsum = [&](uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
  };
  tot_nodes = wsum(tot_nodes);
  tot_evals = wsum(tot_evals);
  tot_minq = wsum(tot_minq);
  tot_zfb = wsum(tot_zfb);
  const uint64_t tr = wsum((uint64_t)rounds);
  tot_fetched = wsum(tot_fetched);
  if (lane == 0) {  // sharded: ~1800 waves per launch would otherwise queue on one L2 line
    unsigned long long* tt = a.totals + (size_t)(blockIdx.x & (TOT_SHARDS - 1)) * 16;
    atomicAdd(&tt[0], (unsigned long long)tot_nodes);
    atomicAdd(&tt[1], (unsigned long long)tot_evals);
    atomicAdd(&tt[2], (unsigned long long)tot_minq);
    atomicAdd(&tt[3], (unsigned long long)tot_zfb);
    atomicAdd(&tt[4], (unsigned long long)tr);
    atomicAdd(&tt[5], (unsigned long long)tot_fetched);
    atomicAdd(&tt[6], (unsigned long long)wave_iters);
    atomicAdd(&tt[7], (unsigned long long)coop_phases);
#ifdef QI_STAMPS
    for (int q = 0; q < 6; ++q) atomicAdd(&tt[8 + q], (unsigned long long)stamp_sum[q]);
#endif
  }

  // ---- last block of the launch: carry over never-claimed input units (whose waves all
  // hit their budget before the queue ran dry) with zeroed records, publish the counters.
  // Every counter read here is an atomic RMW, performed after the other blocks' returned
  // atomics; nothing the other blocks stored plainly is read.
  {
    uint32_t old = 0;
    if (lane == 0) old = atomicAdd(&cc[C_DONE], 1u);
    old = __shfl(old, 0);
    if (old == nb_used - 1u) {
      uint32_t hd = 0, out = 0;
      if (lane == 0) {
        hd = atomicAdd(&cc[C_HEAD], 0u);
        out = atomicAdd(&cc[C_OUT], 0u);
      }
      hd = __shfl(hd, 0);
      out = __shfl(out, 0);
      const uint32_t head = (uint32_t)min((uint64_t)static_end + hd, (uint64_t)n_in);
      const uint32_t left = n_in - head;
      for (uint32_t i = lane; i < left; i += WAVE) {
        uint32_t* r = records + (size_t)(head + i) * RL::WORDS;
        for (int w = 0; w < RL::WORDS; ++w) r[w] = 0u;
        const uint32_t dst = out + i;
        if (dst < a.out_cap) {
          const uint4* s4 = (const uint4*)(a.units_in + (size_t)(head + i) * UW);
          uint4* d4 = (uint4*)(a.units_out + (size_t)dst * UW);
          for (int q = 0; q < UW / 4; ++q) d4[q] = s4[q];
        } else {
          atomicOr(&a.glob[1], FLAG_OUT_OVERFLOW);
        }
      }
      if (lane == 0) {
        out += left;
        if (left) atomicExch(&cc[C_OUT], out);
        a.host_ctr[HC_OUT] = out;
        a.host_ctr[HC_NIN] = n_in;
        a.host_ctr[HC_LOGB] = log_base;
        a.host_ctr[HC_STOP] = 0u;
        a.host_ctr[HC_DONE] = 1u;
      }
    }
  }
#undef ST_
#undef DOW_
#undef UR_
}

}  // namespace dev
}  // namespace qi
