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
using __hip_internal::uint16_t;
#endif

namespace qi {
namespace dev {

constexpr int WAVE = 64;
typedef uint32_t qi_v4u __attribute__((ext_vector_type(4)));

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
  static constexpr int WORDS = RAW <= 8 ? 8 : (RAW <= 16 ? 16 : (RAW <= 32 ? 32 : (RAW <= 64 ? 64 : 128)));
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
  uint32_t qmin0, qmin1;       // LocalFlat::qmin: |X| below it => empty fixpoint
  uint32_t scc_mask[32];       // the searched SCC (all m local vertices, m <= 1024)
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
// Lane 0's value, wave-uniform: v_readlane (a __shfl from lane 0 is an LDS ds_bpermute
// round trip).
__device__ __forceinline__ uint32_t lane0(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 0); }
__device__ __forceinline__ uint64_t lane0(uint64_t v) {
  return ((uint64_t)lane0((uint32_t)(v >> 32)) << 32) | lane0((uint32_t)v);
}

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
  {  // a non-empty fixpoint needs >= qmin vertices (LocalFlat::qmin): skip the rounds
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < MW; ++w) c += __popc(X[w]);
    const uint32_t q = POL == 0 ? f.qmin0 : (POL == 1 ? f.qmin1 : (pol ? f.qmin1 : f.qmin0));
    if (c < q) {
#pragma unroll
      for (int w = 0; w < MW; ++w) X[w] = 0u;
    }
  }
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

// findBestNode with the reference's own rule (cpp:229-246): uniform over the vertices of
// Q \ D with the maximal in-degree.  The reference draws from a process-global random
// engine; here the draw is a hash of (seed, path key, depth) of the node, so a search is
// reproducible and independent of the schedule.  `pick` = that hash.
template <int MW>
__device__ __forceinline__ uint32_t best_node_random(const LocalDev& f, const uint32_t (&Q)[MW], const uint32_t (&D)[MW],
                                                  uint32_t& zero_fallback, uint32_t pick) {
  uint32_t bestdeg = 0;
  uint32_t C[MW];  // candidates with the best degree so far
#pragma unroll
  for (int w = 0; w < MW; ++w) C[w] = 0u;
  bool any = false;
  for (uint32_t g = 0; g < f.G; ++g) {
    uint32_t deg = 0, cand_any = 0;
    uint32_t M[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      deg += __popc(Q[w] & K(f.grp_col)[g * MW + w]);
      M[w] = Q[w] & ~D[w] & K(f.grp_members)[g * MW + w];
      cand_any |= M[w];
    }
    const uint32_t e0 = K(f.grp_extra_off)[g], e1 = K(f.grp_extra_off)[g + 1];
    for (uint32_t e = e0; e < e1; ++e) {
#pragma unroll
      for (int w = 0; w < MW; ++w) deg += __popc(Q[w] & K(f.grp_extra)[e * MW + w]);
    }
    if (!cand_any) continue;
    if (!any || deg > bestdeg) {
      any = true;
      bestdeg = deg;
#pragma unroll
      for (int w = 0; w < MW; ++w) C[w] = M[w];
    } else if (deg == bestdeg) {
#pragma unroll
      for (int w = 0; w < MW; ++w) C[w] |= M[w];
    }
  }
  zero_fallback += (bestdeg == 0u) ? 1u : 0u;
  uint32_t cnt = 0;
#pragma unroll
  for (int w = 0; w < MW; ++w) cnt += __popc(C[w]);
  if (!cnt) return 0xFFFFFFFFu;
  uint32_t k = pick % cnt;
  uint32_t v = 0xFFFFFFFFu;
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    const uint32_t c = __popc(C[w]);
    if (v == 0xFFFFFFFFu) {
      if (k < c) {
        uint32_t x = C[w];
        for (uint32_t i = 0; i < k; ++i) x &= x - 1u;  // drop the k lowest candidates
        v = (uint32_t)w * 32u + (uint32_t)__builtin_ctz(x);
      } else {
        k -= c;
      }
    }
  }
  return v;
}

// The draw of a node: a mix of the seed, its path key and its depth.
template <int MW>
__device__ __forceinline__ uint32_t tie_hash(uint32_t seed, const uint32_t (&Kk)[MW], uint32_t depth) {
  uint32_t h = seed ^ (depth * 0x9E3779B9u);
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    h ^= Kk[w] + 0x7F4A7C15u + (h << 6) + (h >> 2);
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
  }
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
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
  static __device__ __forceinline__ uint32_t scc_word(const LocalDev& f, int w) { return f.scc_mask[w]; }
  static __device__ __forceinline__ uint32_t qmin0(const LocalDev& f) { return f.qmin0; }
  // the removal-sensitivity pass is generated per SCC only (SpecEval::min_bad)
  static constexpr bool FASTMIN = false;
  static __device__ __forceinline__ void min_bad(const LocalDev&, const uint32_t (&)[MW], uint32_t (&bad)[MW]) {
#pragma unroll
    for (int w = 0; w < MW; ++w) bad[w] = 0u;
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
// bytes per vertex index in order lists: 1 up to 256 local vertices, 2 beyond
template <int MW>
struct OrdBytes {
  static constexpr int VB = MW > 8 ? 2 : 1;
};
// witness: key[MW], depth, dlen, q1[MW], D order (OrdBytes<MW>::VB bytes per entry)
template <int MW>
struct WitLayout {
  static constexpr int ORDW = (UnitLayout<MW>::DMAX * OrdBytes<MW>::VB + 3) / 4;
  static constexpr int WORDS = 2 * MW + 2 + ORDW;
};

// Per-launch counter block (CTR_WORDS words).  Launches are chained on the device: launch
// k reads its input count, log position and stop state from launch k-1's block (or from a
// host-written seed block), so the host enqueues launches without reading anything back
// in between.  Every atomically updated word has a 128-B line of its own: atomics of many
// waves on one line are served one at a time (measured 11.5 ns each, returned or not, same
// word or not: tools/atomic_probe.hip), so a full grid's claims, spill reservations and
// finish counts on ONE line put a floor of ~130 us under a launch whose waves end together.
// The last block of a launch carries never-claimed input units over and publishes the
// final block to pinned host memory (HC_* words), where the host polls it.
enum : int {
  C_OUT = 0,       // units written to units_out (spills + carried-over units)   [atomic]
  C_HEAD = 32,     // dynamic claims past the statically assigned range           [atomic]
  C_DONE = 64,     // used blocks that finished                                   [atomic]
  C_EVX = 96,      // stack evictions granted from the shared output pool          [atomic]
  C_DIAG = 100,    // QI_DIAG_LAUNCH: max wave iterations, sum / max wave ticks, max ~start, max end [atomic]
  C_NIN = 128,     // input units of this launch (the previous block's C_OUT)
  C_LOGB = 129,    // first segment-log record of this launch
  C_STOP = 130,    // 1: capacity would be exceeded; this launch (and the rest of the chain) did nothing
  C_STATIC = 131,  // end of the statically assigned range (64 units per used block)
  C_LOGN = 132,    // log base of the next launch (written by this launch's last block)
  C_HALT = 133,    // 1: this launch carried units over (its lanes ran out of budget with
                   // units left); the rest of the chain does nothing and the host sorts
                   // the frontier into preorder before it goes on
  C_PEAKED = 134,  // launches of the chain so far that ran with the run budget (> 0: the
                   // frontier has covered the lanes once, what follows is its decay)
  CTR_WORDS = 160,
  HC_OUT = 0, HC_NIN = 1, HC_LOGB = 2, HC_STOP = 3, HC_DONE = 4, HC_LOGN = 5, HC_HALT = 6,
  HC_BEST = 8,     // u64 (two words): the device-side best key after this launch
  HC_FLAG = 10,    // u64, ONE 8-byte store, written last: bit 63 = published, bit 62 = stopped,
                   // low 32 bits = units out.  The host spins on it in pinned memory to pace
                   // its look-ahead (no event per launch); the other words are read after
                   // the chain's final stream synchronisation.
  HC_DIAG = 16,    // kernels built with QI_DIAG_LAUNCH only: running nodes, running wave iterations, then
                   // of this launch: max wave iterations, sum and max of the waves' run times and the
                   // span first wave start .. last wave end (10 ns ticks)
  HC_WORDS = 32
};
// Output capacity per launch: n_in (carried-over units) + per used lane SPILL_RESERVE(S)
// units for its one final spill (current node, top of stack, S stacked entries, a claimed
// unit, one forced eviction) + a shared pool for stack evictions (>= evict_max per lane).
// An eviction the pool cannot grant makes the lane spill and stop instead (FLAG_POOL); the
// host then grows the buffers.  Every lane therefore digs as deep as its node budget
// allows while there is room, and a launch never writes past out_cap.
__host__ __device__ constexpr uint32_t spill_reserve(uint32_t smax) { return smax + 4u; }
constexpr int TOT_SHARDS = 64;  // running totals: [TOT_SHARDS][16] u64, shard = block % 64

__device__ __forceinline__ void publish_flag(uint32_t* host_ctr, bool stop, uint32_t out) {
  __hip_atomic_store((unsigned long long*)(host_ctr + HC_FLAG),
                     (1ull << 63) | (stop ? (1ull << 62) : 0ull) | (unsigned long long)out, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr int POLL_REPS = 64;
constexpr int KEY_WORDS_MAX = 32;  // path-key words of the largest kernel shape (MW <= 32)
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
  const unsigned long long* xbest;  // the same key over every cooperating engine (other streams,
                                 // GPUs or processes): a word in pinned host memory that the
                                 // hosts fold their launches' best keys into; block 0 of a launch
                                 // polls it and forwards it; == best64 for a lone engine
  uint32_t* poll_rep;            // [POLL_REPS][32 words] what the waves poll, replicated on 128-B
                                 // lines (wave b reads line b % POLL_REPS): words 0-1 the best key,
                                 // word 2 the sequence number of the last launch seen dry.  Every
                                 // wave polling ONE best key / queue head serialised at that line
                                 // (~25 ns per access: 0.8 ms per search at 64-iteration polls).
  uint32_t* diag_waves;          // QI_DIAG_WAVES builds: [blocks][4] start, dry, first spill, end (10 ns ticks)
  uint32_t seq;                  // this launch's sequence number (unique per engine, never 0xFFFFFFFF)
  uint32_t tiebreak;             // findBestNode ties: 0 lowest vertex index, 1 the seeded uniform draw
                                 // (informational: the rule is compiled into the kernel, search_body's TIE)
  uint32_t tie_seed;
  uint32_t grow_budget;          // per-lane node budget while the frontier is below half the lanes
  uint32_t run_budget;
  uint32_t grace;                // extra steps per lane once the unit queue is dry
  uint32_t run_at;               // run budget once n_in >= run_at/8 of the resident lanes
  uint32_t evict_max;
  uint32_t half_m;
  uint32_t coop_slot;            // lanes per pending owner in the cooperative phase (pow2)
  uint32_t coop_slot_log2;
  uint32_t has_best;             // host-known best key (multiword) for pruning
  uint32_t best_depth;
  uint32_t best_key[KEY_WORDS_MAX];
};
static_assert(sizeof(SearchArgs) <= 1024, "kernel argument block");

enum : uint32_t { FLAG_OUT_OVERFLOW = 1u, FLAG_WIT_OVERFLOW = 2u, FLAG_POOL = 8u };

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
  static_assert(MW <= 32, "path keys hold at most 32 words (SearchArgs::best_key, the engines' key buffers)");
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    if (K[w] != B[w]) return K[w] > B[w];
  }
  return d > db;
}

template <int MW>
__device__ __forceinline__ void key_prefix_bit(uint32_t (&K)[MW], uint32_t de) {
  // keep path positions < de, then set position de (inclusion branch at depth de)
  if constexpr (MW == 1) {  // de <= 31: three shifts and a merge
    K[0] = (K[0] & ~(0xFFFFFFFFu >> de)) | (0x80000000u >> de);
    return;
  }
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

// Per-lane node budget of a launch from how well its input covers the resident lanes:
// a small frontier grows (a few nodes per lane, then spill: more units next launch); a
// frontier that covers most lanes runs long.
// Once a launch of the chain has run with the run budget (`peaked`), the rest do too: a
// shrinking frontier holds deep, small subtrees, and relaunching them every grow-budget
// steps only adds launches (their lanes stop `grace` steps after the queue runs dry anyway).
__device__ __forceinline__ uint32_t launch_budget(const SearchArgs& a, uint32_t n_in, bool peaked) {
  const uint64_t lanes8 = (uint64_t)gridDim.x * WAVE;
  const uint64_t n8 = (uint64_t)n_in * 8u;
  return (!peaked && n8 < lanes8 * a.run_at) ? a.grow_budget : a.run_budget;
}

// Wave-aggregated reservation of n (per lane, n < 2^NB) slots on a global counter: the
// exclusive wave prefix sum is bit-sliced over NB ballots (mbcnt per bit plane), so it
// needs no LDS round trips; one atomic per wave.  Convergent.
template <int NB>
__device__ __forceinline__ uint32_t reserve(uint32_t n, uint32_t* counter, uint32_t& total_out) {
  uint32_t pre = 0, total = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint64_t m = __ballot((n >> b) & 1u);
    pre += rank_in(m) << b;
    total += (uint32_t)__popcll(m) << b;
  }
  uint32_t base = 0;
  if (lane_id() == 0 && total) base = atomicAdd(counter, total);
  base = lane0(base);
  total_out = total;
  return base + pre;
}

// LDS words of one search wavefront (search_body's carve-up below).
template <int MW, int SMAX>
constexpr int search_lds_words() {
  // DFS stack below the top entry: T', D' words + a packed (b, depth, |D|) word per level
  return SMAX * (2 * MW + 1) * WAVE
         + 2 * MW * WAVE                        // co_NE, co_VIS
         + (MW + 1) * WAVE                      // co_D, co_OWN
         + ((UnitLayout<MW>::DMAX + 3) / 4) * WAVE;  // D order
}

// Diagnostic build only (QI_STAMPS, run-time specialised kernel with jit=3): per-wave
// s_memtime sums of the loop sections, added into totals[8..15].  The production kernels
// contain no stamps.
// Loop sections (fine ids) and the six buckets a stamp build reports them in
// (QI_STAMP_SET: 0 = everything, coarse; 1 and 2 = two fine views; -1 = not recorded).
enum : int { F_POP = 0, F_INSTALL, F_POLL, F_SPILL, F_GFP1, F_GFP2, F_BEST, F_PUSH, F_FLUSH, F_CLAIM, F_FASTP, F_FASTMIN,
             F_COOP, F_W_INSTALL, F_W_CLAIM, F_W_POP, F_RESET, F_FAST };
#ifndef QI_STAMP_SET
#define QI_STAMP_SET 0
#endif
constexpr int stamp_bucket(int f) {
  if (QI_STAMP_SET == 1)
    return f == F_POP ? 0 : f == F_INSTALL ? 1 : f == F_BEST ? 2 : f == F_PUSH ? 3 : f == F_FLUSH ? 4 : f == F_CLAIM ? 5 : -1;
  if (QI_STAMP_SET == 4)  // fast steps against everything else
    return f == F_FAST ? 0 : 1;
  if (QI_STAMP_SET == 3)  // explicit waits only: unit loads at install, the queue head's atomic at claim, LDS refill at pop
    return f == F_W_INSTALL ? 0 : f == F_W_CLAIM ? 1 : f == F_W_POP ? 2 : -1;
  if (QI_STAMP_SET == 2)
    return f == F_FASTP ? 0 : f == F_FASTMIN ? 1 : f == F_COOP ? 2 : f == F_POLL ? 3 : f == F_SPILL ? 4
           : (f == F_GFP1 || f == F_GFP2) ? 5 : -1;
  return f == F_FAST ? 2 : f <= F_INSTALL ? 0 : f == F_POLL ? 1 : f == F_SPILL ? 2 : f <= F_GFP2 ? 3 : f <= F_CLAIM ? 4 : 5;
}
#ifdef QI_STAMPS
#define QI_STAMP(slot)                                                   \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();                  \
    __builtin_amdgcn_sched_barrier(0);                                   \
    if (stamp_bucket(slot) >= 0) stamp_sum[stamp_bucket(slot) < 0 ? 0 : stamp_bucket(slot)] += now_ - stamp_prev; \
    stamp_prev = now_;                                                   \
  } while (0)
// stamp set 3: an explicit counter wait bracketed by stamps (what the wave waits there)
#if QI_STAMP_SET == 3
#define QI_WAIT_STAMP(what, id)                 \
  do {                                          \
    QI_STAMP(F_RESET);                          \
    asm volatile("s_waitcnt " what ::: "memory"); \
    QI_STAMP(id);                               \
  } while (0)
#else
#define QI_WAIT_STAMP(what, id) \
  do {                          \
  } while (0)
#endif
#elif defined(QI_MARKS)
// diagnostics: assembly markers at the section boundaries (static instruction counts)
#define QI_STAMP(slot) asm volatile(";QIMARK " #slot ::: "memory")
#define QI_WAIT_STAMP(what, id) \
  do {                          \
  } while (0)
#else
#define QI_WAIT_STAMP(what, id) \
  do {                          \
  } while (0)
#define QI_STAMP(slot) \
  do {                 \
  } while (0)
#endif

// single-round fixpoint when one root TN serves every vertex (generated evaluator)
#ifndef QI_ONE_ROOT
#define QI_ONE_ROOT 1
#endif
// removal-sensitivity minimality for |D| = qmin + 1 leaves (EV::FASTMIN)
#ifndef QI_FASTMIN
#define QI_FASTMIN 1
#endif
// packed D-order words per lane in LDS (a specialised kernel sizes them for its SCC)
#ifndef QI_LDS_OW
#define QI_LDS_OW 0
#endif
// Iterations (fast steps included) between polls of the dry flag (the poll is taken in the
// first full iteration past the interval).  A wave with an empty lane learns that the queue
// is dry from its own failed claim; the poll ends the waves whose lanes are all still busy.
// With every lane's unit turnover paid per full iteration (not per node) the waves of a
// launch should end together: 768 / 576 / 384 / 192 / 128 / 96 / 64 / 32 iterations gave
// 1.74 / 1.69 / 1.62 / 1.59 / 1.55 / 1.49-1.51 / 1.51 / 1.50 ms per search (before the fast
// steps the optimum was 384: ending busy waves early cost more in unit turnover).
#ifndef QI_POLL_EVERY
#define QI_POLL_EVERY 96
#endif
// The best key is polled more often than the dry flag acts: every QI_POLL_EVERY /
// QI_BEST_POLLS iterations (a witness found elsewhere prunes sooner); the dry flag counts in
// every QI_BEST_POLLS-th of these polls.
#ifndef QI_BEST_POLLS
#define QI_BEST_POLLS 2
#endif
// Fast steps: up to QI_FAST_STEPS lean iterations run between two full ones while at least
// QI_FAST_MIN lanes can pop or process a node without any service (no unit to install, no
// quorum leaf, no full stack) and no witness is known (nothing to prune).  The full
// iteration below carries every rarely needed path; paying for it on every node made the
// loop issue-bound on control code.
#ifndef QI_FAST_STEPS
#define QI_FAST_STEPS 12
#endif
#ifndef QI_FAST_MIN
#define QI_FAST_MIN 28
#endif
// run budget for every launch after the first one that had it (see launch_budget): 0 off,
// 1 always, 2 only while no witness is known (measured: two_tier(8,192) 0.43 / 0.40 / 0.41 ms,
// planted_deep 0.97 / 1.15 / 0.97 ms, the bench workload 2.21 / 2.18 / 2.21 ms)
#ifndef QI_DECAY_RUN
#define QI_DECAY_RUN 2
#endif
// fast steps of a dry wave run with this many eligible lanes (no unit can be installed any
// more, so waiting for a full iteration serves only quorum leaves and full stacks)
// fast steps in growth launches too (their per-lane budget stays exact)
#ifndef QI_GROW_FAST
#define QI_GROW_FAST 1
#endif
#ifndef QI_FAST_MIN_DRY
#define QI_FAST_MIN_DRY 8
#endif
// share of a full grid's input that is dealt out statically, as one slab per block (see static_end)
#ifndef QI_SLAB_PCT
#define QI_SLAB_PCT 75
#endif
// TIE: findBestNode's tie rule, fixed per kernel (a run-time choice in the node loop cost
// 15-50 % per search): false = lowest vertex index, true = the seeded uniform draw.
template <int MW, int TW, int SMAX, class EV, bool TIE = false>
__device__ __forceinline__ void search_body(const SearchArgs& a) {
  using UL = UnitLayout<MW>;
  using RL = RecLayout<MW>;
  using WL = WitLayout<MW>;
  constexpr int DMAX = UL::DMAX;
  constexpr int UW = UL::WORDS;
  // stack entry: T' [MW] | D of the inclusion child [MW] | packed (b, depth, |D| before b)
  constexpr int SE = 2 * MW + 1;
  constexpr int RB = (SMAX + 3 < 64) ? 6 : (SMAX + 3 < 128 ? 7 : 8);  // bits of a lane's spill count
  // packed D-order words (4 vertex bytes each) per lane in LDS; a specialised kernel sizes
  // them for its SCC (|D| <= m/2 + 1: QI_LDS_OW), which for m <= 31 frees the 256 B that
  // take a wave from 7 to 8 resident per CU
  constexpr int OW = (QI_LDS_OW > 0 && QI_LDS_OW < (DMAX + 3) / 4) ? QI_LDS_OW : (DMAX + 3) / 4;
  // the next unit is loaded into registers one node ahead (small units); large units are
  // loaded when installed
  constexpr bool PREFETCH = UW <= 20;
  constexpr int FW = PREFETCH ? UW : 4;
  constexpr bool WIDE = PREFETCH;  // small units and their records leave as 16- / 8-byte stores
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* st = lds;                                          // [SMAX][SE][64]
  uint32_t* co_NE = st + SMAX * SE * WAVE;                      // [MW][64] per pending rank
  uint32_t* co_VIS = co_NE + MW * WAVE;                         // [MW][64] per pending rank
  uint32_t* co_D = co_VIS + MW * WAVE;                          // [MW][64] pending owners' D
  uint32_t* co_OWN = co_D + MW * WAVE;                          // [64] owner lane | dlen << 8
  uint32_t* dow = co_OWN + WAVE;                                // [OW][64] D in branch order

  const uint32_t lane = threadIdx.x;
  const LocalDev& f = a.f;
  // ---- chained launch prologue: input count, log position, capacity (wave-uniform) ----
  const uint32_t* pc = a.prev;
  uint32_t* cc = a.counters;
  if (pc[C_STOP] || pc[C_HALT]) {  // an earlier launch stopped or halted: the frontier stays
    if (blockIdx.x == 0 && lane == 0) {
      cc[C_STOP] = 1u;
      a.host_ctr[HC_STOP] = 1u;
      a.host_ctr[HC_DONE] = 1u;
      publish_flag(a.host_ctr, true, 0u);
    }
    return;
  }
  const uint32_t n_in = pc[C_OUT];
  const uint32_t log_base = pc[C_LOGN];
  const uint32_t nb_used = min((n_in + (uint32_t)WAVE - 1u) / (uint32_t)WAVE, gridDim.x);
  // Statically assigned units: block b owns the slab [b * slab, (b + 1) * slab), its lanes' first
  // units and then pools of 64 taken without an atomic; only the rest of the input
  // (QI_SLAB_PCT % of it is dealt out as slabs) is claimed dynamically, to even out the waves.
  // The dynamic queue's head is ONE word: a full grid's waves run out of units in bursts,
  // and each claim then waited ~3 us for that line (6.5 % of all wave cycles).
  uint32_t slab = (uint32_t)WAVE;
  if (nb_used == gridDim.x)
    slab *= max(1u, (uint32_t)(((uint64_t)n_in * (uint32_t)QI_SLAB_PCT / 100u) / ((uint64_t)nb_used * WAVE)));
  const uint32_t static_end = min(n_in, nb_used * slab);
  // evictions share what the final spills and the carried-over units leave of out_cap
  const uint64_t spill_need = (uint64_t)n_in + (uint64_t)nb_used * WAVE * spill_reserve(SMAX);
  const uint32_t evict_pool = spill_need < (uint64_t)a.out_cap ? (uint32_t)((uint64_t)a.out_cap - spill_need) : 0u;
  // (QI_DECAY_RUN 2: not once a witness is known -- short launches then prune sooner)
  const uint32_t peaked_n = pc[C_PEAKED];  // run-budget launches of this chain so far
  const bool peaked_in = QI_DECAY_RUN && peaked_n != 0u && (QI_DECAY_RUN == 1 || *a.best64 == ~0ull);
  const uint32_t budget = launch_budget(a, n_in, peaked_in);
  {
    // the final spills, and at least evict_max evictions per used lane
    const uint64_t need_out = spill_need + (uint64_t)nb_used * WAVE * (uint64_t)a.evict_max;
    const uint64_t need_log = (uint64_t)log_base + n_in;
    const bool stop = need_out > (uint64_t)a.out_cap || need_log > (uint64_t)a.log_cap;
    if (blockIdx.x == 0 && lane == 0) {
      cc[C_NIN] = n_in;
      cc[C_LOGB] = log_base;
      cc[C_STATIC] = static_end;
      cc[C_STOP] = stop ? 1u : 0u;
      cc[C_PEAKED] = peaked_n + ((!stop && nb_used != 0 && budget == a.run_budget) ? 1u : 0u);
      if (stop || nb_used == 0) {  // nothing runs: publish now (else the last block does)
        cc[C_LOGN] = log_base;
        a.host_ctr[HC_LOGN] = log_base;
        a.host_ctr[HC_OUT] = 0u;
        a.host_ctr[HC_NIN] = n_in;
        a.host_ctr[HC_LOGB] = log_base;
        a.host_ctr[HC_STOP] = stop ? 1u : 0u;
        a.host_ctr[HC_DONE] = 1u;
        publish_flag(a.host_ctr, stop, 0u);
      }
    }
    if (stop || blockIdx.x >= nb_used) return;
  }
  uint32_t* const records = a.records + (size_t)log_base * RL::WORDS;
#define ST_IDX(lvl, w, ln) (((lvl) * SE + (w)) * WAVE + (ln))
#define ST_(lvl, w) st[ST_IDX(lvl, w, lane)]
#define DOW_(w) dow[(w) * WAVE + lane]
  // byte i of this lane's D order (ds_write_b8 into the packed word)
  auto set_ord = [&](uint32_t i, uint32_t v) {
    ((uint8_t*)dow)[(((i >> 2) * WAVE + lane) << 2) + (i & 3u)] = (uint8_t)v;
  };

  // current node
  uint32_t T[MW], D[MW], K[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) T[w] = D[w] = K[w] = 0;
  uint32_t depth = 0, dlen = 0;
  bool has = false, done = false;
  // top of the DFS stack in registers (packed word: b | depth << 8 | |D| << 17); `nst`
  // entries below it in LDS (circular from sbase_)
  uint32_t tT[MW], tD[MW], tpk = 0;
#pragma unroll
  for (int w = 0; w < MW; ++w) tT[w] = tD[w] = 0;
  bool tvalid = false;
  uint32_t nst = 0, sbase_ = 0;
  auto spos = [&](uint32_t i) -> uint32_t {  // circular stack position of entry i (0 = bottom)
    const uint32_t p = sbase_ + i;
    return p >= (uint32_t)SMAX ? p - (uint32_t)SMAX : p;
  };
  uint32_t steps = 0;
  bool must_spill = false;  // an eviction found the pool empty: spill at the next iteration
  uint32_t limit = budget;  // per-lane step limit; shrinks to steps+grace when the queue dries
  const bool exact_budget = budget <= 2u * (uint32_t)QI_FAST_STEPS;  // wave-uniform: a growth launch
  bool dry = false;         // wave-uniform: no unit left to claim (head >= n_in)
  // wave-uniform: the iteration at which a dry wave spills whatever its lanes still hold --
  // all lanes at once, so the wave reserves its output slots with ONE atomic
  uint32_t force_at = 0xFFFFFFFFu;
  uint32_t iter = 0;        // wave-uniform: iterations so far, fast steps included
  uint32_t next_poll = 0;   // the poll is due in the first full iteration with iter >= next_poll
  bool poll_issued = true;  // its loads are in flight (the first ones are issued before the loop)
  uint32_t poll_n = 0;      // polls so far (the queue head counts in every QI_BEST_POLLS-th)
  // the next unit of this lane: claimed index (= its log record index) + (PREFETCH) its
  // words in registers; installed at the start of the iteration after the lane ran out
  bool fpend = false;
  uint32_t fidx = 0;
  uint32_t fdat[FW];
#pragma unroll
  for (int q = 0; q < FW; ++q) fdat[q] = 0;
  // current segment (one per installed unit)
  bool seg_open = false;
  uint32_t seg_idx = 0, seg_depth = 0, seg_evals = 0, seg_minq = 0, seg_zfb = 0;
  uint32_t seg_s0 = 0;  // the lane's step count when the segment opened: its nodes = steps - seg_s0
  uint32_t seg_K[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) seg_K[w] = 0;
  uint64_t tot_nodes = 0, tot_evals = 0, tot_minq = 0, tot_zfb = 0, tot_fetched = 0;
  uint32_t rounds = 0;
  uint32_t wave_iters = 0, coop_phases = 0;  // wave-uniform: occupancy accounting
#ifdef QI_STAMPS
  uint64_t stamp_sum[6] = {0, 0, 0, 0, 0, 0};
  uint64_t stamp_prev = __builtin_amdgcn_s_memtime();
  const uint64_t wave_t0 = __builtin_amdgcn_s_memrealtime();
#endif
#if defined(QI_DIAG_LAUNCH) || defined(QI_DIAG_WAVES)
  const uint32_t diag_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
  uint32_t diag_dry = 0, diag_sp0 = 0, diag_spr = 0, diag_sp1 = 0, diag_loop0 = 0;  // 0 = did not happen
#define QI_DIAG_MARK(v) do { if (!(v)) (v) = (uint32_t)__builtin_amdgcn_s_memrealtime() | 1u; } while (0)
#else
#define QI_DIAG_MARK(v) do { } while (0)
#endif
  uint64_t best64 = ~0ull;
  // lane 0's poll loads are issued one iteration before the poll that reads them, so
  // their latency hides behind that iteration (the first poll, at iteration 0, reads these)
  uint32_t* const my_rep = a.poll_rep + (size_t)(blockIdx.x & (POLL_REPS - 1)) * 32;
  uint32_t poll_d = 0;      // lane 0: the polled dry-launch sequence number
  uint64_t poll_b = ~0ull;  // lane 0: the polled best key
  uint64_t poll_x = ~0ull;  // lane 0 of block 0: the cooperating engines' shared key
  const bool forwarder = blockIdx.x == 0 && a.xbest != a.best64;  // wave-uniform
  auto issue_poll = [&]() {  // lane 0
    poll_b = __hip_atomic_load((unsigned long long*)my_rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    poll_d = __hip_atomic_load(my_rep + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (forwarder) poll_x = __hip_atomic_load(a.xbest, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  // a best key into the canonical word and every polled replica (witnesses are rare)
  auto publish_best = [&](unsigned long long key) {
    atomicMin(a.best64, key);
    for (int r = 0; r < POLL_REPS; ++r) atomicMin((unsigned long long*)(a.poll_rep + (size_t)r * 32), key);
  };
  if (lane == 0) issue_poll();

  auto load_unit = [&]() {  // issue the loads of unit fidx (consumed at install)
    if constexpr (PREFETCH) {
      const uint4* src = (const uint4*)(a.units_in + (size_t)fidx * UW);
#pragma unroll
      for (int q = 0; q < UW / 4; ++q) {
        const uint4 v = src[q];
        fdat[4 * q + 0] = v.x;
        fdat[4 * q + 1] = v.y;
        fdat[4 * q + 2] = v.z;
        fdat[4 * q + 3] = v.w;
      }
    }
  };
  auto unit_word = [&](int wi) -> uint32_t {  // word wi of the claimed unit
    if constexpr (PREFETCH) return fdat[wi];
    else return a.units_in[(size_t)fidx * UW + wi];
  };
  // the statically assigned first unit of this lane (no atomic)
  if (blockIdx.x * slab + lane < n_in) {
    fidx = blockIdx.x * slab + lane;
    fpend = true;
    load_unit();
  }
  // wave-uniform pool of claimed unit indices: the rest of this block's slab first
  uint32_t pool_next = min(blockIdx.x * slab + (uint32_t)WAVE, n_in), pool_end = min((blockIdx.x + 1u) * slab, n_in);
  bool pool_dead = static_end >= n_in;

  // A closed segment's record is written at the end of the iteration (flush_record), not
  // where the segment closes: a store just before the next unit's install would make
  // the install's wait for its prefetched loads also wait for the store.
  bool rec_pend = false;
  uint32_t rec[RL::WORDS], rec_idx = 0;
#pragma unroll
  for (int w = 0; w < RL::WORDS; ++w) rec[w] = 0;
  auto flush_record = [&]() {
    if (rec_pend) {
      uint32_t* r = records + (size_t)rec_idx * RL::WORDS;
      if constexpr (WIDE && RL::WORDS % 2 == 0) {  // 8-byte stores (record stride and log base are 8-byte multiples)
#pragma unroll
        for (int w = 0; w < RL::WORDS; w += 2) *(uint2*)(r + w) = make_uint2(rec[w], rec[w + 1]);
      } else {
#pragma unroll
        for (int w = 0; w < RL::WORDS; ++w) r[w] = rec[w];
      }
      rec_pend = false;
    }
  };
  auto close_segment = [&]() {
    flush_record();
#pragma unroll
    for (int w = 0; w < MW; ++w) rec[w] = seg_K[w];
    rec[MW] = seg_depth;
    const uint32_t seg_count = steps - seg_s0;
    rec[MW + 1] = seg_count;
    rec[MW + 2] = seg_evals;
    rec[MW + 3] = seg_minq;
    rec[MW + 4] = seg_zfb;
    rec_idx = seg_idx;
    rec_pend = true;
    tot_nodes += seg_count;
    tot_evals += seg_evals;
    tot_minq += seg_minq;
    tot_zfb += seg_zfb;
    seg_open = false;
  };

  auto pruned = [&](const uint32_t (&KK)[MW], uint32_t d) -> bool {
    bool p = false;
    // MW == 1: best64 is exact and the host writes its best there (no kernel-argument key)
    if (MW > 1 && a.has_best) p = after_key<MW>(KK, d, a.best_key, a.best_depth);
    p = p || (best_pack<MW>(KK, d) > best64);
    return p;
  };

  // write one unit (T, D given as masks, order = DOW[0..ol) + optional extra byte)
  auto write_unit = [&](uint32_t slot, const uint32_t (&UT)[MW], const uint32_t (&UD)[MW], const uint32_t (&UK)[MW],
                        uint32_t udepth, uint32_t ol, int extra_b) {
    if (slot >= a.out_cap) {
      atomicOr(&a.glob[1], FLAG_OUT_OVERFLOW);
      return;
    }
    uint32_t* u = a.units_out + (size_t)slot * UW;
    const uint32_t ulen = ol + (extra_b >= 0 ? 1u : 0u);
    if constexpr (WIDE) {
      // small units go out whole, as 16-byte stores: a launch end writes ~4 units per lane,
      // and word-by-word (4-byte stores 48 B apart across the wave) that took 50-90 us of a
      // decaying launch's ~300
      uint32_t uw[UW];
#pragma unroll
      for (int q = 0; q < UW; ++q) uw[q] = 0u;
#pragma unroll
      for (int w = 0; w < MW; ++w) {
        uw[UL::T_ + w] = UT[w];
        uw[UL::D_ + w] = UD[w];
        uw[UL::K_ + w] = UK[w];
      }
      uw[UL::DEPTH] = udepth;
      uw[UL::DLEN] = ulen;
#pragma unroll
      for (int i = 0; i < OW && UL::ORD + i < UW; ++i) {  // bytes >= ulen are don't-care
        uint32_t word = DOW_(i);
        if (extra_b >= 0 && (uint32_t)i == (ol >> 2)) {
          const uint32_t sh = 8u * (ol & 3u);
          word = (word & ~(0xFFu << sh)) | ((uint32_t)extra_b << sh);
        }
        uw[UL::ORD + i] = word;
      }
      uint4* u4 = (uint4*)u;
#pragma unroll
      for (int q = 0; q < UW / 4; ++q) u4[q] = make_uint4(uw[4 * q], uw[4 * q + 1], uw[4 * q + 2], uw[4 * q + 3]);
      return;
    }
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      u[UL::T_ + w] = UT[w];
      u[UL::D_ + w] = UD[w];
      u[UL::K_ + w] = UK[w];
    }
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
  // a stack entry (T', D', packed) as a unit: the inclusion child it stands for
  auto write_entry = [&](uint32_t slot, const uint32_t (&ET)[MW], const uint32_t (&ED)[MW], uint32_t pk) {
    uint32_t UK[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) UK[w] = K[w];
    const uint32_t b = pk & 255u, de = (pk >> 8) & 511u, dle = pk >> 17;
    key_prefix_bit<MW>(UK, de);
    write_unit(slot, ET, ED, UK, de + 1, dle, (int)b);
  };
  auto write_lds_entry = [&](uint32_t slot, uint32_t pos) {
    uint32_t ET[MW], ED[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      ET[w] = ST_(pos, w);
      ED[w] = ST_(pos, MW + w);
    }
    write_entry(slot, ET, ED, ST_(pos, 2 * MW));
  };
  // a claimed but not installed unit goes back out unchanged, its record zeroed
  auto write_claimed = [&](uint32_t slot) {
    uint32_t* r = records + (size_t)fidx * RL::WORDS;
    if constexpr (WIDE && RL::WORDS % 2 == 0) {
#pragma unroll
      for (int w = 0; w < RL::WORDS; w += 2) *(uint2*)(r + w) = make_uint2(0u, 0u);
    } else {
#pragma unroll
      for (int w = 0; w < RL::WORDS; ++w) r[w] = 0u;
    }
    if (slot >= a.out_cap) {
      atomicOr(&a.glob[1], FLAG_OUT_OVERFLOW);
      return;
    }
    uint32_t* u = a.units_out + (size_t)slot * UW;
    if constexpr (WIDE) {
      uint4* u4 = (uint4*)u;
#pragma unroll
      for (int q = 0; q < UW / 4; ++q) u4[q] = make_uint4(fdat[4 * q], fdat[4 * q + 1], fdat[4 * q + 2], fdat[4 * q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < UW; ++q) u[q] = unit_word(q);
    }
  };

  // D is a minimal quorum (cpp:283-285): credit cpp:184, |D| x cpp:192 and the visitor
  // (cpp:368); VIS = GFP(scc \ D) with outside vertices available.  A non-empty VIS is a
  // disjoint quorum: record the witness, the unit ends here (cpp:369-377).
  auto minimal_quorum = [&](const uint32_t (&VIS)[MW], bool vis_any) {
    seg_evals += 2u + dlen;
    ++seg_minq;
    if (vis_any) {
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
      publish_best((unsigned long long)best_pack<MW>(K, depth));
      nst = 0;  // everything left in this unit follows the witness in preorder
      tvalid = false;
    }
  };

  // Claim the next units for the lanes that hold nothing (no node, no top entry, empty
  // stack), at the start of a full iteration; the units are installed at its end, so their
  // loads have the whole iteration to land before the install's vmcnt wait.  Indices come
  // from a wave-uniform pool of 64 claimed with one atomic (a returning atomic per
  // iteration would cost a memory round trip every iteration).  Convergent.
  auto claim = [&]() {
    // (claiming earlier, while a node or stack entries are still held, hoards units: the
    // queue runs dry sooner, 24 launches instead of 19 and 2.3 vs 1.87 ms per search)
    bool want = !done && !fpend && !has && !tvalid && nst == 0 && steps < limit;
    uint64_t wm = __ballot(want);
    while (wm) {
      if (pool_next >= pool_end) {
        if (pool_dead) break;
        uint32_t base = 0;
#if defined(QI_STAMPS) && QI_STAMP_SET == 3  // the wait for the queue head (stamp set 3)
        QI_STAMP(F_RESET);
#endif
        if (lane == 0) base = static_end + atomicAdd(&cc[C_HEAD], (uint32_t)WAVE);
        base = lane0(base);
#if defined(QI_STAMPS) && QI_STAMP_SET == 3
        QI_STAMP(F_W_CLAIM);
#endif
        if (base >= n_in) {
          pool_dead = true;
          // tell the waves that poll this line: no unit is left to claim in this launch
          if (lane == 0) __hip_atomic_store(my_rep + 2, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        pool_next = base;
        pool_end = min(base + (uint32_t)WAVE, n_in);
      }
      const uint32_t avail = pool_end - pool_next;
      const uint32_t r = rank_in(wm);
      if (want && r < avail) {
        fidx = pool_next + r;
        fpend = true;
        want = false;
        load_unit();
      }
      pool_next += min((uint32_t)__popcll(wm), avail);
      wm = __ballot(want);
    }
    if (pool_dead && !dry) {  // the queue ran out: grace period, then spill
      dry = true;
      QI_DIAG_MARK(diag_dry);
      limit = min(limit, steps + a.grace);
      force_at = wave_iters + a.grace;
    }
  };

  // A lane that holds nothing closes its segment (its unit's subtree is done) ...
  auto close_finished = [&]() {
    if (!done && !has && !tvalid && seg_open) close_segment();
  };
  // ... and installs its claimed unit.
  auto install_claimed = [&]() {
    if (!done && !has && !tvalid) {
      if (seg_open) close_segment();
      if (fpend && steps < limit) {
        QI_WAIT_STAMP("vmcnt(0)", F_W_INSTALL);
        uint32_t UK[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          T[w] = unit_word(UL::T_ + w);
          D[w] = unit_word(UL::D_ + w);
          UK[w] = unit_word(UL::K_ + w);
        }
        const uint32_t ud = unit_word(UL::DEPTH);
        dlen = unit_word(UL::DLEN);
        const uint32_t nw = (dlen + 3) / 4;
        if constexpr (OW <= 8) {
#pragma unroll
          for (int i = 0; i < OW; ++i)
            if ((uint32_t)i < nw) DOW_(i) = unit_word(UL::ORD + i);
        } else {
          for (uint32_t i = 0; i < nw; ++i) DOW_(i) = unit_word(UL::ORD + (int)i);
        }
        fpend = false;
        ++tot_fetched;
        seg_idx = fidx;
        seg_open = true;
        seg_s0 = steps;
        seg_evals = seg_minq = seg_zfb = 0;
#pragma unroll
        for (int w = 0; w < MW; ++w) seg_K[w] = K[w] = UK[w];
        seg_depth = depth = ud;
        nst = 0;
        sbase_ = 0;
        tvalid = false;
        // a unit past the best witness keeps its open, empty segment: the next close writes
        // its zero record
        has = !pruned(UK, ud);
      }
    }
  };

  install_claimed();  // the statically assigned first units
  for (;;) {
    QI_DIAG_MARK(diag_loop0);
    // ---- (0) fast steps: pop or process one node per lane, common outcomes only --------
    // A lane whose node is a quorum leaf (cpp:281) or whose push would need an eviction is
    // held, uncommitted, for the full iteration; lanes without node and stack wait there too.
    if ((QI_GROW_FAST || !exact_budget) && best64 == ~0ull && !(MW > 1 && a.has_best)) {
      bool hold = false;
      // (a growth launch's few lanes step while any of them can; its per-lane budget is exact,
      // and `steps < limit` keeps it so.  Run launches let lanes overshoot a grace-period limit
      // by a fast run: stopping them one by one would undo the wave's single spill)
      const uint32_t fast_min = exact_budget ? 1u : (dry ? (uint32_t)QI_FAST_MIN_DRY : (uint32_t)QI_FAST_MIN);
#pragma unroll 1
      for (int fs = 0; fs < QI_FAST_STEPS; ++fs) {
        const bool elig = !done && !hold && (has || tvalid) && (!exact_budget || steps < limit);
        if ((uint32_t)__popcll(__ballot(elig)) < fast_min) break;
        ++wave_iters;
        ++iter;
#ifdef QI_DIAG_FAST  // diagnostics: fast steps counted in the cooperative-phase counter
        ++coop_phases;
#endif
        if (elig && !has) {  // pop (no witness known: nothing to prune)
          const uint32_t b = tpk & 255u, de = (tpk >> 8) & 511u, dle = tpk >> 17;
          key_prefix_bit<MW>(K, de);
#pragma unroll
          for (int w = 0; w < MW; ++w) {
            T[w] = tT[w];
            D[w] = tD[w];
          }
          set_ord(dle, b);
          dlen = dle + 1;
          depth = de + 1;
          has = true;
          if (nst > 0) {
            --nst;
            const uint32_t pos = spos(nst);
#pragma unroll
            for (int w = 0; w < MW; ++w) {
              tT[w] = ST_(pos, w);
              tD[w] = ST_(pos, MW + w);
            }
            tpk = ST_(pos, 2 * MW);
          } else {
            tvalid = false;
          }
        }
        const bool full = tvalid && nst == (uint32_t)SMAX;  // a push would need an eviction
        uint32_t any = 0;
#pragma unroll
        for (int w = 0; w < MW; ++w) any |= T[w] | D[w];
        const bool leaf0 = dlen > a.half_m || !any;  // cpp:261 / cpp:266
        const bool ev = elig && !full && !leaf0;
        uint32_t X[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) X[w] = ev ? D[w] : 0u;
        const uint32_t r0 = rounds;
        const bool dq = EV::template gfp<0>(f, X, 0u, rounds);  // cpp:281
        if (dq) rounds = r0;  // re-evaluated (and counted) by the full iteration
        hold = hold || (elig && (full || dq));
        const bool go = elig && !full && !dq;  // this lane commits its node in this step
        const bool ev2 = go && !leaf0;
#pragma unroll
        for (int w = 0; w < MW; ++w) X[w] = ev2 ? (T[w] | D[w]) : 0u;
        const bool qne = EV::template gfp<0>(f, X, 0u, rounds);  // cpp:301
        if (go) {
          ++steps;
          if (leaf0) has = false;
        }
        if (ev2) {
          seg_evals += 2u;
          uint32_t dout = 0, qd = 0;
#pragma unroll
          for (int w = 0; w < MW; ++w) {
            dout |= D[w] & ~X[w];
            qd |= X[w] & ~D[w];
          }
          if (!qne || dout || !qd) {  // cpp:303, 308-314, 325
            has = false;
          } else {
            uint32_t pb;  // cpp:317
            if constexpr (TIE) pb = best_node_random<MW>(f, X, D, seg_zfb, tie_hash<MW>(a.tie_seed, K, depth));
            else pb = EV::best(f, X, D, seg_zfb);
#pragma unroll
            for (int w = 0; w < MW; ++w) X[w] &= ~D[w];
            X[pb >> 5] &= ~(1u << (pb & 31u));  // toRemove' = Q \ D \ {b} (cpp:330-334)
            if (tvalid) {  // the old top goes to LDS (room checked above)
              const uint32_t pos = spos(nst);
#pragma unroll
              for (int w = 0; w < MW; ++w) {
                ST_(pos, w) = tT[w];
                ST_(pos, MW + w) = tD[w];
              }
              ST_(pos, 2 * MW) = tpk;
              ++nst;
            }
#pragma unroll
            for (int w = 0; w < MW; ++w) {
              tT[w] = X[w];
              tD[w] = D[w];
              T[w] = X[w];
            }
            tD[pb >> 5] |= 1u << (pb & 31u);
            tpk = pb | (depth << 8) | (dlen << 17);
            tvalid = true;
            ++depth;  // continue with the exclusion branch (cpp:336)
          }
        }
      }
    }
    QI_STAMP(F_FAST);
    // the grace period of a dry wave is over: every lane spills in this iteration (per-lane
    // step limits alone would let lanes that idled during the grace period lag behind)
    if (wave_iters >= force_at) limit = 0;
    // (Before the claim: the compiler waits for every outstanding load where it copies the
    // polled registers, which after the claim would include the unit loads just issued.)
    // Poll this wave's line (loads issued one full iteration ahead): the best key, and
    // whether a wave sharing the line found the unit queue dry.  Once no unit is left to
    // claim, every lane gets a short grace period and then spills: the next launch spreads
    // the remaining subtrees over all lanes instead of letting a few lanes grind through
    // deep subtrees while the rest idle.
    if (poll_issued && iter >= next_poll) {
      poll_issued = false;
      next_poll = iter + (uint32_t)(QI_POLL_EVERY / QI_BEST_POLLS);
      uint32_t d = 0;
      uint64_t b = ~0ull;
      if (lane == 0) {
        d = poll_d;
        b = poll_b;
        if (forwarder && poll_x < b) {  // a key from another engine: into this device's words
          b = poll_x;
          publish_best(poll_x);
        }
      }
      d = lane0(d);
      best64 = lane0(b);
      const bool dry_poll = (poll_n++ % (uint32_t)QI_BEST_POLLS) == 0u;
      if (dry_poll && !dry && d == a.seq) {
        dry = true;
        QI_DIAG_MARK(diag_dry);
        limit = min(limit, steps + a.grace);
        force_at = wave_iters + a.grace;
      }
    } else if (!poll_issued && iter + 2u * ((uint32_t)QI_FAST_STEPS + 1u) >= next_poll) {
      // at least one full iteration before the poll that reads them
      poll_issued = true;
      if (lane == 0) issue_poll();
    }
    ++iter;
    QI_STAMP(F_POLL);
    // Claim units for the lanes that ran out during the fast steps; the loads have this
    // whole iteration to land: the units are installed at its end, so the lanes go into the
    // next fast steps with a node.  (Record stores follow the loads: vmcnt counts both in
    // issue order.)
    claim();
    QI_STAMP(F_CLAIM);
    flush_record();
    QI_STAMP(F_FLUSH);
    // ---- (1) lanes without a node: pop the top of stack (units are installed at the end) ----
    if (!done && !has) {
      if (tvalid) {
        const uint32_t b = tpk & 255u, de = (tpk >> 8) & 511u, dle = tpk >> 17;
        uint32_t NK[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) NK[w] = K[w];
        key_prefix_bit<MW>(NK, de);
        if (pruned(NK, de + 1)) {  // deeper entries precede shallower ones: drop all
          tvalid = false;
          nst = 0;
        } else {
#pragma unroll
          for (int w = 0; w < MW; ++w) {
            T[w] = tT[w];
            D[w] = tD[w];
            K[w] = NK[w];
          }
          set_ord(dle, b);
          dlen = dle + 1;
          depth = de + 1;
          has = true;
          if (nst > 0) {  // refill the top from LDS; first used at the next pop
            --nst;
            const uint32_t pos = spos(nst);
#pragma unroll
            for (int w = 0; w < MW; ++w) {
              tT[w] = ST_(pos, w);
              tD[w] = ST_(pos, MW + w);
            }
            tpk = ST_(pos, 2 * MW);
            QI_WAIT_STAMP("lgkmcnt(0)", F_W_POP);
          } else {
            tvalid = false;
          }
        }
      }
      QI_STAMP(F_POP);
    }
    // (a lane that finished during the fast steps may be found done just below: its
    // segment closes here)
    close_finished();
    QI_STAMP(F_INSTALL);
    // a lane with nothing left is done once it cannot get a unit any more (a claimed unit
    // past the budget is spilled below)
    if (!has && !tvalid && nst == 0 && !fpend && (steps >= limit || pool_dead)) done = true;

    // ---- (3) budget exhausted: spill current node, top, stack and claimed unit ---------
    {
      const bool spill = (has && (steps >= limit || must_spill)) || (!has && fpend && steps >= limit);
      if (__any(spill)) {
        QI_DIAG_MARK(diag_sp0);
        uint32_t total = 0;
        const uint32_t n = spill ? (has ? 1u : 0u) + (tvalid ? 1u : 0u) + nst + (fpend ? 1u : 0u) : 0u;
        uint32_t slot = reserve<RB>(n, &cc[C_OUT], total);
        QI_DIAG_MARK(diag_spr);
        if (spill) {
          if (has) write_unit(slot++, T, D, K, depth, dlen, -1);
          if (tvalid) write_entry(slot++, tT, tD, tpk);
          for (uint32_t i = nst; i > 0; --i) write_lds_entry(slot++, spos(i - 1));
          if (fpend) write_claimed(slot++);
          nst = 0;
          tvalid = false;
          fpend = false;
          if (seg_open) close_segment();
          has = false;
          done = true;
        }
#ifdef QI_DIAG_LAUNCH
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        diag_sp1 = (uint32_t)__builtin_amdgcn_s_memrealtime() | 1u;
#endif
      }
    }
    if (!__any(!done)) break;

    QI_STAMP(F_SPILL);
    // ---- (4) one search node per active lane (cpp:258-345) ---------------------------
    ++wave_iters;
    bool pending = false;
    bool active = has;
    if (active) {
      ++steps;
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
    QI_STAMP(F_GFP1);
#pragma unroll
    for (int w = 0; w < MW; ++w) X[w] = active2 ? (T[w] | D[w]) : 0u;
    const bool qne = EV::template gfp<0>(f, X, 0u, rounds);  // cpp:301
    QI_STAMP(F_GFP2);
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
        if constexpr (TIE) pb = best_node_random<MW>(f, X, D, seg_zfb, tie_hash<MW>(a.tie_seed, K, depth));
        else pb = EV::best(f, X, D, seg_zfb);  // cpp:317
#pragma unroll
        for (int w = 0; w < MW; ++w) X[w] &= ~D[w];
        X[pb >> 5] &= ~(1u << (pb & 31u));  // toRemove' = Q \ D \ {b} (cpp:330-334)
        push = true;
      }
    }
    QI_STAMP(F_BEST);
    // push the inclusion branch (cpp:343-345): the old top goes to LDS (a full stack
    // first evicts its shallowest entry into the next frontier; wave-aggregated slot
    // reservation, convergent), the new entry becomes the top.  Then continue with the
    // exclusion branch (cpp:336): same D, T = T', key bit 0.
    {
      const bool evict = push && tvalid && nst == (uint32_t)SMAX;
      if (__any(evict)) {
        const uint64_t em = __ballot(evict);
        uint32_t tok = 0;
        if (lane == 0) tok = atomicAdd(&cc[C_EVX], (uint32_t)__popcll(em));
        tok = lane0(tok);
        const bool granted = evict && tok + rank_in(em) < evict_pool;
        const bool forced = evict && !granted;  // no pool slot: the old top leaves through this lane's spill reserve
        uint32_t total = 0;
        const uint32_t slot = reserve<1>(evict ? 1u : 0u, &cc[C_OUT], total);
        if (granted) {
          write_lds_entry(slot, spos(0));
          sbase_ = spos(1);
          --nst;
        } else if (forced) {
          write_entry(slot, tT, tD, tpk);
          tvalid = false;
          must_spill = true;
          atomicOr(&a.glob[1], FLAG_POOL);
        }
      }
      if (push) {
        if (tvalid) {
          const uint32_t pos = spos(nst);
#pragma unroll
          for (int w = 0; w < MW; ++w) {
            ST_(pos, w) = tT[w];
            ST_(pos, MW + w) = tD[w];
          }
          ST_(pos, 2 * MW) = tpk;
          ++nst;
        }
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          tT[w] = X[w];
          tD[w] = D[w];
          T[w] = X[w];
        }
        tD[pb >> 5] |= 1u << (pb & 31u);
        tpk = pb | (depth << 8) | (dlen << 17);
        tvalid = true;
        ++depth;
      }
    }

    QI_STAMP(F_PUSH);
    // ---- (5) quorum leaves: isMinimalQuorum + visitor ---------------------------------
    // Quorum leaves with |D| - 1 < qmin: no D \ {v} can hold a quorum (LocalFlat::qmin),
    // so D is minimal without evaluating them (still credited, as the reference makes the
    // calls); only the visitor's fixpoint remains, evaluated here per lane.
    {
      const bool fastp = pending && dlen < EV::qmin0(f) + 1u;
      if (__any(fastp)) {
        uint32_t Y[MW];
        uint32_t vany = 0;
#pragma unroll
        for (int w = 0; w < MW; ++w) Y[w] = fastp ? (EV::scc_word(f, w) & ~D[w]) : 0u;
        EV::template gfp<1>(f, Y, 1u, rounds);  // visitor: scc \ Q, outside available
#pragma unroll
        for (int w = 0; w < MW; ++w) vany |= Y[w];
        if (fastp) {
          has = false;
          pending = false;
          minimal_quorum(Y, vany != 0u);
        }
      }
    }
    QI_STAMP(F_FASTP);
#if QI_FASTMIN
    // Quorum leaves with |D| = qmin + 1: every D \ {v} has qmin vertices, so it holds a
    // quorum iff it is a fixpoint itself, which one removal-sensitivity pass decides for
    // all v at once (EV::min_bad: the v whose removal unsatisfies some remaining member).
    // isMinimal's first hit (cpp:188-198) is the first D-order position of a v not in bad;
    // none means D is minimal, and only then does the visitor's fixpoint run (cpp:368).
    // Credited evals as in the cooperative phase.  No cooperative phase for these leaves.
    if constexpr (EV::FASTMIN) {
      const bool fm = pending && dlen == EV::qmin0(f) + 1u;
      if (__any(fm)) {
        uint32_t Xd[MW], bad[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) Xd[w] = fm ? D[w] : 0u;
        EV::min_bad(f, Xd, bad);
        bool minimal = false;
        if (fm) {
          uint32_t ow[OW];
#pragma unroll
          for (int i = 0; i < OW; ++i) ow[i] = DOW_(i);
          uint32_t goodpos = 0;  // bit i: the i-th vertex of the D order is removable
          if constexpr (MW == 1) {
            const uint32_t good = ~bad[0];
#pragma unroll
            for (int i = 0; i < OW * 4; ++i)  // v_bfe + v_lshrrev + v_and + v_lshl_or per position
              goodpos |= ((good >> ((ow[i >> 2] >> (8 * (i & 3))) & 31u)) & 1u) << i;
          } else {
#pragma unroll
            for (int i = 0; i < OW * 4; ++i) {
              const uint32_t v = (ow[i >> 2] >> (8 * (i & 3))) & 255u;
              uint32_t bw = bad[0];
#pragma unroll
              for (int w = 1; w < MW; ++w) bw = (v >> 5) == (uint32_t)w ? bad[w] : bw;
              goodpos |= (((bw >> (v & 31u)) & 1u) ^ 1u) << i;
            }
          }
          goodpos &= dlen >= 32u ? 0xFFFFFFFFu : ((1u << dlen) - 1u);
          if (goodpos) {  // not minimal: isMinimal stops at the first removable vertex
            seg_evals += 2u + (uint32_t)__builtin_ctz(goodpos);  // cpp:184 + (pos+1) x cpp:192
            has = false;
            pending = false;
          } else {
            minimal = true;
          }
        }
        if (__any(minimal)) {
          uint32_t Y[MW];
          uint32_t vany = 0;
#pragma unroll
          for (int w = 0; w < MW; ++w) Y[w] = minimal ? (EV::scc_word(f, w) & ~D[w]) : 0u;
          EV::template gfp<1>(f, Y, 1u, rounds);  // visitor: scc \ Q, outside available
#pragma unroll
          for (int w = 0; w < MW; ++w) vany |= Y[w];
          if (minimal) {
            has = false;
            pending = false;
            minimal_quorum(Y, vany != 0u);
          }
        }
      }
    }
#endif
    // Remaining quorum leaves (|D| >= qmin + 2), wave-cooperative: every pending lane needs
    // |D| single-removal fixpoints (isMinimalQuorum, cpp:188-198) and the complement check
    // of the visitor (cpp:368).  Done per lane they would serialise the wave (the first
    // removable vertex sits at a ~uniform position of the D order), so they are spread over
    // the wave in fixed slots of S = a.coop_slot lanes per pending lane: lane l serves owner
    // (l / S) of the current pass, job k = l % S (+ chunk offset when |D|+1 > S).  The
    // owner's D, lane and |D| arrive through an LDS slot, results by one LDS ds_or per
    // successful job.
    QI_STAMP(F_FASTMIN);
    const uint64_t pm = __ballot(pending);
    if (pm) {
      ++coop_phases;
      const uint32_t npend = (uint32_t)__popcll(pm);
      const uint32_t r = rank_in(pm);
      const uint32_t S = a.coop_slot, lgS = a.coop_slot_log2;
      const uint32_t P = (uint32_t)WAVE >> lgS;  // owners per pass
      if (pending) {  // owner slot r: results zeroed, D / lane / |D| published
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          co_NE[w * WAVE + r] = 0u;
          co_VIS[w * WAVE + r] = 0u;
          co_D[w * WAVE + r] = D[w];
        }
        co_OWN[r] = lane | (dlen << 8);
      }
      __syncthreads();
      for (uint32_t q0 = 0; q0 < npend; q0 += P) {
        const uint32_t oi = q0 + (lane >> lgS);
        const uint32_t oc = min(oi, (uint32_t)WAVE - 1u);  // slots >= npend: stale, masked by `act`
        const uint32_t own = co_OWN[oc];
        const uint32_t ol = own & 63u, dl = own >> 8;
        uint32_t Dr[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) Dr[w] = co_D[w * WAVE + oc];
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
            else if (vis) Y[w] = EV::scc_word(f, w) & ~Dr[w];  // visitor: scc \ Q, outside available
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
          minimal_quorum(VIS, vis_any != 0u);
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
    QI_STAMP(F_COOP);
    install_claimed();
    QI_STAMP(F_INSTALL);
  }
  flush_record();

  // indices of this wave's pool that no lane took: carry the units over unchanged
  if (pool_next < pool_end) {
    const uint32_t left = pool_end - pool_next;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&cc[C_OUT], left);
    base = lane0(base);
    for (uint32_t i = lane; i < left; i += WAVE) {
      const uint32_t src = pool_next + i, dst = base + i;
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
    atomicAdd(&tt[14], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - wave_t0));  // 100 MHz ticks
    atomicAdd(&tt[15], 1ull);                                                           // waves
#endif
  }

#ifdef QI_DIAG_WAVES  // diagnostics without atomics: this wave's timestamps, one plain 16-byte store
  if (lane == 0 && a.diag_waves) {
    (void)diag_spr; (void)diag_sp1; (void)diag_loop0;
    *(uint4*)(a.diag_waves + (size_t)blockIdx.x * 4) =
        make_uint4(diag_t0, diag_dry, diag_sp0, (uint32_t)__builtin_amdgcn_s_memrealtime());
  }
#endif
#ifdef QI_DIAG_LAUNCH
  if (lane == 0) {
    const uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    atomicMax(&cc[C_DIAG], wave_iters);
    atomicAdd(&cc[C_DIAG + 1], t1 - diag_t0);
    atomicMax(&cc[C_DIAG + 2], t1 - diag_t0);
    atomicMax(&cc[C_DIAG + 3], ~diag_t0);
    atomicMax(&cc[C_DIAG + 4], t1);
    // phase sums over the waves that went dry and spilled: start -> loop, loop -> dry,
    // dry -> first spill, spill (slot reservation + unit stores), last spill -> end
    if (diag_dry && diag_sp0 && diag_sp1) {
      atomicAdd(&cc[C_DIAG + 5], 1u);
      atomicAdd(&cc[C_DIAG + 6], diag_loop0 - diag_t0);
      atomicAdd(&cc[C_DIAG + 7], diag_dry - diag_loop0);
      atomicAdd(&cc[C_DIAG + 8], diag_sp0 - diag_dry);
      atomicAdd(&cc[C_DIAG + 9], diag_sp1 - diag_sp0);
      atomicAdd(&cc[C_DIAG + 10], t1 - diag_sp1);
      atomicAdd(&cc[C_DIAG + 11], diag_spr - diag_sp0);  // of the spill: waiting for the slot reservation
    }
  }
#endif
  // ---- last block of the launch: carry over never-claimed input units (whose waves all
  // hit their budget before the queue ran dry) with zeroed records, publish the counters.
  // Every counter read here is an atomic RMW, performed after the other blocks' returned
  // atomics; nothing the other blocks stored plainly is read.
  {
    uint32_t old = 0;
    if (lane == 0) old = atomicAdd(&cc[C_DONE], 1u);
    old = lane0(old);
    if (old == nb_used - 1u) {
      uint32_t hd = 0, out = 0;
      if (lane == 0) {
        hd = atomicAdd(&cc[C_HEAD], 0u);
        out = atomicAdd(&cc[C_OUT], 0u);
        // this launch's best key for the host (folded into the engines' shared word)
        const unsigned long long bb = atomicMin(a.best64, ~0ull);
        a.host_ctr[HC_BEST] = (uint32_t)bb;
        a.host_ctr[HC_BEST + 1] = (uint32_t)(bb >> 32);
      }
#ifdef QI_DIAG_LAUNCH  // diagnostics: running node / wave-iteration totals after this launch (low words)
      {
        unsigned long long dn = atomicAdd(&a.totals[(size_t)lane * 16 + 0], 0ull);
        unsigned long long di = atomicAdd(&a.totals[(size_t)lane * 16 + 6], 0ull);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          dn += __shfl_xor(dn, d);
          di += __shfl_xor(di, d);
        }
        if (lane == 0) {
          a.host_ctr[HC_DIAG] = (uint32_t)dn;
          a.host_ctr[HC_DIAG + 1] = (uint32_t)di;
          a.host_ctr[HC_DIAG + 2] = atomicAdd(&cc[C_DIAG], 0u);
          a.host_ctr[HC_DIAG + 3] = atomicAdd(&cc[C_DIAG + 1], 0u);
          a.host_ctr[HC_DIAG + 4] = atomicAdd(&cc[C_DIAG + 2], 0u);
          a.host_ctr[HC_DIAG + 5] = atomicAdd(&cc[C_DIAG + 4], 0u) + atomicAdd(&cc[C_DIAG + 3], 0u) + 1u;  // end - start
          for (int q = 0; q < 7; ++q) a.host_ctr[HC_DIAG + 6 + q] = atomicAdd(&cc[C_DIAG + 5 + q], 0u);
        }
      }
#endif
      hd = lane0(hd);
      out = lane0(out);
      const uint32_t lane0_out = out;
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
        // never-claimed units: the global queue outlived every lane's node budget
        cc[C_HALT] = left ? 1u : 0u;
        a.host_ctr[HC_HALT] = left ? 1u : 0u;
        out += left;
        if (out != lane0_out) atomicExch(&cc[C_OUT], out);
        cc[C_LOGN] = log_base + n_in;
        a.host_ctr[HC_LOGN] = log_base + n_in;
        a.host_ctr[HC_OUT] = out;
        a.host_ctr[HC_NIN] = n_in;
        a.host_ctr[HC_LOGB] = log_base;
        a.host_ctr[HC_STOP] = 0u;
        a.host_ctr[HC_DONE] = 1u;
        publish_flag(a.host_ctr, false, out);
      }
    }
  }
#undef ST_
#undef ST_IDX
#undef DOW_
}

}  // namespace dev
}  // namespace qi
