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

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "qi_device.h"
#include "../../include/quorum_intersection.h"

namespace qi {

#define HIP_CHECK(x)                                                                        \
  do {                                                                                      \
    hipError_t e__ = (x);                                                                   \
    if (e__ != hipSuccess)                                                                  \
      throw Error(QI_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e__));          \
  } while (0)

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

struct SearchArgs {
  LocalDev f;
  const uint32_t* units_in;
  uint32_t n_in;
  uint32_t* units_out;
  uint32_t out_cap;
  uint32_t* counters;            // [0] out_count [1] head [2] wit_count [3] flags
  uint32_t* records;             // [n_in][RecLayout::WORDS]
  uint32_t* wit;
  uint32_t wit_cap;
  unsigned long long* totals;    // nodes, evals, minq, zero_fallback, rounds, units_fetched
  unsigned long long* best64;    // exact preorder key when MW == 1
  uint32_t budget;
  uint32_t grace;                // extra steps per lane once the unit queue is dry
  uint32_t evict_max;
  uint32_t half_m;
  uint32_t has_best;             // host-known best key (multiword) for pruning
  uint32_t best_depth;
  uint32_t best_key[8];
  uint32_t scc_mask[8];
};

enum : uint32_t { FLAG_OUT_OVERFLOW = 1u, FLAG_WIT_OVERFLOW = 2u };

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

template <int MW, int TW, int SMAX>
__global__ __launch_bounds__(64) void search_kernel(SearchArgs a) {
  using UL = UnitLayout<MW>;
  using RL = RecLayout<MW>;
  using WL = WitLayout<MW>;
  constexpr int DMAX = UL::DMAX;
  constexpr int UW = UL::WORDS;
  constexpr int SE = MW + 1;  // stack entry words: T'[MW], packed(b, depth, dlen)

  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* st = lds;                                          // [SMAX][SE][64]
  uint32_t* co_D = st + SMAX * SE * WAVE;                       // [MW][64]
  uint32_t* co_NE = co_D + MW * WAVE;                           // [MW][64]
  uint32_t* co_VIS = co_NE + MW * WAVE;                         // [MW][64]
  uint32_t* co_off = co_VIS + MW * WAVE;                        // [65] (+pad)
  uint32_t* uring = co_off + 68;                                // [UW][64] staged units
  uint8_t* dord = (uint8_t*)(uring + UW * WAVE);                // [DMAX][64]

  const uint32_t lane = threadIdx.x;
  const LocalDev& f = a.f;
#define ST_(lvl, w) st[((lvl) * SE + (w)) * WAVE + lane]
#define DO_(i) dord[(i) * WAVE + lane]
#define UR_(w, slot) uring[(w) * WAVE + (slot)]

  uint32_t T[MW], D[MW], K[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) T[w] = D[w] = K[w] = 0;
  uint32_t depth = 0, dlen = 0;
  bool has = false, done = false;
  uint32_t nst = 0, sbase = 0;
  uint32_t steps = 0, evictions = 0;
  uint32_t limit = a.budget;  // per-lane step limit; shrinks to steps+grace when the queue dries
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

  // wave-uniform LDS ring of staged units (see (2) below)
  uint32_t ring_src = 0, ring_cnt = 0, ring_next = 0;
  bool ring_dead = false;
  uint64_t best64 = ~0ull;
  auto refill = [&](uint32_t base) {  // convergent: every lane stages one unit
    const uint32_t cnt = min(a.n_in - base, (uint32_t)WAVE);
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
  if (blockIdx.x * WAVE < a.n_in) refill(blockIdx.x * WAVE);
  else ring_dead = true;

  auto close_segment = [&]() {
    uint32_t* r = a.records + (size_t)seg_idx * RL::WORDS;
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
    if (MW == 1) p = p || ((((uint64_t)KK[0] << 32) | d) > best64);
    return p;
  };

  // write one unit (T, D given as masks, order = dord[0..ol) + optional extra byte)
  auto write_unit = [&](uint32_t slot, const uint32_t (&UT)[MW], const uint32_t (&UD)[MW], const uint32_t (&UK)[MW],
                        uint32_t udepth, uint32_t ol, int extra_b) {
    if (slot >= a.out_cap) {
      atomicOr(&a.counters[3], FLAG_OUT_OVERFLOW);
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
    for (uint32_t i = 0; i < (uint32_t)(DMAX + 3) / 4; ++i) {
      uint32_t word = 0;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t p = i * 4 + j;
        uint32_t byte = 0;
        if (p < ol) byte = DO_(p);
        else if (p == ol && extra_b >= 0) byte = (uint32_t)extra_b;
        word |= byte << (8 * j);
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
    for (uint32_t i = 0; i < dle; ++i) {
      const uint32_t v = DO_(i);
      UD[v >> 5] |= 1u << (v & 31u);
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
        for (uint32_t i = dle; i < dlen; ++i) {
          const uint32_t v = DO_(i);
          D[v >> 5] &= ~(1u << (v & 31u));
        }
        D[b >> 5] |= 1u << (b & 31u);
        DO_(dle) = (uint8_t)b;
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
        if (lane == 0) base = atomicAdd(&a.counters[1], (uint32_t)WAVE);
        base = __shfl(base, 0);
        if (base >= a.n_in) {
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
        for (uint32_t i = 0; i < (dlen + 3) / 4; ++i) {
          const uint32_t word = UR_(UL::ORD + i, slot);
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            if (i * 4 + j < dlen) DO_(i * 4 + j) = (uint8_t)(word >> (8 * j));
        }
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
        h = __hip_atomic_load(&a.counters[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (MW == 1) b = __hip_atomic_load(a.best64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      h = __shfl(h, 0);
      best64 = __shfl(b, 0);
      if (!dry && (ring_dead || h >= a.n_in)) {
        dry = true;
        limit = min(limit, steps + a.grace);
      }
    }

    // ---- (3) budget exhausted: spill current node + stack to the next frontier --------
    {
      const bool spill = has && (steps >= limit || evictions >= a.evict_max);
      if (__any(spill)) {
        uint32_t total = 0;
        const uint32_t n = spill ? 1u + nst : 0u;
        uint32_t slot = reserve(n, &a.counters[0], total);
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
    const bool dq = gfp<MW, TW, 0>(f, X, 0u, rounds);  // cpp:281
    if (active) {
      ++seg_evals;
      pending = dq;
    }
    const bool active2 = active && !dq;
#pragma unroll
    for (int w = 0; w < MW; ++w) X[w] = active2 ? (T[w] | D[w]) : 0u;
    const bool qne = gfp<MW, TW, 0>(f, X, 0u, rounds);  // cpp:301
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
        pb = best_node<MW>(f, X, D, seg_zfb);  // cpp:317
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
        const uint32_t slot = reserve(evict ? 1u : 0u, &a.counters[0], total);
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

    // ---- (5) quorum leaves: isMinimalQuorum + visitor, wave-cooperative --------------
    const uint64_t pm = __ballot(pending);
    if (pm) {
      ++coop_phases;
      const uint32_t npend = (uint32_t)__popcll(pm);
      const uint32_t r = rank_in(pm);
      uint32_t nj = pending ? dlen + 1u : 0u;
      uint32_t x = nj;
#pragma unroll
      for (int d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if ((int)lane >= d) x += y;
      }
      const uint32_t J = __shfl(x, WAVE - 1);
      if (pending) {
        co_off[r] = x - nj;
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          co_D[w * WAVE + r] = D[w];
          co_NE[w * WAVE + r] = 0u;
          co_VIS[w * WAVE + r] = 0u;
        }
      }
      if (lane == 0) co_off[npend] = J;
      __syncthreads();
      for (uint32_t j0 = 0; j0 < J; j0 += WAVE) {
        const uint32_t j = j0 + lane;
        const bool act = j < J;
        uint32_t lo = 0;
        if (act) {
          uint32_t hi = npend - 1;
          while (lo < hi) {  // last owner with co_off[o] <= j
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (co_off[mid] <= j) lo = mid;
            else hi = mid - 1;
          }
        }
        const uint32_t o = lo;
        uint32_t Dr[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) Dr[w] = act ? co_D[w * WAVE + o] : 0u;
        const uint32_t k = act ? j - co_off[o] : 0u;
        const uint32_t dl = act ? co_off[o + 1] - co_off[o] - 1u : 0u;
        const bool vis = act && k == dl;
        uint32_t v = 0;
        if (act && !vis) {  // k-th member of D in index order
          uint32_t kk = k;
          bool found = false;
#pragma unroll
          for (int w = 0; w < MW; ++w) {
            uint32_t c = Dr[w];
            const uint32_t pc = (uint32_t)__popc(c);
            if (!found && kk < pc) {
              for (uint32_t i = 0; i < kk; ++i) c &= c - 1u;
              v = (uint32_t)w * 32u + (uint32_t)__builtin_ctz(c);
              found = true;
            } else if (!found) {
              kk -= pc;
            }
          }
        }
        uint32_t Y[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) {
          if (!act) Y[w] = 0u;
          else if (vis) Y[w] = a.scc_mask[w] & ~Dr[w];   // visitor: scc \ Q, outside available
          else Y[w] = Dr[w];
        }
        if (act && !vis) Y[v >> 5] &= ~(1u << (v & 31u));  // isMinimal: D \ {v}
        const bool ne = gfp<MW, TW, 2>(f, Y, vis ? 1u : 0u, rounds);
        if (act && !vis && ne) atomicOr(&co_NE[(v >> 5) * WAVE + o], 1u << (v & 31u));
        if (vis) {
#pragma unroll
          for (int w = 0; w < MW; ++w) co_VIS[w * WAVE + o] = Y[w];
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
            const uint32_t slot = atomicAdd(&a.counters[2], 1u);
            if (slot < a.wit_cap) {
              uint32_t* wv = a.wit + (size_t)slot * WL::WORDS;
#pragma unroll
              for (int w = 0; w < MW; ++w) {
                wv[w] = K[w];
                wv[MW + 2 + w] = VIS[w];
              }
              wv[MW] = depth;
              wv[MW + 1] = dlen;
              for (uint32_t i = 0; i < (uint32_t)WL::ORDW; ++i) {
                uint32_t word = 0;
#pragma unroll
                for (uint32_t jj = 0; jj < 4; ++jj)
                  if (i * 4 + jj < dlen) word |= (uint32_t)DO_(i * 4 + jj) << (8 * jj);
                wv[2 * MW + 2 + i] = word;
              }
            } else {
              atomicOr(&a.counters[3], FLAG_WIT_OVERFLOW);
            }
            if (MW == 1) atomicMin(a.best64, ((unsigned long long)K[0] << 32) | depth);
            nst = 0;  // everything left in this unit follows the witness in preorder
          }
        } else {  // not minimal: isMinimal stops at the first removable vertex in D order
          uint32_t pos = 0;
          for (uint32_t i = 0; i < dlen; ++i) {
            const uint32_t v = DO_(i);
            if ((NE[v >> 5] >> (v & 31u)) & 1u) {
              pos = i;
              break;
            }
          }
          seg_evals += 2u + pos;  // cpp:184 + (pos+1) x cpp:192
        }
      }
      __syncthreads();
    }
  }

  // units claimed by this wave's ring but never fetched: carry them over unchanged
  {
    const uint32_t ring_pos = ring_src + ring_next;
    const uint32_t left = (ring_next < ring_cnt) ? ring_cnt - ring_next : 0u;
    if (left) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&a.counters[0], left);
      base = __shfl(base, 0);
      for (uint32_t i = lane; i < left; i += WAVE) {
        const uint32_t src = ring_pos + i, dst = base + i;
        uint32_t* r = a.records + (size_t)src * RL::WORDS;
        for (int w = 0; w < RL::WORDS; ++w) r[w] = 0u;
        if (dst < a.out_cap) {
          const uint4* s4 = (const uint4*)(a.units_in + (size_t)src * UW);
          uint4* d4 = (uint4*)(a.units_out + (size_t)dst * UW);
          for (int q = 0; q < UW / 4; ++q) d4[q] = s4[q];
        } else {
          atomicOr(&a.counters[3], FLAG_OUT_OVERFLOW);
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
  if (lane == 0) {
    atomicAdd(&a.totals[0], (unsigned long long)tot_nodes);
    atomicAdd(&a.totals[1], (unsigned long long)tot_evals);
    atomicAdd(&a.totals[2], (unsigned long long)tot_minq);
    atomicAdd(&a.totals[3], (unsigned long long)tot_zfb);
    atomicAdd(&a.totals[4], (unsigned long long)tr);
    atomicAdd(&a.totals[5], (unsigned long long)tot_fetched);
    atomicAdd(&a.totals[6], (unsigned long long)wave_iters);
    atomicAdd(&a.totals[7], (unsigned long long)coop_phases);
  }
#undef ST_
#undef DO_
#undef UR_
}

// Zero-record the units never claimed from the global head (host carries them over).
template <int MW>
__global__ void zero_records_kernel(uint32_t* records, uint32_t from, uint32_t to) {
  const uint32_t i = from + blockIdx.x * blockDim.x + threadIdx.x;
  if (i < to) {
    uint32_t* r = records + (size_t)i * RecLayout<MW>::WORDS;
    for (int w = 0; w < RecLayout<MW>::WORDS; ++w) r[w] = 0u;
  }
}

// Preorder-filtered sums over a log chunk: segment roots at or before (key, depth).
template <int MW>
__global__ void reduce_kernel(const uint32_t* records, uint64_t n, uint32_t has_key, const uint32_t* key,
                              uint32_t depth, unsigned long long* out) {
  uint64_t s[4] = {0, 0, 0, 0};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t* r = records + i * RecLayout<MW>::WORDS;
    uint32_t K[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) K[w] = r[w];
    if (has_key && after_key<MW>(K, r[MW], key, depth)) continue;
    s[0] += r[MW + 1];
    s[1] += r[MW + 2];
    s[2] += r[MW + 3];
    s[3] += r[MW + 4];
  }
  for (int q = 0; q < 4; ++q) {
    uint64_t v = s[q];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&out[q], (unsigned long long)v);
  }
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

__global__ __launch_bounds__(64) void gfp_batch_kernel(GlobalDev g, const unsigned long long* nodes,
                                                        const unsigned long long* avail, uint32_t count,
                                                        unsigned long long* out, unsigned long long* rounds_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm[];
  unsigned long long* A = sm;             // [words] available set (changes as X shrinks)
  unsigned long long* X = A + g.words;    // [words] current candidates
  uint8_t* sat = (uint8_t*)(X + g.words); // [T]
  const uint32_t lane = threadIdx.x;
  const uint32_t q = blockIdx.x;
  if (q >= count) return;
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

// =====================================================================================
// Host-side device management
// =====================================================================================
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

namespace {

template <typename T>
T* dalloc(size_t count) {
  void* p = nullptr;
  if (count == 0) count = 1;
  HIP_CHECK(hipMalloc(&p, count * sizeof(T)));
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

class GfpDeviceImpl : public GfpDevice {
 public:
  GfpDeviceImpl(int device, const GlobalFlat& g) : device_(device) {
    DeviceGuard dg(device_);
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&e0_));
    HIP_CHECK(hipEventCreate(&e1_));
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
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  ~GfpDeviceImpl() override {
    DeviceGuard dg(device_);
    for (auto* p : bufs_) (void)hipFree((void*)p);
    (void)hipFree(rounds_);
    (void)hipFree(io_);
    (void)hipEventDestroy(e0_);
    (void)hipEventDestroy(e1_);
    (void)hipStreamDestroy(stream_);
  }
  void run(const uint64_t* nodes, const uint64_t* avail, uint32_t count, uint64_t* out) override {
    if (count == 0) return;
    DeviceGuard dg(device_);
    const size_t per = (size_t)count * d_.words;
    if (io_cap_ < per) {
      (void)hipFree(io_);
      io_ = dalloc<unsigned long long>(3 * per);
      io_cap_ = per;
    }
    unsigned long long* dn = io_;
    unsigned long long* da = io_ + per;
    unsigned long long* dout = io_ + 2 * per;
    HIP_CHECK(hipMemcpyAsync(dn, nodes, per * 8, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(da, avail, per * 8, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemsetAsync(rounds_, 0, 8, stream_));
    const size_t shm = (size_t)d_.words * 16 + ((d_.T + 15) / 16) * 16;
    if (shm > 160 * 1024) throw Error(QI_ERR_UNSUPPORTED, "gfp_batch: FBAS too large for LDS staging");
    HIP_CHECK(hipEventRecord(e0_, stream_));
    hipLaunchKernelGGL(dev::gfp_batch_kernel, dim3(count), dim3(64), shm, stream_, d_, dn, da, count, dout, rounds_);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(e1_, stream_));
    HIP_CHECK(hipMemcpyAsync(out, dout, per * 8, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0_, e1_));
    last_ms_ = ms;
  }
  double last_kernel_ms() const override { return last_ms_; }

 private:
  int device_;
  hipStream_t stream_{};
  hipEvent_t e0_{}, e1_{};
  dev::GlobalDev d_{};
  std::vector<const uint32_t*> bufs_;
  unsigned long long* rounds_ = nullptr;
  unsigned long long* io_ = nullptr;
  size_t io_cap_ = 0;
  double last_ms_ = 0;
};

template <int MW, int TW, int SMAX>
class SearchDeviceImpl : public SearchDevice {
  using UL = dev::UnitLayout<MW>;
  using RL = dev::RecLayout<MW>;
  using WL = dev::WitLayout<MW>;

 public:
  SearchDeviceImpl(int device, const LocalFlat& f, const SearchConfig& cfg) : device_(device), cfg_(cfg), m_(f.m) {
    DeviceGuard dg(device_);
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&e0_));
    HIP_CHECK(hipEventCreate(&e1_));
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
    for (uint32_t w = 0; w < 8; ++w) scc_mask_[w] = 0;
    for (uint32_t v = 0; v < f.m; ++v) scc_mask_[v >> 5] |= 1u << (v & 31);

    int cus = device_cu_count(device_);
    max_blocks_ = cfg_.max_blocks ? cfg_.max_blocks : (uint32_t)cus * 8u;
    counters_ = dalloc<uint32_t>(4);
    totals_ = dalloc<unsigned long long>(8);
    best64_ = dalloc<unsigned long long>(1);
    red_ = dalloc<unsigned long long>(4);
    keydev_ = dalloc<uint32_t>(8);
    wit_cap_ = 1u << 16;
    wit_ = dalloc<uint32_t>((size_t)wit_cap_ * WL::WORDS);
    HIP_CHECK(hipMemsetAsync(totals_, 0, 8 * sizeof(unsigned long long), stream_));
    unsigned long long inf = ~0ull;
    HIP_CHECK(hipMemcpyAsync(best64_, &inf, 8, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    shm_ = (size_t)(SMAX * (MW + 1) * 64 + 3 * MW * 64 + 68 + UL::WORDS * 64) * 4 + (size_t)UL::DMAX * 64;
    shm_ = (shm_ + 15) / 16 * 16;
    HIP_CHECK(hipFuncSetAttribute((const void*)dev::search_kernel<MW, TW, SMAX>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm_));
    reset_root();
  }

  ~SearchDeviceImpl() override {
    DeviceGuard dg(device_);
    for (auto* p : bufs_) (void)hipFree(p);
    for (int i = 0; i < 2; ++i) (void)hipFree(units_[i]);
    for (auto& c : log_) (void)hipFree(c.ptr);
    (void)hipFree(counters_);
    (void)hipFree(totals_);
    (void)hipFree(best64_);
    (void)hipFree(red_);
    (void)hipFree(keydev_);
    (void)hipFree(wit_);
    (void)hipEventDestroy(e0_);
    (void)hipEventDestroy(e1_);
    (void)hipStreamDestroy(stream_);
  }

  uint32_t key_words() const override { return MW; }
  uint32_t unit_bytes() const override { return UL::BYTES; }

  void reset_root() override {
    DeviceGuard dg(device_);
    ensure_cap(0, 1);
    std::vector<uint32_t> u(UL::WORDS, 0);
    for (int w = 0; w < MW; ++w) u[UL::T_ + w] = scc_mask_[w];  // toRemove = scc, dontRemove = {} (cpp:393)
    HIP_CHECK(hipMemcpyAsync(units_[cur_], u.data(), UL::BYTES, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    n_ = 1;
  }

  void clear_frontier() override { n_ = 0; }

  uint64_t frontier_size() const override { return n_; }

  StepInfo step() override {
    DeviceGuard dg(device_);
    StepInfo si;
    si.frontier_in = n_;
    if (n_ == 0) return si;
    const uint32_t lanes_full = max_blocks_ * 64u;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n_ + 63) / 64, max_blocks_);
    const uint32_t budget = (n_ >= (uint64_t)lanes_full / 2) ? cfg_.run_budget : cfg_.grow_budget;
    const uint64_t lanes = (uint64_t)blocks * 64u;
    const uint64_t out_need = n_ + lanes * (SMAX + 1 + cfg_.evict_max);
    if (out_need > 0xFFFFFFF0ull) throw Error(QI_ERR_CAPACITY, "search frontier exceeds 2^32 units");
    ensure_cap(1 - cur_, out_need);
    uint32_t* rec = log_reserve(n_);
    uint32_t init[4] = {0, (uint32_t)std::min<uint64_t>(n_, lanes), 0, 0};
    HIP_CHECK(hipMemcpyAsync(counters_, init, sizeof init, hipMemcpyHostToDevice, stream_));

    dev::SearchArgs a{};
    a.f = d_;
    a.units_in = units_[cur_];
    a.n_in = (uint32_t)n_;
    a.units_out = units_[1 - cur_];
    a.out_cap = (uint32_t)cap_[1 - cur_];
    a.counters = counters_;
    a.records = rec;
    a.wit = wit_;
    a.wit_cap = wit_cap_;
    a.totals = totals_;
    a.best64 = best64_;
    a.budget = budget;
    a.grace = cfg_.grace;
    a.evict_max = cfg_.evict_max;
    a.half_m = m_ / 2;
    a.has_best = has_best_ ? 1u : 0u;
    a.best_depth = best_depth_;
    for (int w = 0; w < 8; ++w) {
      a.best_key[w] = w < (int)best_key_.size() ? best_key_[w] : 0u;
      a.scc_mask[w] = scc_mask_[w];
    }
    HIP_CHECK(hipEventRecord(e0_, stream_));
    hipLaunchKernelGGL((dev::search_kernel<MW, TW, SMAX>), dim3(blocks), dim3(64), shm_, stream_, a);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(e1_, stream_));
    uint32_t c[4];
    HIP_CHECK(hipMemcpyAsync(c, counters_, sizeof c, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0_, e1_));
    if (c[3] & dev::FLAG_OUT_OVERFLOW) throw Error(QI_ERR_CAPACITY, "search frontier buffer overflow");
    if (c[3] & dev::FLAG_WIT_OVERFLOW) throw Error(QI_ERR_CAPACITY, "witness buffer overflow");
    uint64_t out = c[0];
    const uint64_t head = std::min<uint64_t>(c[1], n_);
    if (head < n_) {  // never-claimed units: zero their records and carry them over
      const uint64_t left = n_ - head;
      if (out + left > cap_[1 - cur_]) throw Error(QI_ERR_CAPACITY, "search frontier buffer overflow");
      HIP_CHECK(hipMemcpyAsync(units_[1 - cur_] + out * UL::WORDS, units_[cur_] + head * UL::WORDS,
                               left * UL::BYTES, hipMemcpyDeviceToDevice, stream_));
      const uint32_t nb = (uint32_t)((left + 255) / 256);
      hipLaunchKernelGGL(dev::zero_records_kernel<MW>, dim3(nb), dim3(256), 0, stream_, rec, (uint32_t)head,
                         (uint32_t)n_);
      HIP_CHECK(hipGetLastError());
      out += left;
    }
    // collect new witnesses
    if (c[2] > wit_seen_) {
      const uint32_t nw = std::min(c[2], wit_cap_) - wit_seen_;
      std::vector<uint32_t> wv((size_t)nw * WL::WORDS);
      HIP_CHECK(hipMemcpyAsync(wv.data(), wit_ + (size_t)wit_seen_ * WL::WORDS, wv.size() * 4,
                               hipMemcpyDeviceToHost, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
      for (uint32_t i = 0; i < nw; ++i) absorb_witness(&wv[(size_t)i * WL::WORDS]);
      si.new_witnesses = nw;
      // next launch reuses the buffer from the start
      wit_seen_ = 0;
      HIP_CHECK(hipMemsetAsync(counters_ + 2, 0, 4, stream_));
    }
    HIP_CHECK(hipStreamSynchronize(stream_));
    si.processed = head;
    si.frontier_out = out;
    si.budget = budget;
    si.blocks = blocks;
    si.kernel_ms = ms;
    si.has_best = has_local_best_ || has_best_;
    sum_ms_ += ms;
    ++launches_;
    n_ = out;
    cur_ = 1 - cur_;
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

  void set_best(const std::vector<uint32_t>& key, uint32_t depth) override {
    best_key_ = key;
    best_key_.resize(MW, 0);
    best_depth_ = depth;
    has_best_ = true;
  }

  bool best(Witness* w) const override {
    if (!has_local_best_) return false;
    if (w) *w = local_best_;
    return true;
  }

  Totals reduce(bool has_key, const std::vector<uint32_t>& key, uint32_t depth) override {
    DeviceGuard dg(device_);
    std::vector<uint32_t> k(8, 0);
    for (size_t i = 0; i < key.size() && i < 8; ++i) k[i] = key[i];
    HIP_CHECK(hipMemcpyAsync(keydev_, k.data(), 32, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemsetAsync(red_, 0, 32, stream_));
    for (auto& c : log_) {
      if (!c.used) continue;
      const uint32_t nb = (uint32_t)std::min<uint64_t>((c.used + 255) / 256, 4096);
      hipLaunchKernelGGL(dev::reduce_kernel<MW>, dim3(nb), dim3(256), 0, stream_, c.ptr, c.used, has_key ? 1u : 0u,
                         keydev_, depth, red_);
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
    return t;
  }

  Totals running_totals() const override {
    DeviceGuard dg(device_);
    unsigned long long r[8];
    HIP_CHECK(hipMemcpyAsync(r, totals_, sizeof r, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    Totals t;
    t.nodes = r[0];
    t.evals = r[1];
    t.minq = r[2];
    t.zero_fallback = r[3];
    t.rounds = r[4];
    t.units = r[5];
    t.wave_iters = r[6];
    t.coop_phases = r[7];
    return t;
  }

  void drop_log() override {
    for (auto& c : log_) c.used = 0;
    DeviceGuard dg(device_);
    HIP_CHECK(hipMemsetAsync(totals_, 0, 8 * sizeof(unsigned long long), stream_));
    unsigned long long inf = ~0ull;
    HIP_CHECK(hipMemcpyAsync(best64_, &inf, 8, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    has_best_ = false;
    has_local_best_ = false;
    sum_ms_ = 0;
    launches_ = 0;
  }

  double sum_kernel_ms() const override { return sum_ms_; }
  uint64_t launches() const override { return launches_; }

 private:
  struct LogChunk {
    uint32_t* ptr = nullptr;
    uint64_t cap = 0, used = 0;
  };

  void keep(const void* p) { bufs_.push_back((void*)p); }

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

  uint32_t* log_reserve(uint64_t n) {
    for (auto& c : log_)
      if (c.cap - c.used >= n) {
        uint32_t* p = c.ptr + c.used * RL::WORDS;
        c.used += n;
        return p;
      }
    LogChunk c;
    c.cap = std::max<uint64_t>(n, 1u << 22);
    c.ptr = dalloc<uint32_t>(c.cap * RL::WORDS);
    c.used = n;
    log_.push_back(c);
    return c.ptr;
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
    for (uint32_t i = 0; i < dl; ++i) w.q2_local.push_back((wv[2 * MW + 2 + i / 4] >> (8 * (i % 4))) & 255u);
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
  uint32_t scc_mask_[8];
  uint32_t max_blocks_ = 0;
  uint32_t* units_[2] = {nullptr, nullptr};
  uint64_t cap_[2] = {0, 0};
  int cur_ = 0;
  uint64_t n_ = 0;
  uint32_t* counters_ = nullptr;
  unsigned long long* totals_ = nullptr;
  unsigned long long* best64_ = nullptr;
  unsigned long long* red_ = nullptr;
  uint32_t* keydev_ = nullptr;
  uint32_t* wit_ = nullptr;
  uint32_t wit_cap_ = 0, wit_seen_ = 0;
  std::vector<LogChunk> log_;
  size_t shm_ = 0;
  bool has_best_ = false;
  std::vector<uint32_t> best_key_;
  uint32_t best_depth_ = 0;
  bool has_local_best_ = false;
  Witness local_best_;
  double sum_ms_ = 0;
  uint64_t launches_ = 0;
};

}  // namespace

std::unique_ptr<GfpDevice> make_gfp_device(int device, const GlobalFlat& g) {
  return std::unique_ptr<GfpDevice>(new GfpDeviceImpl(device, g));
}

std::unique_ptr<SearchDevice> make_search_device(int device, const LocalFlat& f, const SearchConfig& cfg) {
  const uint32_t mw = f.mw, tw = f.tw;
  if (mw <= 1 && tw <= 1) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<1, 1, 32>(device, f, cfg));
  if (mw <= 1 && tw <= 2) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<1, 2, 32>(device, f, cfg));
  if (mw <= 1 && tw <= 4) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<1, 4, 32>(device, f, cfg));
  if (mw <= 2 && tw <= 2) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<2, 2, 32>(device, f, cfg));
  if (mw <= 2 && tw <= 4) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<2, 4, 32>(device, f, cfg));
  if (mw <= 4 && tw <= 4) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<4, 4, 16>(device, f, cfg));
  if (mw <= 4 && tw <= 8) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<4, 8, 16>(device, f, cfg));
  if (mw <= 8 && tw <= 8) return std::unique_ptr<SearchDevice>(new SearchDeviceImpl<8, 8, 16>(device, f, cfg));
  throw Error(QI_ERR_UNSUPPORTED, "searched SCC too large for the device kernels (|SCC| > 256 or > 256 TNs)");
}

}  // namespace qi
