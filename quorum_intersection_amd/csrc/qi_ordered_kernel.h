// =====================================================================================
//  qi_ordered_kernel.h -- the search for SCCs whose quorum sets have threshold 0.
//
//  With threshold 0 containsQuorumSlice holds iff the FIRST entry is unavailable (the
//  size_t counters wrap, cpp:99-117), so the slice predicate is anti-monotone and the
//  reference's Gauss-Seidel fixpoint (cpp:148-169) depends on the order of `nodes`:
//    cpp:281, 184, 192   D in branch order (dontRemove, cpp:275-278 / 188)
//    cpp:301             D, then toRemove (cpp:294-297)
//    cpp:368 / 658       the SCC in ascending vertex order (cpp:628-633)
//  and toRemove is the iteration order of a libstdc++ std::unordered_set<size_t> built
//  from the previous fixpoint's survivors (cpp:308, 321-334).  This kernel reproduces
//  all of it exactly: every lane walks a subtree ("unit") depth-first like
//  search_body, but a node carries D AND toRemove as ordered vertex lists, every
//  fixpoint is a sequential sweep in list order (TN sat bits re-evaluated after each
//  removal), findBestNode counts in-degrees over the survivor list with repetitions
//  (zero-fallback = quorum.begin(), cpp:221), and toRemove is rebuilt by emulating the
//  hash table's node list (identity hash, prime bucket counts, insert at bucket head,
//  rehash relinking) -- HashList below, checked against the real container in tests.
//
//  Frontier units, segment records, witnesses and the chained-launch counter protocol
//  are those of qi_search_kernel.h; only the unit payload differs (OrdUnitLayout).
//  Monotone SCCs never come here: their fixpoints are order-free and search_body's
//  Jacobi masks are exact.
// =====================================================================================
#pragma once
#include "qi_search_kernel.h"

namespace qi {
namespace dev {

// ------------------------------------------------------------------------------------
// libstdc++ (GCC 11) std::unordered_set<size_t> node order.
//
// std::hash<size_t> is the identity and the bucket of key k is k % bucket_count.  The
// range constructor used at cpp:308 starts with one bucket and inserts element by
// element; _Prime_rehash_policy grows the table before the 1st, 14th, 30th, 60th and
// 128th distinct insertion to 13, 29, 59, 127, 257 buckets (max_load_factor 1; measured
// with bucket_count() in tests/test_oracle.py).  All nodes live on one singly linked
// list; a bucket holds the node BEFORE its first node (or the list head sentinel).
// Insertion into a non-empty bucket links after that node; into an empty bucket at the
// list head.  A rehash walks the old list and relinks every node the same way into the
// new buckets.  Erasing (cpp:321-323) unlinks without reordering, so the iteration order
// of the survivors is the list order restricted to them.
// ------------------------------------------------------------------------------------
constexpr uint32_t kHashBuckets[7] = {13u, 29u, 59u, 127u, 257u, 541u, 1109u};
constexpr int kHashSizes = 7;

__host__ __device__ inline int hash_grow_at(uint32_t k) {  // k-th distinct insertion (1-based)
  return k == 1u ? 0 : k == 14u ? 1 : k == 30u ? 2 : k == 60u ? 3 : k == 128u ? 4 : k == 258u ? 5 : k == 542u ? 6 : -1;
}
// buckets needed for up to CAP distinct elements
constexpr int hash_buckets_for(int cap) {
  return cap < 14 ? 13 : cap < 30 ? 29 : cap < 60 ? 59 : cap < 128 ? 127 : cap < 258 ? 257 : cap < 542 ? 541 : 1109;
}

// CAP: elements (local vertex ids < CAP), NB: bucket capacity.  bmod(v, r) = key(v) %
// kHashBuckets[r].
template <int CAP, int NB>
struct HashList {
  static constexpr uint16_t NIL = 0xFFFFu, BB = 0xFFFEu;  // BB: the list-head sentinel
  uint16_t nxt[CAP];
  uint16_t bkt[NB];
  uint16_t head;
  int r;          // current bucket-count index (-1: the initial single bucket)
  uint32_t cnt;   // distinct elements

  __host__ __device__ void clear() {
    head = NIL;
    r = -1;
    cnt = 0;
    bkt[0] = NIL;
  }
  __host__ __device__ uint32_t nb() const { return r < 0 ? 1u : kHashBuckets[r]; }

  template <class Mod>
  __host__ __device__ void rehash(int nr, const Mod& bmod) {
    const uint32_t n = kHashBuckets[nr];
    for (uint32_t b = 0; b < n; ++b) bkt[b] = NIL;
    uint16_t p = head;
    head = NIL;
    uint32_t bbegin = 0;
    while (p != NIL) {
      const uint16_t next = nxt[p];
      const uint32_t b = bmod(p, nr);
      if (bkt[b] == NIL) {
        nxt[p] = head;
        head = p;
        bkt[b] = BB;
        if (nxt[p] != NIL) bkt[bbegin] = p;
        bbegin = b;
      } else if (bkt[b] == BB) {
        nxt[p] = head;
        head = p;
      } else {
        const uint16_t u = bkt[b];
        nxt[p] = nxt[u];
        nxt[u] = p;
      }
      p = next;
    }
    r = nr;
  }

  // insert a vertex that is not yet present
  template <class Mod>
  __host__ __device__ void insert(uint16_t v, const Mod& bmod) {
    const int g = hash_grow_at(cnt + 1u);
    if (g >= 0) rehash(g, bmod);
    const uint32_t b = r < 0 ? 0u : bmod(v, r);
    const uint16_t u = bkt[b];
    if (u == NIL) {
      nxt[v] = head;
      head = v;
      if (nxt[v] != NIL) bkt[r < 0 ? 0u : bmod(nxt[v], r)] = v;
      bkt[b] = BB;
    } else if (u == BB) {
      nxt[v] = head;
      head = v;
    } else {
      nxt[v] = nxt[u];
      nxt[u] = v;
    }
    ++cnt;
  }
};

// ------------------------------------------------------------------------------------
// Ordered unit: path key, depth, |D| (with repetitions), |toRemove|, D in branch order,
// toRemove in hash order (OrdBytes<MW>::VB bytes per local vertex: 1 up to 256 vertices).
// ------------------------------------------------------------------------------------
template <int MW>
struct OrdUnitLayout {
  static constexpr int VB = OrdBytes<MW>::VB;
  static constexpr int EPW = 4 / VB;        // entries per 32-bit word
  static constexpr int DMAX = MW * 16 + 1;  // |D| <= m/2 + 1
  static constexpr int OWD = (DMAX + EPW - 1) / EPW;
  static constexpr int OWT = MW * 32 / EPW; // up to 32*MW toRemove entries
  static constexpr int K_ = 0, DEPTH = MW, DLEN = MW + 1, TLEN = MW + 2, DORD = MW + 3, TORD = MW + 3 + OWD;
  static constexpr int RAW = MW + 3 + OWD + OWT;
  static constexpr int WORDS = (RAW + 3) / 4 * 4;
  static constexpr int BYTES = WORDS * 4;
};

enum : uint32_t { FLAG_DEPTH = 4u };  // glob[1]: a path outgrew the key (non-terminating recursion)

struct OrdArgs {
  SearchArgs a;
  const uint32_t* vroot;    // [m] root TN of each local vertex, 0xFFFFFFFF: never satisfied
  const uint32_t* adj_off;  // [m+1] out-edges inside the SCC, with multiplicity (cpp:222-247)
  const uint32_t* adj;
  const uint16_t* bktmod;   // [kHashSizes][m] global vertex index % kHashBuckets[r]
  uint32_t* ostack;         // [blocks][smax][SEW][64] per-lane DFS stacks
  uint8_t* ows;             // MW > 8: per-lane workspace [blocks * 64][OrdWorkspace<MW>::BYTES]
  uint32_t smax;
  uint32_t depth_max;       // < 32*MW: path keys hold one bit per level
  uint32_t jacobi;          // 1: monotone SCC (here only for its size): Jacobi rounds give the
                            // same survivor set as any sweep order, and far fewer TN passes
  uint32_t probe;           // node budget of the root's lane while the frontier is the root
                            // alone: a depth-first probe before the parallel expansion
};

// TN satisfaction bits under availability A (inside the SCC; POL as in gfp)
template <int MW, int TW, int POL>
__device__ __forceinline__ void tn_sat(const LocalDev& f, const uint32_t (&A)[MW], uint32_t (&sb)[TW]) {
  using R = TnRec<MW, TW>;
  if constexpr (TW > 8) {  // |SCC| or TNs beyond 256: rolled loops, dynamic word indexing
    for (int w = 0; w < TW; ++w) sb[w] = 0;
    const __attribute__((address_space(4))) uint32_t* rec = K(f.tn);
    for (uint32_t t = 0; t < f.T; ++t, rec += R::WORDS) {
      uint32_t c = 0;
      for (int w = 0; w < MW; ++w) c += __popc(A[w] & rec[w]);
      for (uint32_t w = 0; w <= (t >> 5); ++w) c += __popc(sb[w] & rec[MW + w]);
      if (rec[R::EXTRA]) c += extra_terms<MW, TW>(f, t, A, sb);
      const int32_t th = POL == 0 ? (int32_t)rec[R::THR0] : (int32_t)rec[R::THR1];
      const uint32_t bit = (((int32_t)c >= th) ? 1u : 0u) ^ rec[R::INV];
      sb[t >> 5] |= bit << (t & 31u);
    }
    return;
  }
#pragma unroll
  for (int w = 0; w < TW; ++w) sb[w] = 0;
#pragma unroll
  for (int tw = 0; tw < TW; ++tw) {
    const uint32_t tb = (uint32_t)tw * 32u;
    const uint32_t te = min(f.T, tb + 32u);
    const __attribute__((address_space(4))) uint32_t* rec = K(f.tn) + (size_t)tb * R::WORDS;
    for (uint32_t t = tb; t < te; ++t, rec += R::WORDS) {
      uint32_t c = 0;
#pragma unroll
      for (int w = 0; w < MW; ++w) c += __popc(A[w] & rec[w]);
#pragma unroll
      for (int w = 0; w <= tw; ++w) c += __popc(sb[w] & rec[MW + w]);
      if (rec[R::EXTRA]) c += extra_terms<MW, TW>(f, t, A, sb);
      const int32_t th = POL == 0 ? (int32_t)rec[R::THR0] : (int32_t)rec[R::THR1];
      const uint32_t bit = (((int32_t)c >= th) ? 1u : 0u) ^ rec[R::INV];
      sb[tw] |= bit << (t - tb);
    }
  }
}

template <int MW>
__device__ __forceinline__ bool mbit(const uint32_t (&X)[MW], uint32_t v) {
  if constexpr (MW > 8) return (X[v >> 5] >> (v & 31u)) & 1u;
  uint32_t w = X[0];
#pragma unroll
  for (int i = 1; i < MW; ++i) w = ((v >> 5) == (uint32_t)i) ? X[i] : w;
  return (w >> (v & 31u)) & 1u;
}
template <int MW>
__device__ __forceinline__ void mset(uint32_t (&X)[MW], uint32_t v, bool on) {
  if constexpr (MW > 8) {
    X[v >> 5] = on ? (X[v >> 5] | (1u << (v & 31u))) : (X[v >> 5] & ~(1u << (v & 31u)));
    return;
  }
#pragma unroll
  for (int i = 0; i < MW; ++i)
    if ((v >> 5) == (uint32_t)i) X[i] = on ? (X[i] | (1u << (v & 31u))) : (X[i] & ~(1u << (v & 31u)));
}

// containsQuorum (cpp:140-177) on an ordered list: Gauss-Seidel sweeps in list order;
// a failing vertex leaves the list and (if available) the availability set at once.
// L[0..len) is filtered in place (survivors keep their order); A is the caller's
// availability (the reference restores it afterwards, cpp:171-173, so it is copied).
template <int MW, int TW, int POL, typename V>
__device__ uint32_t gs_fixpoint(const LocalDev& f, const uint32_t* vroot, V* L, uint32_t len,
                                const uint32_t (&A0)[MW], uint32_t& rounds, bool jacobi) {
  uint32_t A[MW], sb[TW];
  if (jacobi) {
    // monotone slices: X = listed and available, X <- X ∩ sat(X) until stable; the
    // survivors keep their list order (cpp:156 filters in order)
    uint32_t X[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) X[w] = 0;
    for (uint32_t i = 0; i < len; ++i)
      if (mbit<MW>(A0, L[i])) mset<MW>(X, L[i], true);
    for (;;) {
      ++rounds;
      tn_sat<MW, TW, POL>(f, X, sb);
      bool changed = false;
      for (uint32_t i = 0; i < len; ++i) {
        const uint32_t v = L[i];
        if (!mbit<MW>(X, v)) continue;
        const uint32_t rt = vroot[v];
        bool ok = rt != 0xFFFFFFFFu;
        if (ok) {
          uint32_t word = sb[0];
          if constexpr (TW > 8) {
            word = sb[rt >> 5];
          } else {
#pragma unroll
            for (int w = 1; w < TW; ++w) word = ((rt >> 5) == (uint32_t)w) ? sb[w] : word;
          }
          ok = (word >> (rt & 31u)) & 1u;
        }
        if (!ok) {
          mset<MW>(X, v, false);
          changed = true;
        }
      }
      if (!changed) break;
    }
    uint32_t o = 0;
    for (uint32_t i = 0; i < len; ++i)
      if (mbit<MW>(X, L[i])) L[o++] = L[i];
    return o;
  }
#pragma unroll
  for (int w = 0; w < MW; ++w) A[w] = A0[w];
  bool sb_ok = false;
  while (len) {
    ++rounds;
    uint32_t o = 0;
    bool dropped = false;
    for (uint32_t i = 0; i < len; ++i) {
      const uint32_t v = L[i];
      bool ok = mbit<MW>(A, v);  // "no self" (cpp:95)
      if (ok) {
        const uint32_t rt = vroot[v];
        if (rt == 0xFFFFFFFFu) {
          ok = false;
        } else {
          if (!sb_ok) {
            tn_sat<MW, TW, POL>(f, A, sb);
            sb_ok = true;
          }
          uint32_t word = sb[0];
          if constexpr (TW > 8) {
            word = sb[rt >> 5];
          } else {
#pragma unroll
            for (int w = 1; w < TW; ++w) word = ((rt >> 5) == (uint32_t)w) ? sb[w] : word;
          }
          ok = (word >> (rt & 31u)) & 1u;
        }
        if (!ok) {  // cpp:157-161: unavailable from here on, for the rest of the sweep too
          mset<MW>(A, v, false);
          sb_ok = false;
        }
      }
      if (ok) L[o++] = (V)v;
      else dropped = true;
    }
    len = o;
    if (!dropped) break;  // cpp:169: a sweep that removed nothing
  }
  return len;
}

// Per-lane lists, degree counters and hash table.  Up to 256 vertices they are private
// (scratch) arrays; beyond, a lane needs ~13 KB, and private segments that large exceed
// what the runtime reserves for every possible wave, so they live in an explicit global
// workspace (OrdArgs::ows) instead.
template <int MW>
struct OrdWorkspace {
  static constexpr bool GLOBAL = MW > 8;
  static constexpr int CAP = 32 * MW, DMAX = MW * 16 + 1, VB = OrdBytes<MW>::VB;
  static constexpr int R16(int b) { return (b + 15) / 16 * 16; }
  static constexpr int OFF_D = 0;
  static constexpr int OFF_T = OFF_D + R16(DMAX * VB);
  static constexpr int OFF_L = OFF_T + R16(CAP * VB);
  static constexpr int OFF_G = OFF_L + R16((CAP + DMAX) * VB);
  static constexpr int OFF_H = OFF_G + R16(CAP * 2);
  static constexpr int BYTES = OFF_H + R16((int)sizeof(HashList<CAP, hash_buckets_for(CAP)>));
};
struct OrdEmpty {};

template <int MW, int TW>
__device__ __forceinline__ void ordered_body(const OrdArgs& oa) {
  using UL = OrdUnitLayout<MW>;
  using RL = RecLayout<MW>;
  using WL = WitLayout<MW>;
  constexpr int DMAX = UL::DMAX;
  constexpr int CAP = 32 * MW;            // local vertices
  constexpr int NB = hash_buckets_for(CAP);
  constexpr int SEW = UL::OWT + 3;        // stack entry: T' entries | b, |D| | depth | |T'|
  constexpr int EPW = UL::EPW, EB = 32 / EPW;  // entries per word, bits per entry
  constexpr uint32_t EMASK = (1u << EB) - 1u;
  using V = std::conditional_t<(UL::VB == 2), uint16_t, uint8_t>;
  const SearchArgs& a = oa.a;
  const LocalDev& f = a.f;
  const uint32_t lane = threadIdx.x;
  const uint32_t m = f.m;

  // ---- chained launch prologue (as search_body) ----
  const uint32_t* pc = a.prev;
  uint32_t* cc = a.counters;
  if (pc[C_STOP] || pc[C_HALT]) {
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
  const uint32_t static_end = min(n_in, nb_used * (uint32_t)WAVE);
  const uint64_t spill_need = (uint64_t)n_in + (uint64_t)nb_used * WAVE * spill_reserve(oa.smax);
  const uint32_t evict_pool = spill_need < (uint64_t)a.out_cap ? (uint32_t)((uint64_t)a.out_cap - spill_need) : 0u;
  {
    const uint64_t need_out = spill_need + (uint64_t)nb_used * WAVE * (uint64_t)a.evict_max;
    const uint64_t need_log = (uint64_t)log_base + n_in;
    const bool stop = need_out > (uint64_t)a.out_cap || need_log > (uint64_t)a.log_cap;
    if (blockIdx.x == 0 && lane == 0) {
      cc[C_NIN] = n_in;
      cc[C_LOGB] = log_base;
      cc[C_STATIC] = static_end;
      cc[C_STOP] = stop ? 1u : 0u;
      if (stop || nb_used == 0) {
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
  // a lone root unit first goes depth-first on one lane: an early witness (cpp:369-377)
  // then ends the search before the parallel growth expands the subtrees after it
  const bool probing = n_in == 1u && oa.probe;  // (no grace: nothing else is left to claim)
  const uint32_t budget = probing ? oa.probe : launch_budget(a, n_in, false);
  uint32_t* const st = oa.ostack + (size_t)blockIdx.x * (oa.smax * SEW * WAVE);
#define OST(lvl, w) st[((size_t)(lvl) * SEW + (w)) * WAVE + lane]

  auto bmod = [&](uint32_t v, int r) -> uint32_t { return oa.bktmod[(uint32_t)r * m + v]; };

  // current node
  uint32_t K[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) K[w] = 0;
  uint32_t depth = 0, dlen = 0, tlen = 0;
  using WS = OrdWorkspace<MW>;
  using HL = HashList<CAP, NB>;
  using DArr = V[DMAX];
  using TArr = V[CAP];
  using LArr = V[CAP + DMAX];
  using GArr = uint16_t[CAP];
  std::conditional_t<WS::GLOBAL, OrdEmpty, DArr> d_store;
  std::conditional_t<WS::GLOBAL, OrdEmpty, TArr> t_store;
  std::conditional_t<WS::GLOBAL, OrdEmpty, LArr> l_store;
  std::conditional_t<WS::GLOBAL, OrdEmpty, GArr> g_store;
  std::conditional_t<WS::GLOBAL, OrdEmpty, HL> h_store;
  V *Dord, *Tord, *Lst;
  uint16_t* deg;
  HL* hlp;
  if constexpr (WS::GLOBAL) {
    uint8_t* w = oa.ows + ((size_t)blockIdx.x * WAVE + lane) * WS::BYTES;
    Dord = (V*)(w + WS::OFF_D);
    Tord = (V*)(w + WS::OFF_T);
    Lst = (V*)(w + WS::OFF_L);
    deg = (uint16_t*)(w + WS::OFF_G);
    hlp = (HL*)(w + WS::OFF_H);
  } else {
    Dord = (V*)&d_store;
    Tord = (V*)&t_store;
    Lst = (V*)&l_store;
    deg = (uint16_t*)&g_store;
    hlp = (HL*)&h_store;
  }
  HL& hl = *hlp;
  bool has = false, done = false;
  uint32_t nst = 0, sbase = 0;
  auto spos = [&](uint32_t i) -> uint32_t {
    const uint32_t p = sbase + i;
    return p >= oa.smax ? p - oa.smax : p;
  };
  uint32_t steps = 0, limit = budget, rounds = 0;
  bool dry = false, must_spill = false;
  bool seg_open = false;
  uint32_t seg_idx = 0, seg_depth = 0, seg_count = 0, seg_evals = 0, seg_minq = 0, seg_zfb = 0;
  uint32_t seg_K[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) seg_K[w] = 0;
  uint64_t tot_nodes = 0, tot_evals = 0, tot_minq = 0, tot_zfb = 0, tot_fetched = 0;
  uint64_t best64 = ~0ull;
  uint32_t iter = 0;

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
    if (MW > 1 && a.has_best) p = after_key<MW>(KK, d, a.best_key, a.best_depth);
    return p || (best_pack<MW>(KK, d) > best64);
  };
  // unit writers: D order = Dord[0..dl) (+ extra entry b >= 0), T order = tb[0..tl)
  auto write_unit = [&](uint32_t slot, const uint32_t (&UK)[MW], uint32_t udepth, uint32_t dl, int b,
                        const V* tb, uint32_t tl, bool t_from_stack, uint32_t spos_) {
    if (slot >= a.out_cap) {
      atomicOr(&a.glob[1], FLAG_OUT_OVERFLOW);
      return;
    }
    uint32_t* u = a.units_out + (size_t)slot * UL::WORDS;
#pragma unroll
    for (int w = 0; w < MW; ++w) u[UL::K_ + w] = UK[w];
    const uint32_t ul = dl + (b >= 0 ? 1u : 0u);
    u[UL::DEPTH] = udepth;
    u[UL::DLEN] = ul;
    u[UL::TLEN] = tl;
    for (uint32_t i = 0; i < (ul + EPW - 1u) / EPW; ++i) {
      uint32_t word = 0;
      for (uint32_t j = 0; j < (uint32_t)EPW; ++j) {
        const uint32_t p = EPW * i + j;
        const uint32_t e = p < dl ? (uint32_t)Dord[p] : (p == dl && b >= 0 ? (uint32_t)b : 0u);
        word |= e << (EB * j);
      }
      u[UL::DORD + i] = word;
    }
    if (t_from_stack) {
      for (uint32_t i = 0; i < (tl + EPW - 1u) / EPW; ++i) u[UL::TORD + i] = OST(spos_, i);
    } else {
      for (uint32_t i = 0; i < (tl + EPW - 1u) / EPW; ++i) {
        uint32_t word = 0;
        for (uint32_t j = 0; j < (uint32_t)EPW && EPW * i + j < tl; ++j) word |= (uint32_t)tb[EPW * i + j] << (EB * j);
        u[UL::TORD + i] = word;
      }
    }
  };
  // stack entry at circular position p as a unit (the inclusion child it stands for)
  auto write_entry = [&](uint32_t slot, uint32_t p) {
    const uint32_t pk = OST(p, UL::OWT), de = OST(p, UL::OWT + 1), tl = OST(p, UL::OWT + 2);
    const uint32_t b = pk & 0xFFFFu, dle = pk >> 16;
    uint32_t UK[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) UK[w] = K[w];
    key_prefix_bit<MW>(UK, de);
    write_unit(slot, UK, de + 1u, dle, (int)b, nullptr, tl, true, p);
  };

  auto claim_next = [&]() -> bool {  // next unit index into seg_idx
    if (dry || steps >= limit) return false;
    const uint32_t h = atomicAdd(&cc[C_HEAD], 1u);
    const uint32_t idx = static_end + h;
    if (idx >= n_in) {
      dry = true;
      if (!probing) limit = min(limit, steps + a.grace);
      return false;
    }
    seg_idx = idx;
    return true;
  };
  auto install = [&](uint32_t idx) {
    const uint32_t* u = a.units_in + (size_t)idx * UL::WORDS;
#pragma unroll
    for (int w = 0; w < MW; ++w) K[w] = seg_K[w] = u[UL::K_ + w];
    depth = seg_depth = u[UL::DEPTH];
    dlen = u[UL::DLEN];
    tlen = u[UL::TLEN];
    for (uint32_t i = 0; i < dlen; ++i) Dord[i] = (V)((u[UL::DORD + i / EPW] >> (EB * (i % EPW))) & EMASK);
    for (uint32_t i = 0; i < tlen; ++i) Tord[i] = (V)((u[UL::TORD + i / EPW] >> (EB * (i % EPW))) & EMASK);
    seg_idx = idx;
    seg_open = true;
    seg_count = seg_evals = seg_minq = seg_zfb = 0;
    nst = 0;
    sbase = 0;
    ++tot_fetched;
    if (pruned(K, depth)) close_segment();  // zero record
    else has = true;
  };

  bool first = blockIdx.x * WAVE + lane < n_in;
  while (!done) {
    // ---- a lane without a node: pop the stack, else the next unit -----------------------
    if (!has) {
      if (nst > 0) {
        const uint32_t p = spos(nst - 1u);
        const uint32_t pk = OST(p, UL::OWT), de = OST(p, UL::OWT + 1), tl = OST(p, UL::OWT + 2);
        uint32_t NK[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) NK[w] = K[w];
        key_prefix_bit<MW>(NK, de);
        if (pruned(NK, de + 1u)) {  // deeper entries precede shallower ones: drop all
          nst = 0;
        } else {
          --nst;
          const uint32_t b = pk & 0xFFFFu, dle = pk >> 16;
          for (uint32_t i = 0; i < (tl + EPW - 1u) / EPW; ++i) {
            const uint32_t word = OST(p, i);
            for (uint32_t j = 0; j < (uint32_t)EPW && EPW * i + j < tl; ++j) Tord[EPW * i + j] = (V)((word >> (EB * j)) & EMASK);
          }
          tlen = tl;
          Dord[dle] = (V)b;
          dlen = dle + 1u;
          depth = de + 1u;
#pragma unroll
          for (int w = 0; w < MW; ++w) K[w] = NK[w];
          has = true;
        }
      }
      if (!has) {
        if (seg_open) close_segment();
        if (first) {
          first = false;
          install(blockIdx.x * WAVE + lane);
        } else if (claim_next()) {
          install(seg_idx);
        } else {
          done = true;
        }
        if (!has) continue;
      }
    }
    // ---- poll the queue head / device best key -----------------------------------------
    if ((iter++ & 31u) == 0u) {
      const uint32_t h = __hip_atomic_load(&cc[C_HEAD], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      best64 = __hip_atomic_load(a.best64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (blockIdx.x == 0 && lane == 0 && a.xbest != a.best64) {
        // block 0 forwards the cooperating engines' shared key (pinned host word) into this
        // device's word, where every wave polls it
        const uint64_t xb = __hip_atomic_load(a.xbest, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (xb < best64) atomicMin(a.best64, (unsigned long long)xb);
      }
      if (!dry && static_end + h >= n_in) {
        dry = true;
        if (!probing) limit = min(limit, steps + a.grace);
      }
    }
    // ---- budget / eviction cap: the node and the stack go to the next frontier ----------
    if (steps >= limit || must_spill) {
      const uint32_t n = 1u + nst;
      uint32_t slot = atomicAdd(&cc[C_OUT], n);
      write_unit(slot++, K, depth, dlen, -1, Tord, tlen, false, 0);
      for (uint32_t i = nst; i > 0; --i) write_entry(slot++, spos(i - 1u));
      nst = 0;
      has = false;
      if (seg_open) close_segment();
      done = true;
      break;
    }

    // ---- one search node (cpp:258-345) --------------------------------------------------
    ++steps;
    ++seg_count;
    has = false;
    if (dlen > a.half_m || (tlen == 0u && dlen == 0u)) continue;  // cpp:261 / 266
    if (depth >= oa.depth_max) {  // the key has no bit left for a child: flag, stop here
      atomicOr(&a.glob[1], FLAG_DEPTH);
      continue;
    }
    uint32_t Dm[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) Dm[w] = 0;
    for (uint32_t i = 0; i < dlen; ++i) mset<MW>(Dm, Dord[i], true);
    // cpp:275-281: GFP(D), nodes = D in branch order, only D available
    for (uint32_t i = 0; i < dlen; ++i) Lst[i] = Dord[i];
    ++seg_evals;
    if (gs_fixpoint<MW, TW, 0>(f, oa.vroot, Lst, dlen, Dm, rounds, oa.jacobi != 0)) {
      // cpp:283 isMinimalQuorum: cpp:184 repeats cpp:281 (same inputs, same result)
      ++seg_evals;
      bool minimal = true;
      for (uint32_t i = 0; i < dlen && minimal; ++i) {  // cpp:188-198
        uint32_t A[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) A[w] = Dm[w];
        mset<MW>(A, Dord[i], false);
        for (uint32_t j = 0; j < dlen; ++j) Lst[j] = Dord[j];
        ++seg_evals;
        if (gs_fixpoint<MW, TW, 0>(f, oa.vroot, Lst, dlen, A, rounds, oa.jacobi != 0)) minimal = false;
      }
      if (minimal) {  // visitor (cpp:357-384): scc in ascending order, D unavailable
        ++seg_minq;
        ++seg_evals;
        uint32_t A[MW];
#pragma unroll
        for (int w = 0; w < MW; ++w) A[w] = f.scc_mask[w] & ~Dm[w];
        for (uint32_t v = 0; v < m; ++v) Lst[v] = (V)v;
        const uint32_t ql = gs_fixpoint<MW, TW, 1>(f, oa.vroot, Lst, m, A, rounds, oa.jacobi != 0);
        if (ql) {  // cpp:369-377: disjoint quorums, the search ends here
          uint32_t Q1[MW];
#pragma unroll
          for (int w = 0; w < MW; ++w) Q1[w] = 0;
          for (uint32_t i = 0; i < ql; ++i) mset<MW>(Q1, Lst[i], true);
          const uint32_t slot = atomicAdd(&a.glob[0], 1u);
          if (slot < a.wit_cap) {
            uint32_t* wv = a.wit + (size_t)slot * WL::WORDS;
#pragma unroll
            for (int w = 0; w < MW; ++w) {
              wv[w] = K[w];
              wv[MW + 2 + w] = Q1[w];
            }
            wv[MW] = depth;
            wv[MW + 1] = dlen;
            for (uint32_t i = 0; i < (dlen + EPW - 1u) / EPW; ++i) {
              uint32_t word = 0;
              for (uint32_t j = 0; j < (uint32_t)EPW && EPW * i + j < dlen; ++j) word |= (uint32_t)Dord[EPW * i + j] << (EB * j);
              wv[2 * MW + 2 + i] = word;
            }
          } else {
            atomicOr(&a.glob[1], FLAG_WIT_OVERFLOW);
          }
          atomicMin(a.best64, (unsigned long long)best_pack<MW>(K, depth));
          nst = 0;  // the rest of this unit follows the witness in preorder
        }
      }
      continue;
    }
    // cpp:294-301: GFP(D ++ toRemove), both available (the sweeps above filtered Lst in
    // place: lay D out again)
    uint32_t A[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) A[w] = Dm[w];
    for (uint32_t i = 0; i < dlen; ++i) Lst[i] = Dord[i];
    for (uint32_t i = 0; i < tlen; ++i) {
      Lst[dlen + i] = Tord[i];
      mset<MW>(A, Tord[i], true);
    }
    ++seg_evals;
    const uint32_t ql = gs_fixpoint<MW, TW, 0>(f, oa.vroot, Lst, dlen + tlen, A, rounds, oa.jacobi != 0);
    if (!ql) continue;  // cpp:303
    uint32_t Qm[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) Qm[w] = 0;
    for (uint32_t i = 0; i < ql; ++i) mset<MW>(Qm, Lst[i], true);
    uint32_t bad = 0, rest = 0;
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      bad |= Dm[w] & ~Qm[w];
      rest |= Qm[w] & ~Dm[w];
    }
    if (bad) continue;  // cpp:309-314
    // findBestNode (cpp:203-250): in-degree from every entry of `quorum` (repetitions
    // count) into quorum \ D; ties -> lowest index; no edge at all -> quorum.begin()
    for (uint32_t v = 0; v < m; ++v) deg[v] = 0;
    for (uint32_t i = 0; i < ql; ++i) {
      const uint32_t u = Lst[i];
      for (uint32_t e = oa.adj_off[u], e1 = oa.adj_off[u + 1]; e < e1; ++e) {
        const uint32_t w = oa.adj[e];
        if (mbit<MW>(Qm, w) && !mbit<MW>(Dm, w)) ++deg[w];
      }
    }
    uint32_t best = Lst[0], bestdeg = 0;
    for (uint32_t v = 0; v < m; ++v)
      if (deg[v] > bestdeg) {
        bestdeg = deg[v];
        best = v;
      }
    if (bestdeg == 0u) ++seg_zfb;
    if (!rest) continue;  // cpp:325: quorumNodes \ D is empty
    // toRemove' (cpp:308, 321-334): the hash table's order, without D and bestNode
    hl.clear();
    uint32_t seen[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) seen[w] = 0;
    for (uint32_t i = 0; i < ql; ++i) {
      const uint32_t v = Lst[i];
      if (mbit<MW>(seen, v)) continue;  // already present (repeated D entries)
      mset<MW>(seen, v, true);
      hl.insert((uint16_t)v, bmod);
    }
    uint32_t tl = 0;
    for (uint16_t v = hl.head; v != HashList<CAP, NB>::NIL; v = hl.nxt[v])
      if (!mbit<MW>(Dm, v) && v != best) Tord[tl++] = (V)v;
    tlen = tl;
    // push the inclusion child (cpp:343-345), continue with the exclusion child (cpp:336)
    if (nst == oa.smax) {  // full: the shallowest entry goes to the next frontier
      const uint32_t slot = atomicAdd(&cc[C_OUT], 1u);
      write_entry(slot, spos(0));
      sbase = spos(1);
      --nst;
      if (atomicAdd(&cc[C_EVX], 1u) >= evict_pool) {  // the pool is dry: this slot came out
        must_spill = true;                            // of the lane's spill reserve; stop
        atomicOr(&a.glob[1], FLAG_POOL);
      }
    }
    {
      const uint32_t p = spos(nst);
      for (uint32_t i = 0; i < (tl + EPW - 1u) / EPW; ++i) {
        uint32_t word = 0;
        for (uint32_t j = 0; j < (uint32_t)EPW && EPW * i + j < tl; ++j) word |= (uint32_t)Tord[EPW * i + j] << (EB * j);
        OST(p, i) = word;
      }
      OST(p, UL::OWT) = best | (dlen << 16);
      OST(p, UL::OWT + 1) = depth;
      OST(p, UL::OWT + 2) = tl;
      ++nst;
    }
    ++depth;
    has = true;
  }

  // wave-reduce the running totals (every lane arrives here)
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
    unsigned long long* tt = a.totals + (size_t)(blockIdx.x & (TOT_SHARDS - 1)) * 16;
    atomicAdd(&tt[0], (unsigned long long)tot_nodes);
    atomicAdd(&tt[1], (unsigned long long)tot_evals);
    atomicAdd(&tt[2], (unsigned long long)tot_minq);
    atomicAdd(&tt[3], (unsigned long long)tot_zfb);
    atomicAdd(&tt[4], (unsigned long long)tr);
    atomicAdd(&tt[5], (unsigned long long)tot_fetched);
  }
  // ---- last block: carry never-claimed units over, publish the counters ----------------
  {
    uint32_t old = 0;
    if (lane == 0) old = atomicAdd(&cc[C_DONE], 1u);
    old = lane0(old);
    if (old == nb_used - 1u) {
      uint32_t hd = 0, out = 0;
      if (lane == 0) {
        hd = atomicAdd(&cc[C_HEAD], 0u);
        out = atomicAdd(&cc[C_OUT], 0u);
      }
      hd = lane0(hd);
      out = lane0(out);
      const uint32_t head = (uint32_t)min((uint64_t)static_end + hd, (uint64_t)n_in);
      const uint32_t left = n_in - head;
      for (uint32_t i = lane; i < left; i += WAVE) {
        uint32_t* r = records + (size_t)(head + i) * RL::WORDS;
        for (int w = 0; w < RL::WORDS; ++w) r[w] = 0u;
        const uint32_t dst = out + i;
        if (dst < a.out_cap) {
          const uint4* s4 = (const uint4*)(a.units_in + (size_t)(head + i) * UL::WORDS);
          uint4* d4 = (uint4*)(a.units_out + (size_t)dst * UL::WORDS);
          for (int q = 0; q < UL::WORDS / 4; ++q) d4[q] = s4[q];
        } else {
          atomicOr(&a.glob[1], FLAG_OUT_OVERFLOW);
        }
      }
      if (lane == 0) {
        const unsigned long long bb = atomicMin(a.best64, ~0ull);  // this launch's best key, for the host
        a.host_ctr[HC_BEST] = (uint32_t)bb;
        a.host_ctr[HC_BEST + 1] = (uint32_t)(bb >> 32);
        cc[C_HALT] = left ? 1u : 0u;
        a.host_ctr[HC_HALT] = left ? 1u : 0u;
        out += left;
        if (left) atomicExch(&cc[C_OUT], out);
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
#undef OST
}

}  // namespace dev
}  // namespace qi
