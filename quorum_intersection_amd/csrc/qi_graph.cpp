// Trust graph, SCC numbering, threshold-node flattening and text output (host C++).
#include <algorithm>
#include <climits>
#include <cmath>
#include <functional>
#include <iomanip>
#include <map>
#include <sstream>
#include <unordered_map>

#include "qi_internal.h"
#include "../../include/quorum_intersection.h"

namespace qi {

// buildDependencyGraph (cpp:438-473): one vertex per JSON entry in file order; the id
// map keeps the LAST vertex of a duplicated publicKey, whose quorum set then receives
// every duplicate's entries (threshold overwritten, lists appended); unknown validator
// ids default-insert vertex 0 (cpp:456).  Edges follow the quorum-set traversal order:
// validators first, then inner sets depth-first.
Graph build_graph(const std::vector<StellarNode>& nodes) {
  Graph g;
  const size_t n = nodes.size();
  g.ids.reserve(n);
  g.names.reserve(n);
  g.qsets.resize(n);
  g.adj.resize(n);
  std::unordered_map<std::string, uint32_t> id_map;
  id_map.reserve(n * 2 + 1);
  for (size_t i = 0; i < n; ++i) {
    g.ids.push_back(nodes[i].publicKey);
    g.names.push_back(nodes[i].name);
    id_map[nodes[i].publicKey] = (uint32_t)i;
  }
  std::function<void(uint32_t, QuorumSet&, const QuorumSetIds&)> add = [&](uint32_t ix, QuorumSet& q,
                                                                         const QuorumSetIds& o) {
    q.threshold = o.threshold;
    q.has_threshold = o.has_threshold;
    for (const auto& id : o.validators) {
      auto it = id_map.find(id);
      uint32_t v;
      if (it == id_map.end()) {
        v = 0;
        id_map.emplace(id, 0u);  // operator[] default-insert semantics
      } else {
        v = it->second;
      }
      q.validators.push_back(v);
      g.adj[ix].push_back(v);
    }
    for (const auto& in : o.inner) {
      q.inner.emplace_back();
      add(ix, q.inner.back(), in);
    }
  };
  for (size_t i = 0; i < n; ++i) {
    const uint32_t ix = id_map[nodes[i].publicKey];
    add(ix, g.qsets[ix], nodes[i].qset);
  }
  return g;
}

// Tarjan with an explicit stack; same discovery/finish order as boost's
// depth_first_search (roots in vertex order, out-edges in insertion order), so the
// component ids equal boost::strong_components' (SCC completion order).
Sccs strong_components(const Graph& g) {
  const uint32_t n = g.n();
  const uint32_t NONE = 0xFFFFFFFFu;
  Sccs s;
  s.comp.assign(n, NONE);
  std::vector<uint32_t> disc(n, NONE), low(n, 0), stack;
  std::vector<uint8_t> on(n, 0);
  std::vector<std::pair<uint32_t, uint32_t>> call;  // (vertex, next edge)
  uint32_t time = 0, ncomp = 0;
  for (uint32_t r = 0; r < n; ++r) {
    if (disc[r] != NONE) continue;
    disc[r] = low[r] = time++;
    stack.push_back(r);
    on[r] = 1;
    call.emplace_back(r, 0u);
    while (!call.empty()) {
      const uint32_t v = call.back().first;
      uint32_t& e = call.back().second;
      if (e < g.adj[v].size()) {
        const uint32_t w = g.adj[v][e++];
        if (disc[w] == NONE) {
          disc[w] = low[w] = time++;
          stack.push_back(w);
          on[w] = 1;
          call.emplace_back(w, 0u);
        } else if (on[w] && disc[w] < low[v]) {
          low[v] = disc[w];
        }
        continue;
      }
      call.pop_back();
      if (!call.empty()) {
        const uint32_t p = call.back().first;
        if (low[v] < low[p]) low[p] = low[v];
      }
      if (low[v] == disc[v]) {
        uint32_t w;
        do {
          w = stack.back();
          stack.pop_back();
          on[w] = 0;
          s.comp[w] = ncomp;
        } while (w != v);
        ++ncomp;
      }
    }
  }
  s.members.assign(ncomp, {});
  for (uint32_t v = 0; v < n; ++v) s.members[s.comp[v]].push_back(v);
  return s;
}

// ------------------------------------------------------------------------------------
// Global flattening (all vertices; per-query availability supplied by the caller)
// ------------------------------------------------------------------------------------
namespace {

struct GKey {
  uint32_t kind, thr, first;
  std::vector<uint32_t> v, c;
  bool operator<(const GKey& o) const {
    if (kind != o.kind) return kind < o.kind;
    if (thr != o.thr) return thr < o.thr;
    if (first != o.first) return first < o.first;
    if (v != o.v) return v < o.v;
    return c < o.c;
  }
};

}  // namespace

GlobalFlat flatten_global(const Graph& g) {
  GlobalFlat out;
  out.n = g.n();
  out.words = (out.n + 63) / 64;
  std::map<GKey, uint32_t> ids;
  std::vector<GKey> keys;
  std::vector<uint32_t> level;
  std::function<uint32_t(const QuorumSet&)> walk = [&](const QuorumSet& q) -> uint32_t {
    std::vector<uint32_t> kids;
    kids.reserve(q.inner.size());
    for (const auto& in : q.inner) kids.push_back(walk(in));
    const uint64_t entries = q.validators.size() + q.inner.size();
    GKey k{TN_NEVER, 0, 0, {}, {}};
    if (entries == 0 || q.threshold > entries) {
      k.kind = TN_NEVER;
    } else if (q.threshold == 0) {
      k.kind = TN_FIRST_UNAVAIL;
      k.first = q.validators.empty() ? (0x80000000u | kids[0]) : q.validators[0];
    } else {
      k.kind = TN_NORMAL;
      k.thr = (uint32_t)q.threshold;
      k.v = q.validators;
      k.c = kids;
      std::sort(k.v.begin(), k.v.end());
      std::sort(k.c.begin(), k.c.end());
    }
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    uint32_t lv = 0;
    if (k.kind == TN_NORMAL)
      for (uint32_t c : k.c) lv = std::max(lv, level[c] + 1);
    if (k.kind == TN_FIRST_UNAVAIL && (k.first >> 31)) lv = level[k.first & 0x7FFFFFFFu] + 1;
    const uint32_t id = (uint32_t)keys.size();
    ids.emplace(k, id);
    keys.push_back(std::move(k));
    level.push_back(lv);
    return id;
  };
  std::vector<uint32_t> root(out.n);
  for (uint32_t v = 0; v < out.n; ++v) root[v] = walk(g.qsets[v]);
  // order TNs by level (stable) and renumber
  const uint32_t T = (uint32_t)keys.size();
  std::vector<uint32_t> order(T);
  for (uint32_t i = 0; i < T; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return level[a] < level[b]; });
  std::vector<uint32_t> remap(T);
  for (uint32_t i = 0; i < T; ++i) remap[order[i]] = i;
  out.T = T;
  out.levels = T ? level[order[T - 1]] + 1 : 0;
  out.level_off.assign(out.levels + 1, 0);
  for (uint32_t i = 0; i < T; ++i) out.level_off[level[order[i]] + 1]++;
  for (uint32_t l = 0; l < out.levels; ++l) out.level_off[l + 1] += out.level_off[l];
  out.kind.resize(T);
  out.thr.resize(T);
  out.first.resize(T);
  out.vref_off.assign(T + 1, 0);
  out.cref_off.assign(T + 1, 0);
  for (uint32_t i = 0; i < T; ++i) {
    const GKey& k = keys[order[i]];
    out.kind[i] = k.kind;
    if (k.kind == TN_FIRST_UNAVAIL) out.nonmonotone = true;
    out.thr[i] = k.thr;
    out.first[i] = (k.kind == TN_FIRST_UNAVAIL && (k.first >> 31)) ? (0x80000000u | remap[k.first & 0x7FFFFFFFu])
                                                                   : k.first;
    for (uint32_t v : k.v) out.vref.push_back(v);
    for (uint32_t c : k.c) out.cref.push_back(remap[c]);
    out.vref_off[i + 1] = (uint32_t)out.vref.size();
    out.cref_off[i + 1] = (uint32_t)out.cref.size();
  }
  out.root.resize(out.n);
  for (uint32_t v = 0; v < out.n; ++v) out.root[v] = remap[root[v]];
  return out;
}

// ------------------------------------------------------------------------------------
// SCC-local flattening for the search kernel
// ------------------------------------------------------------------------------------
namespace {

constexpr int32_t NEVER_THR = INT32_MAX;

struct LKey {
  int32_t t0, t1;
  uint32_t inv;
  std::vector<uint32_t> v, c;  // sorted local multisets
  bool operator<(const LKey& o) const {
    if (t0 != o.t0) return t0 < o.t0;
    if (t1 != o.t1) return t1 < o.t1;
    if (inv != o.inv) return inv < o.inv;
    if (v != o.v) return v < o.v;
    return c < o.c;
  }
};

uint32_t words_for(uint32_t bits) {
  uint32_t w = (bits + 31) / 32;
  return w ? w : 1;
}

// multiset -> multiplicity planes (plane p = elements occurring more than p times)
std::vector<std::vector<uint32_t>> planes(const std::vector<uint32_t>& sorted, uint32_t words) {
  std::vector<std::vector<uint32_t>> out;
  size_t i = 0;
  while (i < sorted.size()) {
    size_t j = i;
    while (j < sorted.size() && sorted[j] == sorted[i]) ++j;
    const size_t mult = j - i;
    while (out.size() < mult) out.emplace_back(words, 0u);
    for (size_t p = 0; p < mult; ++p) out[p][sorted[i] >> 5] |= 1u << (sorted[i] & 31);
    i = j;
  }
  return out;
}

}  // namespace

// Lower bound on the number of SCC vertices in any set that satisfies a TN (cpp:90-138
// with monotone thresholds), per polarity.  Items of a TN are its validator refs (points =
// multiplicity, cost 1) and its inner sets (points = multiplicity, cost = their bound).
// When the vertex supports of the items are pairwise disjoint, costs add and the bound is
// the exact minimum-cost cover of `threshold` points (0/1 knapsack over points); when they
// overlap, only "one item must be satisfied" is used.  The minimum over the SCC's roots
// bounds every non-empty greatest fixpoint from below.
uint32_t min_quorum_size(const LocalFlat& L, int pol) {
  constexpr uint32_t INF = 0xFFFFFFFFu;
  const uint32_t T = L.T, mw = L.mw, tw = L.tw;
  std::vector<uint32_t> cost(T, INF);
  std::vector<std::vector<uint32_t>> sup(T, std::vector<uint32_t>(mw, 0u));
  for (uint32_t t = 0; t < T; ++t) {  // children-first order
    // multiplicities from plane 0 + extra planes
    std::vector<uint32_t> vm(L.m, 0), cm(T, 0);
    for (uint32_t v = 0; v < L.m; ++v)
      if ((L.vmask[(size_t)t * mw + (v >> 5)] >> (v & 31)) & 1u) ++vm[v];
    for (uint32_t c = 0; c < T; ++c)
      if ((L.cmask[(size_t)t * tw + (c >> 5)] >> (c & 31)) & 1u) ++cm[c];
    for (uint32_t e = L.extra_off[t]; e < L.extra_off[t + 1]; ++e) {
      const uint32_t src = L.extra_src[e], msk = L.extra_mask[e];
      for (uint32_t b = 0; b < 32; ++b) {
        if (!((msk >> b) & 1u)) continue;
        if (src < mw) ++vm[src * 32 + b];
        else ++cm[(src - mw) * 32 + b];
      }
    }
    struct Item { uint32_t pts, cost; };
    std::vector<Item> items;
    bool disjoint = true;
    std::vector<uint32_t> acc(mw, 0u);
    auto add_support = [&](const std::vector<uint32_t>& s) {
      for (uint32_t w = 0; w < mw; ++w) {
        if (acc[w] & s[w]) disjoint = false;
        acc[w] |= s[w];
      }
    };
    for (uint32_t v = 0; v < L.m; ++v)
      if (vm[v]) {
        items.push_back({vm[v], 1u});
        std::vector<uint32_t> one(mw, 0u);
        one[v >> 5] = 1u << (v & 31);
        add_support(one);
      }
    for (uint32_t c = 0; c < T; ++c)
      if (cm[c]) {
        if (cost[c] != INF) items.push_back({cm[c], cost[c]});
        add_support(sup[c]);
      }
    sup[t] = acc;
    const int32_t th = L.thr[2 * t + pol];
    if (L.flags[t] & 1u) {
      cost[t] = 0;
    } else if (th <= 0) {
      cost[t] = 0;
    } else if (th == INT32_MAX) {
      cost[t] = INF;
    } else if (disjoint) {
      std::vector<uint64_t> dp((size_t)th + 1, INF);
      dp[0] = 0;
      for (const Item& it : items)
        for (int32_t p = th; p >= 0; --p) {
          if (dp[p] == INF) continue;
          const int32_t q = std::min<int32_t>(th, p + (int32_t)it.pts);
          dp[q] = std::min<uint64_t>(dp[q], dp[p] + it.cost);
        }
      cost[t] = dp[th] >= INF ? INF : (uint32_t)dp[th];
    } else {
      uint32_t lo = INF;
      for (const Item& it : items) lo = std::min(lo, it.cost);
      cost[t] = lo;
    }
  }
  uint32_t q = INF;
  for (uint32_t r = 0; r < L.R; ++r) q = std::min(q, cost[L.root_tn[r]]);
  return std::min(q, L.m + 1);  // no satisfiable root: every fixpoint is empty
}

LocalFlat flatten_local(const Graph& g, const std::vector<uint32_t>& scc) {
  LocalFlat L;
  L.m = (uint32_t)scc.size();
  L.mw = words_for(L.m);
  L.scc = scc;
  std::vector<int32_t> local(g.n(), -1);
  for (uint32_t i = 0; i < L.m; ++i) local[scc[i]] = (int32_t)i;

  std::map<LKey, uint32_t> ids;
  std::vector<LKey> keys;
  // returns TN id; NEVER nodes are deduplicated like any other
  std::function<uint32_t(const QuorumSet&)> walk = [&](const QuorumSet& q) -> uint32_t {
    std::vector<uint32_t> kids;
    kids.reserve(q.inner.size());
    for (const auto& in : q.inner) kids.push_back(walk(in));
    const uint64_t entries = q.validators.size() + q.inner.size();
    LKey k{NEVER_THR, NEVER_THR, 0, {}, {}};
    if (entries == 0 || q.threshold > entries) {
      // never satisfied
    } else if (q.threshold == 0) {
      // true iff the first entry is unavailable (size_t wrap, cpp:99-117)
      if (!q.validators.empty()) {
        const int32_t lv = local[q.validators[0]];
        if (lv >= 0) {
          k.t0 = k.t1 = 0;
          k.inv = 1;
          k.v.push_back((uint32_t)lv);
        } else {
          k.t0 = 0;            // outside unavailable -> satisfied
          k.t1 = NEVER_THR;    // outside available   -> not satisfied
        }
      } else {
        k.t0 = k.t1 = 0;
        k.inv = 1;
        k.c.push_back(kids[0]);
      }
    } else {
      int32_t out_cnt = 0;
      for (uint32_t v : q.validators) {
        if (local[v] >= 0) k.v.push_back((uint32_t)local[v]);
        else ++out_cnt;
      }
      k.c = kids;
      std::sort(k.v.begin(), k.v.end());
      std::sort(k.c.begin(), k.c.end());
      k.t0 = (int32_t)q.threshold;
      k.t1 = (int32_t)q.threshold - out_cnt;
    }
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    const uint32_t id = (uint32_t)keys.size();
    ids.emplace(k, id);
    keys.push_back(std::move(k));
    return id;
  };
  std::vector<uint32_t> root(L.m);
  for (uint32_t i = 0; i < L.m; ++i) root[i] = walk(g.qsets[scc[i]]);

  // keep TNs reachable from roots that can ever be satisfied; ids are already
  // children-first (post-order), compaction preserves that order
  const uint32_t T0 = (uint32_t)keys.size();
  std::vector<uint8_t> live(T0, 0);
  std::function<void(uint32_t)> mark = [&](uint32_t t) {
    if (live[t]) return;
    live[t] = 1;
    for (uint32_t c : keys[t].c) mark(c);
  };
  auto never = [&](uint32_t t) { return keys[t].t0 == NEVER_THR && keys[t].t1 == NEVER_THR && !keys[t].inv; };
  for (uint32_t i = 0; i < L.m; ++i)
    if (!never(root[i])) mark(root[i]);
  std::vector<uint32_t> remap(T0, 0xFFFFFFFFu);
  uint32_t T = 0;
  for (uint32_t t = 0; t < T0; ++t)
    if (live[t]) remap[t] = T++;
  L.T = T;
  L.tw = words_for(T);
  L.thr.assign((size_t)T * 2, 0);
  L.flags.assign(T, 0);
  L.vmask.assign((size_t)T * L.mw, 0);
  L.cmask.assign((size_t)T * L.tw, 0);
  L.extra_off.assign(T + 1, 0);
  for (uint32_t t0 = 0; t0 < T0; ++t0) {
    if (!live[t0]) continue;
    const uint32_t t = remap[t0];
    const LKey& k = keys[t0];
    L.thr[2 * t] = k.t0;
    L.thr[2 * t + 1] = k.t1;
    uint32_t fl = k.inv ? 1u : 0u;
    if (k.inv || (k.t0 == 0 && k.t1 == NEVER_THR)) L.nonmonotone = true;
    auto vp = planes(k.v, L.mw);
    std::vector<uint32_t> cl;
    for (uint32_t c : k.c) cl.push_back(remap[c]);
    std::sort(cl.begin(), cl.end());
    auto cp = planes(cl, L.tw);
    for (uint32_t w = 0; w < L.mw && !vp.empty(); ++w) L.vmask[(size_t)t * L.mw + w] = vp[0][w];
    for (uint32_t w = 0; w < L.tw && !cp.empty(); ++w) L.cmask[(size_t)t * L.tw + w] = cp[0][w];
    for (size_t p = 1; p < vp.size(); ++p)
      for (uint32_t w = 0; w < L.mw; ++w)
        if (vp[p][w]) {
          L.extra_src.push_back(w);
          L.extra_mask.push_back(vp[p][w]);
          fl |= 2u;
        }
    for (size_t p = 1; p < cp.size(); ++p)
      for (uint32_t w = 0; w < L.tw; ++w)
        if (cp[p][w]) {
          L.extra_src.push_back(L.mw + w);
          L.extra_mask.push_back(cp[p][w]);
          fl |= 2u;
        }
    L.flags[t] = fl;
    L.extra_off[t + 1] = (uint32_t)L.extra_src.size();
  }
  // distinct live roots and their users
  std::map<uint32_t, uint32_t> rid;
  for (uint32_t i = 0; i < L.m; ++i) {
    if (!live[root[i]]) continue;
    const uint32_t t = remap[root[i]];
    auto it = rid.find(t);
    uint32_t r;
    if (it == rid.end()) {
      r = (uint32_t)L.root_tn.size();
      rid.emplace(t, r);
      L.root_tn.push_back(t);
      L.root_users.resize(L.root_users.size() + L.mw, 0u);
    } else {
      r = it->second;
    }
    L.root_users[(size_t)r * L.mw + (i >> 5)] |= 1u << (i & 31);
  }
  L.R = (uint32_t)L.root_tn.size();
  L.vroot.assign(L.m, LocalFlat::NO_ROOT);
  for (uint32_t i = 0; i < L.m; ++i)
    if (live[root[i]]) L.vroot[i] = remap[root[i]];
  L.ladj_off.assign(L.m + 1, 0);
  for (uint32_t i = 0; i < L.m; ++i) {
    for (uint32_t w : g.adj[scc[i]])
      if (local[w] >= 0) L.ladj.push_back((uint32_t)local[w]);
    L.ladj_off[i + 1] = (uint32_t)L.ladj.size();
  }

  // findBestNode columns: in-edges from SCC members, with multiplicity (cpp:222-247)
  std::vector<std::vector<uint32_t>> col(L.m);
  for (uint32_t i = 0; i < L.m; ++i)
    for (uint32_t w : g.adj[scc[i]])
      if (local[w] >= 0) col[(uint32_t)local[w]].push_back(i);
  std::map<std::vector<uint32_t>, uint32_t> gid;
  std::vector<std::vector<uint32_t>> gcols;
  std::vector<uint32_t> member_of(L.m);
  for (uint32_t w = 0; w < L.m; ++w) {
    std::sort(col[w].begin(), col[w].end());
    auto it = gid.find(col[w]);
    if (it == gid.end()) {
      const uint32_t id = (uint32_t)gcols.size();
      gid.emplace(col[w], id);
      gcols.push_back(col[w]);
      member_of[w] = id;
    } else {
      member_of[w] = it->second;
    }
  }
  L.G = (uint32_t)gcols.size();
  L.grp_members.assign((size_t)L.G * L.mw, 0);
  L.grp_col.assign((size_t)L.G * L.mw, 0);
  L.grp_extra_off.assign(L.G + 1, 0);
  for (uint32_t w = 0; w < L.m; ++w) L.grp_members[(size_t)member_of[w] * L.mw + (w >> 5)] |= 1u << (w & 31);
  for (uint32_t gi = 0; gi < L.G; ++gi) {
    auto p = planes(gcols[gi], L.mw);
    for (uint32_t w = 0; w < L.mw && !p.empty(); ++w) L.grp_col[(size_t)gi * L.mw + w] = p[0][w];
    for (size_t q = 1; q < p.size(); ++q)
      for (uint32_t w = 0; w < L.mw; ++w) L.grp_extra.push_back(p[q][w]);
    L.grp_extra_off[gi + 1] = L.grp_extra_off[gi] + (uint32_t)(p.size() > 1 ? p.size() - 1 : 0);
  }
  if (!L.nonmonotone) {
    for (int pol = 0; pol < 2; ++pol) L.qmin[pol] = min_quorum_size(L, pol);
  }
  return L;
}

// ------------------------------------------------------------------------------------
// Text output
// ------------------------------------------------------------------------------------
// printQuorum (cpp:475-490).  The reference prints an indeterminate threshold for null
// quorum sets (cpp:405/454/482); this prints 0 there.
void print_quorum(const std::vector<uint32_t>& quorum, const Graph& g, std::ostream& out) {
  for (uint32_t v : quorum) {
    out << g.names[v] << " " << g.ids[v] << "\n( quorumslice: threshold = " << g.qsets[v].threshold << " ";
    for (uint32_t w : g.qsets[v].validators) out << g.ids[w] << " ";
    out << ") \n\n";
  }
  out << "\n";
}

// printGraphvizWithSccs + NodeWriter (cpp:492-530) in boost::write_graphviz layout.
void print_graphviz(const Graph& g, std::ostream& out, const Sccs& s) {
  const unsigned ncol = (unsigned)s.members.size();
  const unsigned offset = ncol ? 0xFFFFFFu / ncol : 0u;  // the reference divides by zero here
  out << "digraph G {\n";
  for (uint32_t v = 0; v < g.n(); ++v) {
    std::ostringstream c;
    c << std::setfill('0') << std::setw(6) << std::hex << offset * (unsigned)s.comp[v];
    const std::string& label = g.names[v].empty() ? g.ids[v] : g.names[v];
    out << v << "[style=filled color=\"#" << c.str() << "\" label=\"" << label << "\" fontcolor=\"white\"];\n";
  }
  for (uint32_t v = 0; v < g.n(); ++v)
    for (uint32_t w : g.adj[v]) out << v << "->" << w << " ;\n";
  out << "}\n";
}

// pageRank (cpp:532-583): float power iteration, rank starts at vertex 0.
std::vector<float> page_rank(const Graph& g, float m, float convergence, uint64_t max_iterations) {
  const size_t nv = g.n();
  std::vector<float> rank(nv, 0.0f);
  if (nv == 0) return rank;
  rank[0] = 1;
  std::vector<float> next = rank;
  float diff = convergence + 1;
  float sum = 1;
  for (uint64_t it = 0; diff > convergence && it < max_iterations; it++) {
    const float mS = m / nv;
    sum = nv * mS;
    std::fill(next.begin(), next.end(), mS);
    for (size_t v = 0; v < nv; ++v) {
      const float deg = float(g.adj[v].size());
      if (0 == deg) continue;
      const float share = (1 - m) / deg * rank[v];
      for (uint32_t w : g.adj[v]) {
        next[w] += share;
        sum += share;
      }
    }
    diff = 0;
    for (size_t v = 0; v < nv; ++v) {
      diff += std::fabs(next[v] - rank[v]);
      next[v] /= sum;
    }
    rank = next;
  }
  return rank;
}

// printPageRank (cpp:585-613): rank descending, label ascending on ties.
void print_page_rank(const Graph& g, std::ostream& out, const std::vector<float>& pr) {
  std::vector<std::pair<std::string, float>> rows;
  rows.reserve(g.n());
  for (uint32_t v = 0; v < g.n(); ++v) rows.emplace_back(g.names[v].empty() ? g.ids[v] : g.names[v], pr[v]);
  std::sort(rows.begin(), rows.end(), [](const std::pair<std::string, float>& a, const std::pair<std::string, float>& b) {
    return a.second == b.second ? a.first < b.first : a.second > b.second;
  });
  for (const auto& r : rows) out << r.first << ": " << r.second << "\n";
}

}  // namespace qi
