// Host driver of the device search: one engine, or the search tree sharded over several
// engines / GPUs (qi_driver.h).  Replaces checkMinimalQuorums' recursion
// (quorum_intersection.cpp:348-400) at its call site cpp:691.
#include "qi_driver.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>

#include "../../include/quorum_intersection.h"

namespace qi {
namespace {

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

bool key_less(const Witness& a, const Witness& b) {
  for (size_t w = 0; w < a.key.size() && w < b.key.size(); ++w)
    if (a.key[w] != b.key[w]) return a.key[w] < b.key[w];
  return a.depth < b.depth;
}

// Run f(e) for every engine index in `idx` on its own host thread; the first exception
// (by engine order) is rethrown after all threads have joined.
template <typename F>
void parallel_for(const std::vector<uint32_t>& idx, F&& f) {
  if (idx.size() == 1) {
    f(idx[0]);
    return;
  }
  std::vector<std::exception_ptr> err(idx.size());
  std::vector<std::thread> th;
  th.reserve(idx.size());
  for (size_t i = 0; i < idx.size(); ++i)
    th.emplace_back([&, i] {
      try {
        f(idx[i]);
      } catch (...) {
        err[i] = std::current_exception();
      }
    });
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

// device buffer owned for the duration of one hand-off
struct DevBuf {
  int dev = 0;
  void* p = nullptr;
  DevBuf(int d, size_t bytes) : dev(d), p(device_alloc(d, bytes)) {}
  ~DevBuf() { device_free(dev, p); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
};

void fill_witness(SearchOutcome& o, const Witness& w, const std::vector<uint32_t>& scc) {
  o.found = true;
  for (uint32_t v : w.q1_local) o.q1.push_back(scc[v]);
  for (uint32_t v : w.q2_local) o.q2.push_back(scc[v]);
}

}  // namespace

std::vector<Move> plan_rebalance(const std::vector<uint64_t>& sizes, uint64_t min_move) {
  const uint64_t world = sizes.size();
  uint64_t total = 0;
  for (uint64_t s : sizes) total += s;
  std::vector<std::pair<uint64_t, uint32_t>> donors, takers;  // (amount, engine)
  for (uint32_t r = 0; r < world; ++r) {
    const uint64_t target = total / world + (r < total % world ? 1 : 0);
    if (sizes[r] > target) donors.push_back({sizes[r] - target, r});
    if (sizes[r] < target) takers.push_back({target - sizes[r], r});
  }
  auto desc = [](const std::pair<uint64_t, uint32_t>& a, const std::pair<uint64_t, uint32_t>& b) {
    return a.first != b.first ? a.first > b.first : a.second > b.second;
  };
  std::sort(donors.begin(), donors.end(), desc);
  std::sort(takers.begin(), takers.end(), desc);
  std::vector<Move> moves;
  size_t i = 0, j = 0;
  while (i < donors.size() && j < takers.size()) {
    const uint64_t c = std::min(donors[i].first, takers[j].first);
    if (c >= min_move) moves.push_back({donors[i].second, takers[j].second, c});
    donors[i].first -= c;
    takers[j].first -= c;
    if (!donors[i].first) ++i;
    if (!takers[j].first) ++j;
  }
  return moves;
}

bool needs_rebalance(const std::vector<uint64_t>& sizes, uint64_t lanes) {
  if (sizes.empty()) return false;
  const uint64_t lo = *std::min_element(sizes.begin(), sizes.end());
  const uint64_t hi = *std::max_element(sizes.begin(), sizes.end());
  return hi > 0 && lo < lanes && hi > 2 * std::max<uint64_t>(lo, 1);
}

SearchOutcome search_front_scc(const Graph& g, const std::vector<uint32_t>& scc, int device, const SearchConfig& cfg) {
  if (device_count() <= device || device < 0)
    throw Error(QI_ERR_DEVICE, "no HIP device for the search (the MI355X path has no CPU fallback)");
  const bool trace = std::getenv("QI_TRACE") != nullptr;  // diagnostics: host-side phase times
  auto t0 = std::chrono::steady_clock::now();
  LocalFlat lf = flatten_local(g, scc);
  auto t1 = std::chrono::steady_clock::now();
  timing::add("flatten_local", ms_since(t0));
  auto sd = make_search_device(device, lf, cfg);
  auto t2 = std::chrono::steady_clock::now();
  timing::add("search_engine_setup", ms_since(t1));
  int steps = 0;
  while (sd->frontier_size()) {  // step() throws QI_ERR_STATE on repeated no-progress steps
    sd->step(0);
    ++steps;
  }
  timing::add("search", ms_since(t2));
  timing::add("search_kernels", sd->sum_kernel_ms());
  timing::count("search_launches", (double)sd->launches());
  timing::count("search_specialised_launches", (double)sd->specialized_launches());
  if (trace)
    std::fprintf(stderr, "[qi] flatten %.3f ms, create %.3f ms, %d steps %.3f ms\n", ms_since(t0) - ms_since(t1),
                 ms_since(t1) - ms_since(t2), steps, ms_since(t2));
  SearchOutcome o;
  o.nonmonotone = lf.nonmonotone;
  Witness w;
  const bool found = sd->best(&w);
  o.totals = found ? sd->reduce(true, w.key, w.depth) : sd->running_totals();
  if (found) fill_witness(o, w, scc);
  o.processed_nodes = found ? sd->running_totals().nodes : o.totals.nodes;
  o.launches = sd->launches();
  o.jit_launches = sd->specialized_launches();
  o.kernel_ms = sd->sum_kernel_ms();
  return o;
}

SearchOutcome search_front_scc_sharded(const Graph& g, const std::vector<uint32_t>& scc, const ShardConfig& sc,
                                       const SearchConfig& cfg) {
  const uint32_t E = (uint32_t)sc.engine_devices.size();
  if (E == 0) throw Error(QI_ERR_ARG, "sharded search without engines");
  const int ndev = device_count();
  for (int d : sc.engine_devices)
    if (d < 0 || d >= ndev) throw Error(QI_ERR_DEVICE, "no HIP device " + std::to_string(d) + " for a search engine");
  const bool trace = std::getenv("QI_TRACE") != nullptr;
  SearchOutcome o;
  o.engines = E;
  // ---- device contexts and peer access (xGMI) between every pair of used devices -------
  auto ti = std::chrono::steady_clock::now();
  const std::set<int> devset(sc.engine_devices.begin(), sc.engine_devices.end());
  o.devices = (uint32_t)devset.size();
  for (int d : devset) device_free(d, device_alloc(d, 64));  // context creation
  for (int a : devset)
    for (int b : devset)
      if (a < b) enable_peer(a, b);
  o.t_device_init_ms = ms_since(ti);

  LocalFlat lf = flatten_local(g, scc);
  o.nonmonotone = lf.nonmonotone;
  std::vector<std::unique_ptr<SearchDevice>> eng(E);
  // engine 0 first: a synchronous run-time specialisation compiles once and every other
  // engine loads the code object from the on-disk cache
  eng[0] = make_search_device(sc.engine_devices[0], lf, cfg);
  std::vector<uint32_t> rest;
  for (uint32_t e = 1; e < E; ++e) rest.push_back(e);
  if (!rest.empty()) parallel_for(rest, [&](uint32_t e) { eng[e] = make_search_device(sc.engine_devices[e], lf, cfg); });
  std::vector<uint32_t> all;
  for (uint32_t e = 0; e < E; ++e) all.push_back(e);
  const uint64_t ub = eng[0]->unit_bytes();
  for (uint32_t e = 1; e < E; ++e) eng[e]->clear_frontier();  // the root lives on engine 0 only
  // the engines' shared best key: a witness on one engine prunes the others inside their
  // chains (the reference stops at the first disjoint pair, cpp:369-377)
  struct PinnedWord {
    uint64_t* p = pinned_word_alloc();
    ~PinnedWord() { pinned_word_free(p); }
  } shared_best;
  struct Unshare {  // before the word is freed, whatever path leaves this function
    std::vector<std::unique_ptr<SearchDevice>>& eng;
    ~Unshare() {
      for (auto& e : eng)
        if (e) try { e->share_best(nullptr); } catch (...) {}
    }
  } unshare{eng};
  if (E > 1 && !std::getenv("QI_NO_SHARED_BEST"))  // (diagnostics: exchange between chains only)
    for (uint32_t e = 0; e < E; ++e) eng[e]->share_best(shared_best.p);

  // ---- (1) engine 0 grows the frontier from the root, (2) every engine keeps its deal ---
  const uint64_t target = sc.seed_units ? sc.seed_units : 2048ull * E;
  if (E > 1) eng[0]->step(target);
  const uint64_t n = eng[0]->frontier_size();
  if (E > 1 && n) {
    std::map<int, std::unique_ptr<DevBuf>> copy;  // the grown frontier on every used device
    const int d0 = sc.engine_devices[0];
    copy[d0].reset(new DevBuf(d0, n * ub));
    eng[0]->export_tail(n, copy[d0]->p);
    for (int d : devset)
      if (d != d0) {
        copy[d].reset(new DevBuf(d, n * ub));
        device_copy(copy[d]->p, d, copy[d0]->p, d0, n * ub);
      }
    parallel_for(all, [&](uint32_t e) {
      eng[e]->clear_frontier();
      eng[e]->import_units(n, copy[sc.engine_devices[e]]->p);
      eng[e]->keep_strided(e, E);
    });
  }

  // ---- (3) chains in parallel; best keys and rebalancing between chains -----------------
  bool has_best = false;
  Witness best;
  uint32_t owner = 0;
  for (;;) {
    std::vector<uint32_t> busy;
    for (uint32_t e = 0; e < E; ++e)
      if (eng[e]->frontier_size()) busy.push_back(e);
    if (busy.empty()) break;
    parallel_for(busy, [&](uint32_t e) { eng[e]->step(0); });
    ++o.exchanges;
    bool improved = false;
    for (uint32_t e = 0; e < E; ++e) {
      Witness w;
      if (eng[e]->best(&w) && (!has_best || key_less(w, best))) {
        best = w;
        owner = e;
        has_best = true;
        improved = true;
      }
    }
    if (improved)
      for (uint32_t e = 0; e < E; ++e) eng[e]->set_best(best.key, best.depth);
    std::vector<uint64_t> sizes(E);
    uint64_t total = 0;
    for (uint32_t e = 0; e < E; ++e) total += sizes[e] = eng[e]->frontier_size();
    if (trace) {
      std::fprintf(stderr, "[qi] shard round %llu: frontiers", (unsigned long long)o.exchanges);
      for (uint64_t s : sizes) std::fprintf(stderr, " %llu", (unsigned long long)s);
      std::fprintf(stderr, "%s\n", has_best ? " (best known)" : "");
    }
    if (!total) break;
    if (E > 1 && needs_rebalance(sizes, sc.lanes)) {
      for (const Move& mv : plan_rebalance(sizes, sc.min_move)) {
        const int ds = sc.engine_devices[mv.src], dd = sc.engine_devices[mv.dst];
        DevBuf bs(ds, mv.count * ub);
        eng[mv.src]->export_tail(mv.count, bs.p);  // the donor's tail: its preorder-last units
        if (dd == ds) {
          eng[mv.dst]->import_units(mv.count, bs.p);
        } else {
          DevBuf bd(dd, mv.count * ub);
          device_copy(bd.p, dd, bs.p, ds, mv.count * ub);
          eng[mv.dst]->import_units(mv.count, bd.p);
        }
        o.units_moved += mv.count;
      }
    }
  }

  for (uint32_t e = 0; e < E; ++e) {  // witnesses of the grow step when no round ran
    Witness w;
    if (eng[e]->best(&w) && (!has_best || key_less(w, best))) {
      best = w;
      owner = e;
      has_best = true;
    }
  }

  // ---- (4) preorder-exact totals against the global best witness -------------------------
  std::vector<Totals> tot(E);
  parallel_for(all, [&](uint32_t e) {
    tot[e] = has_best ? eng[e]->reduce(true, best.key, best.depth) : eng[e]->running_totals();
  });
  for (uint32_t e = 0; e < E; ++e) {
    o.processed_nodes += has_best ? eng[e]->running_totals().nodes : tot[e].nodes;
    o.totals.nodes += tot[e].nodes;
    o.totals.evals += tot[e].evals;
    o.totals.minq += tot[e].minq;
    o.totals.zero_fallback += tot[e].zero_fallback;
    o.totals.rounds += tot[e].rounds;
    o.totals.units += tot[e].units;
    o.totals.wave_iters += tot[e].wave_iters;
    o.totals.coop_phases += tot[e].coop_phases;
    o.launches += eng[e]->launches();
    o.jit_launches += eng[e]->specialized_launches();
    o.kernel_ms += eng[e]->sum_kernel_ms();
  }
  if (has_best) {
    Witness w;
    eng[owner]->best(&w);
    fill_witness(o, w, scc);
  }
  return o;
}

}  // namespace qi
