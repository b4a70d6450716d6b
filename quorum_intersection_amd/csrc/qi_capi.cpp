// C-ABI (include/quorum_intersection.h) and the host driver that replaces
// solve(Graph) (quorum_intersection.cpp:615-707).  Device work goes through
// qi_device.h; there is no CPU fallback: without a GPU every device entry point
// returns QI_ERR_DEVICE.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>

#include "../../include/quorum_intersection.h"
#include "qi_device.h"
#include "qi_driver.h"
#include "qi_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const qi::Error& e) {
    return fail(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return fail(QI_ERR_CAPACITY, "out of host memory");
  } catch (const std::exception& e) {
    return fail(QI_ERR_STATE, e.what());
  }
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

struct qi_fbas {
  qi::Graph g;
  qi::Sccs sccs;
  int device = 0;
  uint32_t edges = 0;
  std::unique_ptr<qi::GlobalFlat> gflat;
  std::unique_ptr<qi::GfpDevice> gfp;

  qi::GfpDevice& gfp_dev() {
    if (!gfp) {
      if (qi::device_count() <= device || device < 0)
        throw qi::Error(QI_ERR_DEVICE, "no HIP device " + std::to_string(device) + " (the MI355X path has no CPU fallback)");
      if (!gflat) {
        qi::timing::Scope t("flatten_global");
        gflat.reset(new qi::GlobalFlat(qi::flatten_global(g)));
      }
      qi::timing::Scope t("gfp_device_setup");
      gfp = qi::make_gfp_device(device, *gflat);
    }
    return *gfp;
  }
};

struct qi_search {
  qi_fbas* f = nullptr;
  qi::LocalFlat lf;
  std::unique_ptr<qi::SearchDevice> sd;
};

namespace {

uint32_t words64(uint32_t n) { return (n + 63) / 64; }

// Per-SCC quorum checks (cpp:643-672) as one batched device call.
std::vector<uint32_t> scc_quorum_check(qi_fbas* f, std::vector<std::vector<uint32_t>>* quorums) {
  const uint32_t n = f->g.n(), W = words64(n);
  const uint32_t C = (uint32_t)f->sccs.members.size();
  std::vector<uint32_t> with;
  if (C == 0) return with;
  std::vector<uint64_t> masks((size_t)C * W, 0), out((size_t)C * W, 0);
  for (uint32_t c = 0; c < C; ++c)
    for (uint32_t v : f->sccs.members[c]) masks[(size_t)c * W + v / 64] |= 1ull << (v % 64);
  {
    qi::GfpDevice& gd = f->gfp_dev();
    qi::timing::Scope t("scc_checks");
    gd.run(masks.data(), masks.data(), C, out.data());
  }
  for (uint32_t c = 0; c < C; ++c) {
    bool any = false;
    std::vector<uint32_t> q;
    for (uint32_t v : f->sccs.members[c])  // survivors in component order (cpp:156)
      if ((out[(size_t)c * W + v / 64] >> (v % 64)) & 1ull) {
        any = true;
        q.push_back(v);
      }
    if (any) {
      with.push_back(c);
      if (quorums) quorums->push_back(std::move(q));
    }
  }
  return with;
}

qi::SearchConfig make_cfg(uint32_t grow, uint32_t run, uint32_t blocks, uint32_t jit = 0, uint32_t batch = 0,
                          uint32_t tiebreak = 0, uint32_t tie_seed = 0) {
  qi::SearchConfig c;
  c.tiebreak = tiebreak;
  c.tie_seed = tie_seed;
  c.jit = jit;
  if (batch) c.batch = batch;
  if (grow) c.grow_budget = grow;
  if (run) c.run_budget = run;
  if (blocks) c.max_blocks = blocks;
  return c;
}

// Engines of a search from the options: device_mask bits (0 = the FBAS's device), one
// engine per device unless `engines` says otherwise (round-robin over the devices).
std::vector<int> engine_devices(const qi_fbas* f, const qi_solve_opts* opts) {
  std::vector<int> devs;
  const uint32_t mask = opts ? opts->device_mask : 0u;
  for (int d = 0; d < 32; ++d)
    if ((mask >> d) & 1u) devs.push_back(d);
  if (devs.empty()) devs.push_back(f->device);
  const uint32_t E = (opts && opts->engines) ? opts->engines : (uint32_t)devs.size();
  if (E > 64) throw qi::Error(QI_ERR_ARG, "at most 64 search engines");
  std::vector<int> out;
  for (uint32_t e = 0; e < E; ++e) out.push_back(devs[e % devs.size()]);
  return out;
}

qi::SearchOutcome run_search(qi_fbas* f, const qi::SearchConfig& cfg, const qi_solve_opts* opts) {
  const auto& scc = f->sccs.members.front();
  const std::vector<int> ed = engine_devices(f, opts);
  if (ed.size() == 1) return qi::search_front_scc(f->g, scc, ed[0], cfg);
  qi::ShardConfig sc;
  sc.engine_devices = ed;
  return qi::search_front_scc_sharded(f->g, scc, sc, cfg);
}

}  // namespace

extern "C" {

const char* qi_last_error(void) { return g_err.c_str(); }
int qi_abi_version(void) { return QI_ABI_VERSION; }
int qi_device_count(void) { return qi::device_count(); }

const char* qi_timing_json(void) {
  thread_local std::string s;
  s = qi::timing::json();
  return s.c_str();
}

int qi_device_warmup(int device, double* ms) {
  return guarded([&] {
    auto t0 = std::chrono::steady_clock::now();
    if (qi::device_count() <= device || device < 0) throw qi::Error(QI_ERR_DEVICE, "no HIP device " + std::to_string(device));
    qi::device_free(device, qi::device_alloc(device, 64));
    qi::device_prepare(device);  // the first stream (hardware queue) and the library's code object
    if (ms) *ms = ms_since(t0);
    return QI_OK;
  });
}

int qi_fbas_from_json(const char* json, size_t len, int device, qi_fbas** out) {
  if (!json || !out) return fail(QI_ERR_ARG, "null argument");
  return guarded([&] {
    std::unique_ptr<qi_fbas> f(new qi_fbas);
    std::vector<qi::StellarNode> nodes;
    {
      qi::timing::Scope t("parse");
      nodes = qi::parse_stellar_json(json, len);
    }
    {
      qi::timing::Scope t("graph_scc");
      f->g = qi::build_graph(nodes);
      f->sccs = qi::strong_components(f->g);
    }
    f->device = device;
    for (const auto& a : f->g.adj) f->edges += (uint32_t)a.size();
    *out = f.release();
    return QI_OK;
  });
}

void qi_fbas_destroy(qi_fbas* f) { delete f; }
uint32_t qi_fbas_num_vertices(const qi_fbas* f) { return f ? f->g.n() : 0; }
uint32_t qi_fbas_num_edges(const qi_fbas* f) { return f ? f->edges : 0; }
uint32_t qi_fbas_num_sccs(const qi_fbas* f) { return f ? (uint32_t)f->sccs.members.size() : 0; }

int qi_fbas_scc_ids(const qi_fbas* f, uint32_t* comp) {
  if (!f || !comp) return fail(QI_ERR_ARG, "null argument");
  std::memcpy(comp, f->sccs.comp.data(), f->sccs.comp.size() * 4);
  return QI_OK;
}

int qi_fbas_adjacency(const qi_fbas* f, uint32_t* offsets, uint32_t* targets) {
  if (!f || !offsets || !targets) return fail(QI_ERR_ARG, "null argument");
  uint32_t o = 0;
  for (uint32_t v = 0; v < f->g.n(); ++v) {
    offsets[v] = o;
    for (uint32_t w : f->g.adj[v]) targets[o++] = w;
  }
  offsets[f->g.n()] = o;
  return QI_OK;
}

int qi_fbas_vertex(const qi_fbas* f, uint32_t v, const char** public_key, const char** name) {
  if (!f || v >= f->g.n()) return fail(QI_ERR_ARG, "bad vertex");
  if (public_key) *public_key = f->g.ids[v].c_str();
  if (name) *name = f->g.names[v].c_str();
  return QI_OK;
}

int qi_gfp_batch(qi_fbas* f, const uint64_t* nodes, const uint64_t* avail, uint32_t count, uint64_t* out) {
  if (!f || (count && (!nodes || !avail || !out))) return fail(QI_ERR_ARG, "null argument");
  return guarded([&] {
    f->gfp_dev().run(nodes, avail, count, out);
    return QI_OK;
  });
}

int qi_gfp_batch_static(qi_fbas* f, const uint64_t* d_nodes, const uint64_t* d_avail, uint32_t count, uint64_t* d_out,
                        void* stream) {
  if (!f || (count && (!d_nodes || !d_avail || !d_out))) return fail(QI_ERR_ARG, "null argument");
  // set-up (table upload, scratch address) allocates and belongs to an earlier call
  if (!f->gfp)
    return fail(QI_ERR_STATE, "qi_gfp_batch_static: no device image yet; call qi_gfp_batch or qi_solve once on this "
                              "qi_fbas first (set-up allocates, this entry point never does)");
  return guarded([&] {
    f->gfp->run_static(d_nodes, d_avail, count, d_out, stream);
    return QI_OK;
  });
}

int qi_solve(qi_fbas* f, const qi_solve_opts* opts, qi_solve_result* res, uint32_t* q1, uint32_t* q2) {
  if (!f || !res) return fail(QI_ERR_ARG, "null argument");
  if (opts && opts->tiebreak > QI_TIE_RANDOM) return fail(QI_ERR_ARG, "tiebreak: QI_TIE_LOWEST or QI_TIE_RANDOM");
  return guarded([&] {
    std::memset(res, 0, sizeof *res);
    res->n_vertices = f->g.n();
    res->n_sccs = (uint32_t)f->sccs.members.size();
    auto t0 = std::chrono::steady_clock::now();
    auto with = scc_quorum_check(f, nullptr);
    res->t_scc_ms = ms_since(t0);
    res->sccs_with_quorum = (uint32_t)with.size();
    res->scc_evals = res->n_sccs;
    res->evals = res->scc_evals;
    res->front_size = f->sccs.members.empty() ? 0 : (uint32_t)f->sccs.members.front().size();
    if (with.size() != 1) {  // cpp:681-688
      res->verdict = 0;
      return QI_OK;
    }
    res->searched = 1;
    qi::SearchConfig cfg = make_cfg(opts ? opts->grow_budget : 0, opts ? opts->run_budget : 0,
                                    opts ? opts->max_blocks : 0, opts ? opts->jit : 0, opts ? opts->batch : 0,
                                    opts ? opts->tiebreak : 0, opts ? opts->tie_seed : 0);
    auto t1 = std::chrono::steady_clock::now();
    qi::SearchOutcome o = run_search(f, cfg, opts);
    res->t_search_ms = ms_since(t1);
    res->t_kernel_ms = o.kernel_ms;
    res->launches = o.launches;
    res->jit_launches = (uint32_t)o.jit_launches;
    res->engines = o.engines;
    res->devices = o.devices;
    res->units_moved = o.units_moved;
    res->t_device_init_ms = o.t_device_init_ms;
    res->nodes_processed = o.processed_nodes;
    res->nodes = o.totals.nodes;
    res->evals += o.totals.evals;
    res->minq = o.totals.minq;
    res->zero_fallback = o.totals.zero_fallback;
    res->rounds = o.totals.rounds;
    res->nonmonotone = o.nonmonotone ? 1u : 0u;
    res->verdict = o.found ? 0 : 1;
    res->q1_len = (uint32_t)o.q1.size();
    res->q2_len = (uint32_t)o.q2.size();
    if (q1) std::copy(o.q1.begin(), o.q1.end(), q1);
    if (q2) std::copy(o.q2.begin(), o.q2.end(), q2);
    return QI_OK;
  });
}

// solve(istream&, ostream&, verbose, graphviz) text (cpp:615-716, 790-797)
int qi_solve_text(qi_fbas* f, int verbose, int graphviz, char** text, int* verdict) {
  return qi_solve_text_ex(f, verbose, graphviz, nullptr, text, verdict);
}

int qi_solve_text_ex(qi_fbas* f, int verbose, int graphviz, const qi_solve_opts* opts, char** text, int* verdict) {
  if (!f || !text || !verdict) return fail(QI_ERR_ARG, "null argument");
  if (opts && opts->tiebreak > QI_TIE_RANDOM) return fail(QI_ERR_ARG, "tiebreak: QI_TIE_LOWEST or QI_TIE_RANDOM");
  return guarded([&] {
    std::ostringstream out;
    const auto& S = f->sccs.members;
    if (graphviz) qi::print_graphviz(f->g, out, f->sccs);
    if (verbose) out << "total number of strongly connected components: " << S.size() << "\n";
    std::vector<std::vector<uint32_t>> quorums;
    auto with = scc_quorum_check(f, &quorums);
    if (verbose)
      for (const auto& q : quorums) {
        out << "found quorum inside of a strongly connected component:\n";
        qi::print_quorum(q, f->g, out);
      }
    bool result;
    if (verbose && !S.empty()) {  // the reference reads sccs.front() of an empty vector here (UB)
      out << "number of strongly connected components containing some quorum: " << with.size() << "\n";
      out << "size of the main strongly connected component: " << S.front().size() << "\n";
      out << "main strongly connected component (all minimal quorums are included in it; "
          << "small size means small resilience of the network):\n";
      qi::print_quorum(S.front(), f->g, out);
    }
    if (with.size() != 1) {
      if (verbose)
        out << "network's configuration is broken - more than one strongly connected component contains a quorum - "
            << with.size() << "\n";
      result = false;
    } else {
      qi::SearchConfig cfg = make_cfg(opts ? opts->grow_budget : 0, opts ? opts->run_budget : 0,
                                      opts ? opts->max_blocks : 0, opts ? opts->jit : 0, opts ? opts->batch : 0,
                                    opts ? opts->tiebreak : 0, opts ? opts->tie_seed : 0);
      qi::SearchOutcome o = run_search(f, cfg, opts);
      if (o.found) {
        if (verbose) {
          out << "found two non-intersecting quorums\n";
          out << "first quorum:\n";
          qi::print_quorum(o.q1, f->g, out);
          out << "second quorum:\n";
          qi::print_quorum(o.q2, f->g, out);
        }
        result = false;
      } else {
        if (verbose) out << "all quorums are intersecting\n";
        result = true;
      }
    }
    out << (result ? "true" : "false") << "\n";
    const std::string s = out.str();
    char* p = (char*)std::malloc(s.size() + 1);
    if (!p) throw std::bad_alloc();
    std::memcpy(p, s.c_str(), s.size() + 1);
    *text = p;
    *verdict = result ? 1 : 0;
    return QI_OK;
  });
}

int qi_pagerank_text(qi_fbas* f, float dangling, float convergence, uint64_t max_iterations, char** text) {
  if (!f || !text) return fail(QI_ERR_ARG, "null argument");
  return guarded([&] {
    std::ostringstream out;
    auto pr = qi::page_rank(f->g, dangling, convergence, max_iterations);
    out << "PageRank:\n";
    qi::print_page_rank(f->g, out, pr);
    const std::string s = out.str();
    char* p = (char*)std::malloc(s.size() + 1);
    if (!p) throw std::bad_alloc();
    std::memcpy(p, s.c_str(), s.size() + 1);
    *text = p;
    return QI_OK;
  });
}

void qi_free(void* p) { std::free(p); }

// ---------------------------------------------------------------------------------
// Step-wise search
// ---------------------------------------------------------------------------------
int qi_search_create(qi_fbas* f, const qi_search_opts* opts, qi_search** out) {
  if (!f || !out) return fail(QI_ERR_ARG, "null argument");
  return guarded([&] {
    auto with = scc_quorum_check(f, nullptr);
    if (with.size() != 1)
      throw qi::Error(QI_ERR_STATE, "no search: " + std::to_string(with.size()) + " SCCs contain a quorum");
    std::unique_ptr<qi_search> s(new qi_search);
    s->f = f;
    s->lf = qi::flatten_local(f->g, f->sccs.members.front());
    s->sd = qi::make_search_device(f->device, s->lf,
                                   make_cfg(opts ? opts->grow_budget : 0, opts ? opts->run_budget : 0,
                                            opts ? opts->max_blocks : 0, opts ? opts->jit : 0,
                                            opts ? opts->batch : 0));
    *out = s.release();
    return QI_OK;
  });
}

void qi_search_destroy(qi_search* s) { delete s; }
uint32_t qi_search_unit_bytes(const qi_search* s) { return s ? s->sd->unit_bytes() : 0; }
uint32_t qi_search_key_words(const qi_search* s) { return s ? s->sd->key_words() : 0; }

int qi_search_reset(qi_search* s) {
  if (!s) return fail(QI_ERR_ARG, "null");
  return guarded([&] { s->sd->reset_root(); return QI_OK; });
}

int qi_search_clear(qi_search* s) {
  if (!s) return fail(QI_ERR_ARG, "null");
  return guarded([&] { s->sd->clear_frontier(); return QI_OK; });
}

static int search_step(qi_search* s, uint64_t until, qi_step_info* info) {
  if (!s) return fail(QI_ERR_ARG, "null");
  return guarded([&] {
    qi::StepInfo si = s->sd->step(until);
    if (info) {
      info->frontier_in = si.frontier_in;
      info->frontier_out = si.frontier_out;
      info->processed = si.processed;
      info->budget = si.budget;
      info->blocks = si.blocks;
      info->new_witnesses = si.new_witnesses;
      info->kernel_ms = si.kernel_ms;
      info->specialized = si.specialized ? 1u : 0u;
      info->launches = si.launches;
      info->dispatches = si.dispatches;
      info->pad = 0;
      info->dispatch_ms = si.dispatch_ms;
    }
    return QI_OK;
  });
}

int qi_search_step(qi_search* s, qi_step_info* info) { return search_step(s, 0, info); }
int qi_search_grow(qi_search* s, uint64_t target, qi_step_info* info) {
  return search_step(s, target ? target : 1, info);
}

uint64_t qi_search_frontier(const qi_search* s) { return s ? s->sd->frontier_size() : 0; }

int qi_search_keep_strided(qi_search* s, uint64_t offset, uint64_t stride) {
  if (!s || stride == 0) return fail(QI_ERR_ARG, "null or stride 0");
  return guarded([&] { s->sd->keep_strided(offset, stride); return QI_OK; });
}

int qi_search_keep_slice(qi_search* s, uint64_t begin, uint64_t end) {
  if (!s) return fail(QI_ERR_ARG, "null");
  return guarded([&] { s->sd->keep_slice(begin, end); return QI_OK; });
}

int qi_search_export(qi_search* s, uint64_t count, void* device_dst) {
  if (!s || (count && !device_dst)) return fail(QI_ERR_ARG, "null");
  return guarded([&] { s->sd->export_tail(count, device_dst); return QI_OK; });
}

int qi_search_import(qi_search* s, uint64_t count, const void* device_src) {
  if (!s || (count && !device_src)) return fail(QI_ERR_ARG, "null");
  return guarded([&] { s->sd->import_units(count, device_src); return QI_OK; });
}

int qi_search_local_best(qi_search* s, uint32_t* key, uint32_t* depth) {
  if (!s) return fail(QI_ERR_ARG, "null");
  qi::Witness w;
  if (!s->sd->best(&w)) return 0;
  if (key) std::copy(w.key.begin(), w.key.end(), key);
  if (depth) *depth = w.depth;
  return 1;
}

int qi_search_set_best(qi_search* s, const uint32_t* key, uint32_t depth) {
  if (!s || !key) return fail(QI_ERR_ARG, "null");
  std::vector<uint32_t> k(key, key + s->sd->key_words());
  s->sd->set_best(k, depth);
  return QI_OK;
}

int qi_search_share_best(qi_search* s, void* host_word) {
  if (!s) return fail(QI_ERR_ARG, "null");
  return guarded([&] {
    s->sd->share_best((uint64_t*)host_word);
    return QI_OK;
  });
}

int qi_search_reduce(qi_search* s, const uint32_t* key, uint32_t depth, qi_totals* out) {
  if (!s || !out) return fail(QI_ERR_ARG, "null");
  return guarded([&] {
    std::vector<uint32_t> k;
    if (key) k.assign(key, key + s->sd->key_words());
    qi::Totals t = key ? s->sd->reduce(true, k, depth) : s->sd->reduce(false, k, 0);
    out->nodes = t.nodes;
    out->evals = t.evals;
    out->minq = t.minq;
    out->zero_fallback = t.zero_fallback;
    out->rounds = t.rounds;
    out->units = t.units;
    out->wave_iters = t.wave_iters;
    out->coop_phases = t.coop_phases;
    for (int q = 0; q < 8; ++q) out->stamps[q] = t.dbg[q];
    return QI_OK;
  });
}

int qi_search_witness(qi_search* s, uint32_t* q1, uint32_t* q1_len, uint32_t* q2, uint32_t* q2_len) {
  if (!s) return fail(QI_ERR_ARG, "null");
  qi::Witness w;
  if (!s->sd->best(&w)) return fail(QI_ERR_STATE, "no witness");
  const auto& scc = s->lf.scc;
  if (q1) for (size_t i = 0; i < w.q1_local.size(); ++i) q1[i] = scc[w.q1_local[i]];
  if (q2) for (size_t i = 0; i < w.q2_local.size(); ++i) q2[i] = scc[w.q2_local[i]];
  if (q1_len) *q1_len = (uint32_t)w.q1_local.size();
  if (q2_len) *q2_len = (uint32_t)w.q2_local.size();
  return QI_OK;
}

int qi_search_restart(qi_search* s) {
  if (!s) return fail(QI_ERR_ARG, "null");
  return guarded([&] {
    s->sd->drop_log();
    s->sd->reset_root();
    return QI_OK;
  });
}

double qi_search_kernel_ms(const qi_search* s) { return s ? s->sd->sum_kernel_ms() : 0.0; }

int qi_search_wait_jit(qi_search* s) {
  if (!s) return fail(QI_ERR_ARG, "null");
  return s->sd->wait_jit() ? 1 : 0;
}

int qi_fbas_jit_precompile(qi_fbas* f, double* ms) {
  if (!f) return fail(QI_ERR_ARG, "null");
  return guarded([&] {
    if (f->sccs.members.empty()) throw qi::Error(QI_ERR_STATE, "empty FBAS");
    auto t0 = std::chrono::steady_clock::now();
    qi::LocalFlat lf = qi::flatten_local(f->g, f->sccs.members.front());
    std::string log;
    if (lf.nonmonotone) throw qi::Error(QI_ERR_UNSUPPORTED, "jit: threshold-0 SCCs run the ordered kernel");
    if (!qi::jit_precompile(lf, &log)) throw qi::Error(QI_ERR_UNSUPPORTED, "jit: " + log);
    if (ms) *ms = ms_since(t0);
    return QI_OK;
  });
}

int qi_hash_iteration_order(const uint32_t* keys, uint32_t n_keys, const uint32_t* seq, uint32_t n_seq,
                            uint32_t* out, uint32_t* n_out) {
  if ((n_keys && !keys) || (n_seq && !seq) || !out || !n_out) return fail(QI_ERR_ARG, "null argument");
  return guarded([&] {
    *n_out = qi::hash_iteration_order(keys, n_keys, seq, n_seq, out);
    return QI_OK;
  });
}

int qi_search_shape(const qi_search* s, qi_shape* out) {
  if (!s || !out) return fail(QI_ERR_ARG, "null");
  const qi::LocalFlat& L = s->lf;
  out->m = L.m;
  out->mask_words = L.mw;
  out->tns = L.T;
  out->tn_words = L.tw;
  uint32_t wc = 0;
  for (uint32_t t = 0; t < L.T; ++t) {
    bool any = false;
    for (uint32_t w = 0; w < L.tw; ++w) any |= L.cmask[(size_t)t * L.tw + w] != 0;
    wc += any ? 1u : 0u;
  }
  out->tns_with_children = wc;
  out->roots = L.R;
  out->groups = L.G;
  out->extra_terms = (uint32_t)L.extra_src.size();
  out->qmin_inside = L.qmin[0];
  out->qmin_outside = L.qmin[1];
  return QI_OK;
}

}  // extern "C"
