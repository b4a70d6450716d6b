/*
 * quorum_intersection.h -- C-ABI of the MI355X-native quorum-intersection checker.
 *
 * The reference (fixxxedpoint/quorum_intersection, quorum_intersection.cpp) is a single
 * C++14 executable with no library or FFI surface.  Its only contract is the process
 * interface (stellarbeat JSON on stdin, -h/-v/-g/-t/-p/-i/-m/-c, "true"/"false" and
 * exit 0/1, cpp:744-800), which the `quorum_intersection` binary built from this library
 * reproduces.  This header is the seam beneath it: plain pointers and sizes, no C++ or
 * torch types, int status codes (0 = OK) and a thread-local error string.  Each entry
 * point names the reference code it replaces.
 *
 * Threading: one host thread per qi_fbas / qi_search (the reference's findBestNode RNG
 * and search counter are process-global statics, cpp:207/258).
 */
#ifndef QUORUM_INTERSECTION_H_
#define QUORUM_INTERSECTION_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QI_ABI_VERSION 4

enum {
  QI_OK = 0,
  QI_ERR_PARSE = 1,       /* JSON / schema error: the reference throws ptree_error and aborts */
  QI_ERR_DEVICE = 2,      /* HIP runtime error, or no GPU: the product never falls back to CPU */
  QI_ERR_ARG = 3,
  QI_ERR_UNSUPPORTED = 4, /* the one input class the drop-in refuses: a searched SCC (sccs.front())
                             of more than 1024 vertices or more than 1024 distinct threshold
                             nodes (the largest compiled kernel shape); the reference searches
                             any size (plain vectors, cpp:140-346) */
  QI_ERR_CAPACITY = 5,
  QI_ERR_STATE = 6
};

/* findBestNode tie-break (cpp:203-250).  The reference samples uniformly among the
 * maximal in-degree vertices; QI_TIE_LOWEST picks the lowest vertex index of that set,
 * which is one of the reference's possible executions and makes counts reproducible.
 * QI_TIE_RANDOM is the reference's own rule with a reproducible draw: uniform over the
 * maximal in-degree vertices of Q \ D, drawn from a hash of (qi_solve_opts.tie_seed, the
 * node's path, its depth) instead of a process-global engine (cpp:207).  Verdicts do not
 * depend on the rule; node counts and, on early exits, the witness do.  Not available for
 * SCCs with threshold-0 quorum sets or beyond 256 vertices (QI_ERR_UNSUPPORTED). */
enum { QI_TIE_LOWEST = 0, QI_TIE_RANDOM = 1 };

typedef struct qi_fbas qi_fbas;
typedef struct qi_search qi_search;

const char* qi_last_error(void);
int qi_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int qi_device_count(void);
/* Create the HIP context of `device` now (runtime + device initialisation, which the
 * first device call would otherwise pay); *ms = wall time.  Lets a caller report device
 * init apart from time-to-verdict. */
int qi_device_warmup(int device, double* ms);
/* With QI_TIMING set in the environment: the phase times of this process so far as a JSON
 * object ({"parse_ms": .., "graph_scc_ms": .., "flatten_global_ms": .., "gfp_device_setup_ms":
 * .., "scc_checks_ms": .., "flatten_local_ms": .., "search_engine_setup_ms": .., "search_ms":
 * .., "search_kernels_ms": ..}); "{}" otherwise.  Valid until the thread's next call. */
const char* qi_timing_json(void);

/* ---------------------------------------------------------------------------------
 * FBAS: parseStellarConfigurationJSON + buildDependencyGraph + strong_components
 * (cpp:402-473, 615-633), host side.  `device` is the HIP ordinal used by the device
 * entry points below (checked lazily, at the first device call).
 * ------------------------------------------------------------------------------- */
int qi_fbas_from_json(const char* json, size_t len, int device, qi_fbas** out);
void qi_fbas_destroy(qi_fbas* f);
uint32_t qi_fbas_num_vertices(const qi_fbas* f);
uint32_t qi_fbas_num_edges(const qi_fbas* f);
uint32_t qi_fbas_num_sccs(const qi_fbas* f);
/* comp[v] = boost::strong_components id of vertex v (cpp:621); n entries. */
int qi_fbas_scc_ids(const qi_fbas* f, uint32_t* comp);
/* Adjacency in insertion order (cpp:458): offsets[n+1], targets[num_edges]. */
int qi_fbas_adjacency(const qi_fbas* f, uint32_t* offsets, uint32_t* targets);
/* Vertex strings (publicKey, name); pointers valid while f lives. */
int qi_fbas_vertex(const qi_fbas* f, uint32_t v, const char** public_key, const char** name);

/* ---------------------------------------------------------------------------------
 * containsQuorum (cpp:140-177), batched on the GPU: for query b, the greatest fixpoint
 * of f(X) = {x in X : x has a quorum slice in X ∪ F} starting from X = nodes_b ∩ avail_b
 * with F = avail_b \ nodes_b always available.  Masks are ceil(n/64) uint64 words per
 * query (bit v%64 of word v/64 = vertex v), host memory.  out_b = surviving vertices
 * (the reference returns them in the order of `nodes`; as a set this is the same).
 * ------------------------------------------------------------------------------- */
int qi_gfp_batch(qi_fbas* f, const uint64_t* nodes, const uint64_t* avail, uint32_t count, uint64_t* out);

/* The same batched containsQuorum for callers that cannot allocate (code under HIP graph
 * capture, tight serving loops, harnesses that forbid hipMalloc).  No counterpart in the
 * reference.  nodes / avail / out are DEVICE memory on the qi_fbas's HIP device, laid out
 * as for qi_gfp_batch.  The per-query state (available set, candidate set, one byte per
 * threshold node) and a counter header live in a fixed array of QI_STATIC_SCRATCH_BYTES
 * that the library holds on every GPU it runs on until the process ends; the call makes no
 * hipMalloc / hipFree / hipHostMalloc and no other allocating call.  `stream`: a
 * hipStream_t to enqueue on without synchronising, or NULL to run on HIP's default stream
 * of that device and wait.  Set-up is not part of it: the qi_fbas must have run qi_gfp_batch or qi_solve
 * once (that uploads the threshold-node tables), else QI_ERR_STATE.  count queries whose
 * state exceeds the array: QI_ERR_CAPACITY (split the batch).  Every call on a GPU uses
 * that GPU's one array: calls that overlap on one GPU (other threads, other streams) race. */
#define QI_STATIC_SCRATCH_BYTES (4u << 20)
int qi_gfp_batch_static(qi_fbas* f, const uint64_t* d_nodes, const uint64_t* d_avail, uint32_t count,
                        uint64_t* d_out, void* stream);

/* ---------------------------------------------------------------------------------
 * solve(Graph) (cpp:615-707): per-SCC quorum checks (cpp:649-672, batched on the GPU),
 * the "exactly one SCC contains a quorum" rule (cpp:681-688) and the branch-and-bound
 * search on sccs.front() (checkMinimalQuorums, cpp:348-400 / 691) on the GPU.
 * ------------------------------------------------------------------------------- */
typedef struct {
  uint32_t tiebreak;       /* QI_TIE_LOWEST or QI_TIE_RANDOM */
  uint32_t grow_budget;    /* 0 = default: per-lane node budget while the frontier grows */
  uint32_t run_budget;     /* 0 = default: per-lane node budget at full occupancy */
  uint32_t max_blocks;     /* 0 = default (8 wavefronts per CU) */
  uint32_t jit;            /* run-time specialised search kernel: 0 auto (from the on-disk
                              cache if there, else compiled in the background once a search
                              needs >= 3 launches), 1 off, 2 before launch 1, 3 = 2 +
                              diagnostic section stamps (not for measurement), 4 cache only
                              (never compiles; the CLI's choice) */
  uint32_t batch;          /* 0 = default: search launches chained on the device per host
                              synchronisation (each reads its input count from the previous) */
  uint32_t engines;        /* search shards: 0 = one per selected device.  Shards split the
                              search tree by branch prefix (one host thread + HIP stream each,
                              round-robin over the devices); >1 on one device runs the same
                              sharded code path on one GPU */
  uint32_t device_mask;    /* HIP devices of the search, bit d = device d; 0 = the qi_fbas
                              device only.  Units move between devices over xGMI
                              (hipMemcpyPeerAsync) */
  uint32_t tie_seed;       /* QI_TIE_RANDOM: seed of the draws */
} qi_solve_opts;

typedef struct {
  int32_t verdict;         /* 1 = all quorums intersect ("true"), 0 = "false" */
  int32_t searched;        /* 1 if checkMinimalQuorums ran */
  uint32_t n_vertices;
  uint32_t n_sccs;
  uint32_t sccs_with_quorum;
  uint32_t front_size;     /* |sccs.front()| */
  uint64_t nodes;          /* iterateMinimalQuorums calls, preorder-exact (cpp:258) */
  uint64_t evals;          /* containsQuorum calls the reference makes, all call sites */
  uint64_t scc_evals;      /* of which per-SCC checks (cpp:658) */
  uint64_t minq;           /* minimal quorums visited (cpp:361) */
  uint64_t zero_fallback;  /* findBestNode default *quorum.begin() taken (cpp:221) */
  uint64_t rounds;         /* Jacobi fixpoint rounds executed on the device (work metric) */
  uint64_t launches;       /* search kernel launches */
  uint32_t q1_len, q2_len; /* witness sizes (verdict 0 after a search) */
  double t_scc_ms;         /* per-SCC checks, host wall */
  double t_search_ms;      /* search, host wall */
  double t_kernel_ms;      /* search kernels, HIP events */
  uint32_t nonmonotone;    /* 1 if the searched SCC has threshold-0 quorum sets: the
                              reference's fixpoints then depend on its sweep orders (D in
                              branch order, toRemove in libstdc++ unordered_set order); the
                              search then runs the order-exact kernel (same counts) */
  uint32_t jit_launches;   /* launches that ran the run-time specialised kernel */
  uint32_t engines;        /* search shards that ran */
  uint32_t devices;        /* distinct HIP devices they ran on */
  uint64_t units_moved;    /* frontier units handed between shards (rebalancing) */
  double t_device_init_ms; /* HIP runtime / device contexts of the search devices, host wall */
  uint64_t nodes_processed; /* search nodes the engines ran; > nodes when work after the first
                               witness in preorder was done before the witness was known */
} qi_solve_result;

/* q1, q2: caller buffers of n_vertices entries (may be NULL).  q1 = disjoint quorum
 * found by the visitor, in sccs.front() order; q2 = the minimal quorum, in branch order
 * (cpp:372-373).  Global vertex indices. */
int qi_solve(qi_fbas* f, const qi_solve_opts* opts, qi_solve_result* res, uint32_t* q1, uint32_t* q2);

/* Text-mode driver = the reference's solve(istream&, ostream&, verbose, graphviz)
 * (cpp:709-716) + verdict line (cpp:790-797).  Returns malloc'd text (free with
 * qi_free); *verdict = 1/0.  verbose/graphviz as -v/-g. */
int qi_solve_text(qi_fbas* f, int verbose, int graphviz, char** text, int* verdict);
/* The same with search options (engines, device_mask, budgets); opts may be NULL. */
int qi_solve_text_ex(qi_fbas* f, int verbose, int graphviz, const qi_solve_opts* opts, char** text, int* verdict);
/* computePageRank (cpp:718-733) text ("PageRank:" + "label: value" lines), host float. */
int qi_pagerank_text(qi_fbas* f, float dangling, float convergence, uint64_t max_iterations, char** text);
void qi_free(void* p);

/* ---------------------------------------------------------------------------------
 * Step-wise search for multi-process drivers (one process per GPU, RCCL over xGMI in
 * the caller).  A unit is a subtree root of iterateMinimalQuorums (cpp:252) packed in
 * qi_search_unit_bytes() bytes; units can be moved between ranks through caller-owned
 * device memory.  Counts stay preorder-exact because every processed segment is logged
 * with its root path key and reduced against the globally preorder-first witness.
 * ------------------------------------------------------------------------------- */
typedef struct {
  uint32_t grow_budget, run_budget, max_blocks; /* 0 = defaults */
  uint32_t jit;                                  /* as qi_solve_opts.jit */
  uint32_t batch;                                /* launches per qi_search_step (0 = default) */
} qi_search_opts;

typedef struct {
  uint64_t frontier_in, frontier_out, processed;
  uint32_t budget, blocks;
  uint64_t new_witnesses;
  double kernel_ms;
  uint32_t specialized;  /* 1 if this step ran the run-time specialised kernel */
  uint32_t launches;     /* chained launches of this step that had input */
  uint32_t dispatches;   /* launches enqueued, incl. the <= 2 empty look-ahead ones */
  uint32_t pad;
  double dispatch_ms;    /* HIP-event time of all enqueued launches (what rocprof averages) */
} qi_step_info;

typedef struct {
  uint64_t nodes, evals, minq, zero_fallback, rounds;
  uint64_t units;        /* frontier units fetched (all launches) */
  uint64_t wave_iters;   /* search-loop iterations summed over wavefronts */
  uint64_t coop_phases;  /* iterations that ran the cooperative minimality phase */
  uint64_t stamps[8];    /* jit = 3 diagnostic build: s_memtime cycles per loop section */
} qi_totals;

/* Shape of the flattened searched SCC (for work accounting). */
typedef struct {
  uint32_t m;          /* |sccs.front()| */
  uint32_t mask_words; /* 32-bit words per vertex mask */
  uint32_t tns;        /* live threshold nodes */
  uint32_t tn_words;   /* 32-bit words per TN-satisfaction mask */
  uint32_t tns_with_children;
  uint32_t roots;      /* distinct root TNs */
  uint32_t groups;     /* findBestNode column groups */
  uint32_t extra_terms;
  uint32_t qmin_inside;  /* lower bound on a non-empty containsQuorum result, outside
                            vertices unavailable (0 = no bound: threshold-0 sets) */
  uint32_t qmin_outside; /* the same with outside vertices available (visitor, cpp:368) */
} qi_shape;

/* Compile (or load from the on-disk cache) the run-time specialised search kernel for
 * sccs.front() with hipRTC; needs no GPU.  *ms = compile wall time. */
int qi_fbas_jit_precompile(qi_fbas* f, double* ms);

/* Requires exactly one SCC with a quorum (else QI_ERR_STATE: no search is defined). */
int qi_search_create(qi_fbas* f, const qi_search_opts* opts, qi_search** out);
void qi_search_destroy(qi_search* s);
uint32_t qi_search_unit_bytes(const qi_search* s);
uint32_t qi_search_key_words(const qi_search* s);  /* 32-bit words of a path key */
int qi_search_reset(qi_search* s);                  /* frontier = {root} (cpp:393) */
int qi_search_clear(qi_search* s);                  /* frontier = {} */
/* One batch of chained launches (qi_search_opts.batch), one host synchronisation. */
int qi_search_step(qi_search* s, qi_step_info* info);
/* As qi_search_step, but stops enqueueing once a finished launch left >= target units
 * (rank 0 grows the frontier it hands out to the other ranks). */
int qi_search_grow(qi_search* s, uint64_t target, qi_step_info* info);
uint64_t qi_search_frontier(const qi_search* s);
int qi_search_keep_slice(qi_search* s, uint64_t begin, uint64_t end);
/* Keep a rank's share of a broadcast frontier: in round q (units q*stride .. q*stride +
 * stride - 1) the unit at offset (offset - q) mod stride; the shares of offsets 0..stride-1
 * partition the frontier. */
int qi_search_keep_strided(qi_search* s, uint64_t offset, uint64_t stride);
int qi_search_export(qi_search* s, uint64_t count, void* device_dst); /* pop `count` from the tail */
int qi_search_import(qi_search* s, uint64_t count, const void* device_src);
/* Best witness found locally: key[key_words], depth; returns 1 if any. */
int qi_search_local_best(qi_search* s, uint32_t* key, uint32_t* depth);
int qi_search_set_best(qi_search* s, const uint32_t* key, uint32_t depth);
/* Early termination across cooperating searches inside a chain of launches (the reference
 * stops the whole search at the first disjoint pair, cpp:369-377).  host_word: 8 bytes of
 * host memory, 8-byte aligned, shared by every qi_search working on the same search (in one
 * process, or mapped into several, e.g. a POSIX shared-memory page on one node); all ones =
 * no witness.  After every launch a search folds its best key into the word (atomic
 * minimum) and its kernels poll it, so a witness found on one GPU prunes the others within
 * a few launches; qi_search_local_best / qi_search_set_best / qi_search_reduce still decide
 * the exact result.  The library pins the page if it is not HIP host memory.  The caller
 * writes all ones before a new search; NULL ends the sharing. */
int qi_search_share_best(qi_search* s, void* host_word);
/* Sums over processed segments at or before (key, depth) in preorder; key NULL = all. */
int qi_search_reduce(qi_search* s, const uint32_t* key, uint32_t depth, qi_totals* out);
/* Witness of the local best: q1 (scc order) / q2 (branch order), global indices. */
int qi_search_witness(qi_search* s, uint32_t* q1, uint32_t* q1_len, uint32_t* q2, uint32_t* q2_len);
/* Forget processed segments / best (start a fresh search on the same FBAS). */
int qi_search_restart(qi_search* s);
double qi_search_kernel_ms(const qi_search* s);
/* Block until a background compile of the specialised kernel (if any) has finished;
 * returns 1 if the next launch will use the specialised kernel. */
int qi_search_wait_jit(qi_search* s);
int qi_search_shape(const qi_search* s, qi_shape* out);

/* The search's reproduction of libstdc++ std::unordered_set<size_t> iteration order
 * (toRemove at cpp:308/331 is that order; it decides the Gauss-Seidel sweeps on
 * threshold-0 SCCs).  keys[v] = global vertex index of local vertex v (n_keys <= 256);
 * the set is built by inserting keys[seq[0]], keys[seq[1]], ... (repeats ignored);
 * out[0..*n_out) = local vertices in iteration order.  Host only, no GPU needed. */
int qi_hash_iteration_order(const uint32_t* keys, uint32_t n_keys, const uint32_t* seq, uint32_t n_seq,
                            uint32_t* out, uint32_t* n_out);

#ifdef __cplusplus
}
#endif

#endif /* QUORUM_INTERSECTION_H_ */
