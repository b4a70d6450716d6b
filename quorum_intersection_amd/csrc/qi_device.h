// Internal interface between the host driver and the HIP device code (qi_device.hip).
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "qi_internal.h"

namespace qi {

// ----------------------------------------------------------------------------------
// Batched greatest-fixpoint evaluation (containsQuorum, cpp:140-177) over the global
// threshold-node CSR: one wavefront per query, membership by wave64 __ballot.
// ----------------------------------------------------------------------------------
class GfpDevice {
 public:
  virtual ~GfpDevice() = default;
  // nodes/avail/out: count x words(n) uint64 masks in host memory.
  virtual void run(const uint64_t* nodes, const uint64_t* avail, uint32_t count, uint64_t* out) = 0;
  // The same fixpoints for callers that cannot allocate: masks in DEVICE memory, per-query
  // state in the library's fixed device scratch array (QI_STATIC_SCRATCH_BYTES per GPU, shared
  // by every call on that GPU), no hipMalloc / hipFree / hipHostMalloc.  stream = a
  // hipStream_t to enqueue on (no synchronisation), or null: HIP's default stream, waited
  // for before returning.  Throws QI_ERR_CAPACITY when count queries do not fit the array.
  virtual void run_static(const uint64_t* d_nodes, const uint64_t* d_avail, uint32_t count, uint64_t* d_out,
                          void* stream) = 0;
  virtual double last_kernel_ms() const = 0;
};
std::unique_ptr<GfpDevice> make_gfp_device(int device, const GlobalFlat& g);

// ----------------------------------------------------------------------------------
// Branch-and-bound search (iterateMinimalQuorums + checkMinimalQuorums, cpp:252-400)
// as a budgeted frontier loop.  A "unit" is a subtree root (T, D, path key, D order);
// one launch runs a per-lane depth-first walk of units for at most `budget` search
// nodes per lane, spilling the rest of its stack back into the next frontier.  Launches
// are chained on the device; step() enqueues a batch of them and synchronises once.
// ----------------------------------------------------------------------------------
struct SearchConfig {
  uint32_t max_blocks = 0;       // 0 = CUs * 8
  uint32_t grow_budget = 3;      // per-lane node budget while the frontier is small (2 / 3 / 4 / 6: 2.25 /
                                 // 2.19 / 3.28 / 3.46 ms on the bench workload, 0.47 / 0.41 / 0.43 / 0.45 ms
                                 // on two_tier(8, 192))
  uint32_t run_budget = 4096;    // per-lane node budget once the frontier fills the GPU
  uint32_t grace = 16;           // per-lane steps after the unit queue runs dry (8/12/16/20/24: 2.27/2.26/2.22/2.32/2.39 ms)
  uint32_t evict_max = 32;       // per-lane stack evictions per launch (bounds the output; 8 stalls deep
                                 // multi-word searches, 8/32/64 equal on the bench)
  uint32_t run_at = 4;           // run budget once the frontier holds >= run_at/8 of the resident lanes
  uint32_t batch = 0;            // max chained launches per step() (0 = 64)
  uint32_t lookahead = 2;        // launches kept in flight beyond the one the host waits for
  bool keep_log = true;          // keep per-segment records for preorder-exact counts
  // Run-time specialised kernel (qi_jit.cpp): 0 = auto (compile in the background once a
  // search reaches `jit_after` launches, switch at the next launch boundary), 1 = off
  // (table-interpreting kernel only), 2 = sync (compile before the first launch),
  // 3 = sync diagnostic build with s_memtime section stamps (never for measurements),
  // 4 = cache only (the specialised kernel if the on-disk cache holds it, else the table
  // kernel; never compiles).  0 and 4 load a cached kernel before the first launch.
  uint32_t jit = 0;
  uint32_t jit_after = 3;
  // findBestNode ties (cpp:229-246): 0 = lowest vertex index (reproducible counts), 1 = a
  // seeded uniform draw over the maximal in-degree vertices, the reference's own rule
  uint32_t tiebreak = 0;
  uint32_t tie_seed = 0;
};

struct StepInfo {
  uint64_t frontier_in = 0, frontier_out = 0;
  uint64_t processed = 0;        // input units of the launches of this step
  uint32_t launches = 0;         // launches that had input (the rest of the batch was empty)
  uint32_t dispatches = 0;       // launches enqueued (incl. the <= lookahead empty ones)
  double dispatch_ms = 0;        // HIP-event time of all enqueued launches
  uint32_t budget = 0, blocks = 0;
  uint64_t new_witnesses = 0;
  double kernel_ms = 0;          // HIP-event time of the search kernel
  bool has_best = false;
  bool specialized = false;      // launched the run-time specialised kernel
};

struct Totals {
  uint64_t nodes = 0, evals = 0, minq = 0, zero_fallback = 0, rounds = 0;
  uint64_t units = 0, wave_iters = 0, coop_phases = 0;  // occupancy accounting (unfiltered)
  uint64_t dbg[8] = {0, 0, 0, 0, 0, 0, 0, 0};           // diagnostic stamps (jit = 3)
};

struct Witness {
  std::vector<uint32_t> key;     // path bits, MSB-first words
  uint32_t depth = 0;
  std::vector<uint32_t> q1_local;  // ascending local indices (visitor GFP survivors)
  std::vector<uint32_t> q2_local;  // D in branch order
};

class SearchDevice {
 public:
  virtual ~SearchDevice() = default;
  virtual int device() const = 0;                   // HIP ordinal the engine runs on
  virtual uint32_t key_words() const = 0;
  virtual uint32_t unit_bytes() const = 0;
  virtual void reset_root() = 0;                    // frontier = {root of cpp:393}
  virtual void clear_frontier() = 0;
  // One chain of launches; with until > 0 the host stops enqueueing once a finished
  // launch left at least `until` units (frontier growth for multi-rank hand-out).
  virtual StepInfo step(uint64_t until = 0) = 0;
  virtual uint64_t frontier_size() const = 0;
  // Frontier hand-off for multi-rank rebalancing: units are moved through caller-owned
  // device memory (e.g. torch tensors sent with RCCL).
  virtual void export_tail(uint64_t count, void* dev_dst) = 0;
  virtual void import_units(uint64_t count, const void* dev_src) = 0;
  virtual void keep_slice(uint64_t begin, uint64_t end) = 0;
  virtual void keep_strided(uint64_t offset, uint64_t stride) = 0;  // units offset, offset+stride, ...
  // Global best (preorder-first witness key) known to the caller, for pruning.
  virtual void set_best(const std::vector<uint32_t>& key, uint32_t depth) = 0;
  virtual bool best(Witness* w) const = 0;          // best witness found on this device
  // Early termination across cooperating engines inside a chain (cpp:369-377 stops the
  // whole search at the first disjoint pair): `host_word` is 8 bytes of host memory shared
  // by the engines of one search (one process, or mapped into several); all ones = no
  // witness.  After every launch the engine folds its best key into it (atomic minimum),
  // and its kernels poll it like their own device-side key, so a witness found on one GPU
  // prunes the others within a few launches instead of at the next host exchange.  The
  // engine pins the word (hipHostRegister) if it is not HIP host memory already; null ends
  // the sharing.  The caller resets the word between searches.
  virtual void share_best(uint64_t* host_word) = 0;
  // Sums over every processed segment whose root precedes-or-equals `key` in preorder
  // (all segments when has_key == false).
  virtual Totals reduce(bool has_key, const std::vector<uint32_t>& key, uint32_t depth) = 0;
  virtual Totals running_totals() const = 0;        // unfiltered running sums
  virtual void drop_log() = 0;                      // forget processed segments
  virtual double sum_kernel_ms() const = 0;
  virtual uint64_t launches() const = 0;
  virtual uint64_t dispatches() const = 0;
  virtual double dispatch_ms() const = 0;
  virtual uint64_t specialized_launches() const = 0;
  virtual bool wait_jit() = 0;                      // finish a pending compile; true if loaded
};
std::unique_ptr<SearchDevice> make_search_device(int device, const LocalFlat& f, const SearchConfig& cfg);

// The ordered kernel's libstdc++ unordered_set order emulation, on the host (tests).
uint32_t hash_iteration_order(const uint32_t* keys, uint32_t n_keys, const uint32_t* seq, uint32_t n_seq,
                              uint32_t* out);

// hipRTC-compile the specialised kernel for this SCC's template shape (no GPU needed).
bool jit_precompile(const LocalFlat& f, std::string* log);

int device_count();
int device_cu_count(int device);
// Device initialisation beyond the context: creates the first pooled stream (the first
// hardware queue of a process costs ~9 ms) and loads the library's base code object (the
// batched fixpoint kernels and the static scratch array).  Optional; the first device call
// pays for it otherwise.
void device_prepare(int device);

// Device memory for frontier hand-offs between engines (qi_shard.cpp): units move
// device-to-device, across GPUs over xGMI with hipMemcpyPeerAsync.
void* device_alloc(int device, size_t bytes);
void device_free(int device, void* p);
void device_copy(void* dst, int dst_device, const void* src, int src_device, size_t bytes);
// One 64-bit word of pinned host memory that every device can map (the engines' shared
// best key, SearchDevice::share_best), initialised to all ones.
uint64_t* pinned_word_alloc();
void pinned_word_free(uint64_t* p);
// Enable peer access from a to b (and b to a); false when the pair has no peer path
// (copies then stage through the host inside the HIP runtime).
bool enable_peer(int a, int b);

}  // namespace qi
