// Host driver of checkMinimalQuorums(sccs.front()) (quorum_intersection.cpp:348-400, 691):
// one search engine, or the search tree sharded by branch prefix over several engines
// (one host thread + HIP stream each) on one or more GPUs.
#pragma once

#include <cstdint>
#include <vector>

#include "qi_device.h"
#include "qi_internal.h"

namespace qi {

struct SearchOutcome {
  bool found = false;
  bool nonmonotone = false;
  Totals totals;
  std::vector<uint32_t> q1, q2;  // global indices (q1 ascending, q2 in branch order)
  uint64_t launches = 0;
  uint64_t jit_launches = 0;
  double kernel_ms = 0;
  uint32_t engines = 1, devices = 1;
  uint64_t units_moved = 0;      // rebalancing hand-offs between engines
  uint64_t exchanges = 0;        // rounds of best-key / frontier-size exchange
  uint64_t processed_nodes = 0;  // search nodes the engines ran, including those after the first
                                 // witness in preorder (totals.nodes counts only the ones before)
  double t_device_init_ms = 0;   // peer access + engine device contexts (sharded runs)
};

struct ShardConfig {
  std::vector<int> engine_devices;  // engine e runs on engine_devices[e]
  uint64_t seed_units = 0;          // units engine 0 grows before the deal (0 = 2048 per engine)
  uint64_t lanes = 1u << 17;        // rebalance when an engine holds fewer units than this
  uint64_t min_move = 64;
};

// One engine on `device`.
SearchOutcome search_front_scc(const Graph& g, const std::vector<uint32_t>& scc, int device, const SearchConfig& cfg);

// Sharded search: engine 0 grows the frontier from the root (cpp:393), every engine keeps
// its dealt share (rounds of E units, offset rotating by one per round), engines run
// chains of launches in parallel, and between chains the host exchanges best keys
// (pruning) and rebalances surplus units (device-to-device / xGMI copies).  Counts are
// preorder-exact for any schedule: every engine reduces its segment log against the
// globally preorder-first witness.
SearchOutcome search_front_scc_sharded(const Graph& g, const std::vector<uint32_t>& scc, const ShardConfig& sc,
                                       const SearchConfig& cfg);

// Pure planning helpers (unit-tested through the Python mirror in distributed.py).
struct Move {
  uint32_t src, dst;
  uint64_t count;
};
std::vector<Move> plan_rebalance(const std::vector<uint64_t>& sizes, uint64_t min_move);
bool needs_rebalance(const std::vector<uint64_t>& sizes, uint64_t lanes);

}  // namespace qi
