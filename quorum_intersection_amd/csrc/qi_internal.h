// Internal host-side data model of the MI355X quorum-intersection checker.
//
// Mirrors the reference's data model (quorum_intersection.cpp:55-87) without Boost:
// a vertex per stellarbeat JSON entry, a recursive threshold tree per vertex, and
// out-edge lists in insertion order (boost adjacency_list<vecS, vecS, directedS>).
#pragma once

#include <cstdint>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

namespace qi {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ----------------------------------------------------------------------------------
// Phase times of the drop-in's time-to-verdict (QI_TIMING): parse, graph + SCCs, flatten,
// device set-up, per-SCC checks, search, text.  Process-wide, filled by every stage when
// enabled, read once by the CLI (qi_timing_json).
// ----------------------------------------------------------------------------------
namespace timing {
bool enabled();                          // QI_TIMING is set
void add(const char* phase, double ms);  // accumulates per phase name, in first-use order
void count(const char* name, double n);  // a plain number beside the phases (no "_ms" suffix)
std::string json();                      // {"phase_ms": value, ...}
struct Scope {                           // adds its lifetime to `phase` (no-op when disabled)
  const char* phase;
  bool on;
  long long t0;
  explicit Scope(const char* p);
  ~Scope();
};
}  // namespace timing

// ----------------------------------------------------------------------------------
// Ingestion (cpp:402-436): boost::property_tree keeps every scalar as text.
// ----------------------------------------------------------------------------------
struct QuorumSetIds {               // GenericQuorumSet<NodeID>
  uint64_t threshold = 0;
  bool has_threshold = false;       // false for null / {} quorum sets
  std::vector<std::string> validators;
  std::vector<QuorumSetIds> inner;
};
struct StellarNode {
  std::string publicKey, name;
  QuorumSetIds qset;
};
// Throws Error(QI_ERR_PARSE) where the reference throws a ptree_error (and aborts).
std::vector<StellarNode> parse_stellar_json(const char* text, size_t len);

// ----------------------------------------------------------------------------------
// Trust graph (cpp:438-473)
// ----------------------------------------------------------------------------------
struct QuorumSet {                  // GenericQuorumSet<GraphQData>
  uint64_t threshold = 0;
  bool has_threshold = false;
  std::vector<uint32_t> validators; // vertex indices, unknown ids -> 0 (cpp:456)
  std::vector<QuorumSet> inner;
};
struct Graph {
  std::vector<std::string> ids, names;
  std::vector<QuorumSet> qsets;
  std::vector<std::vector<uint32_t>> adj;  // out-edges, insertion order, parallel edges kept
  uint32_t n() const { return (uint32_t)ids.size(); }
};
Graph build_graph(const std::vector<StellarNode>& nodes);

// boost::strong_components numbering (cpp:621): DFS roots 0..n-1, out-edges in order,
// component id = SCC completion order.  sccs[c] lists vertices ascending (cpp:628-633).
struct Sccs {
  std::vector<uint32_t> comp;
  std::vector<std::vector<uint32_t>> members;
};
Sccs strong_components(const Graph& g);

// ----------------------------------------------------------------------------------
// Flattened threshold-node CSR (device input).  Threshold nodes (TN) are the nodes of
// all quorum-set trees, deduplicated structurally and listed children-first.
//
// Semantics of one TN under availability A (cpp:90-138, "node itself available" is a
// per-vertex test done by the caller):
//   entries == 0 or threshold > entries      -> false
//   threshold == 0                           -> true iff the FIRST entry is unavailable
//                                               (size_t wrap of the early-exit counters)
//   otherwise                                -> (#available validator refs, with
//                                               multiplicity) + (#satisfied inner sets)
//                                               >= threshold
// ----------------------------------------------------------------------------------
enum : uint32_t { TN_NORMAL = 0, TN_NEVER = 1, TN_FIRST_UNAVAIL = 2 };

// Global form: every vertex, masks over all n vertices (used by the batched GFP kernel
// for containsQuorum(nodes, avail) queries, e.g. the per-SCC checks at cpp:649-672).
struct GlobalFlat {
  uint32_t n = 0, words = 0;        // vertices, 64-bit words per vertex mask
  uint32_t T = 0;                   // threshold nodes
  uint32_t levels = 0;              // evaluation levels (leaves = 0)
  bool nonmonotone = false;         // some TN has threshold 0 (anti-monotone slice)
  std::vector<uint32_t> level_off;  // [levels+1] TN ranges per level (TNs sorted by level)
  std::vector<uint32_t> kind;       // [T]
  std::vector<uint32_t> thr;        // [T] threshold (NORMAL)
  std::vector<uint32_t> first;      // [T] FIRST_UNAVAIL: bit31 = child flag, low bits = index
  std::vector<uint32_t> vref_off;   // [T+1] CSR of validator refs (with repetition)
  std::vector<uint32_t> vref;
  std::vector<uint32_t> cref_off;   // [T+1] CSR of child TN refs (with repetition)
  std::vector<uint32_t> cref;
  std::vector<uint32_t> root;       // [n] root TN of each vertex
};
GlobalFlat flatten_global(const Graph& g);

// SCC-local form for the search kernel (cpp:252-400): vertices of the searched SCC are
// renumbered 0..m-1 in ascending global order (so "lowest local index" = "lowest vertex
// index"); references to vertices outside the SCC fold into a per-TN count that is added
// when the call site treats outside vertices as available (only the visitor, cpp:354/368).
// Masks are arrays of 32-bit words so a wave64 lane evaluates a TN with v_and_b32 +
// v_bcnt_u32_b32 pairs.
struct LocalFlat {
  uint32_t m = 0;                   // |SCC|
  uint32_t mw = 0;                  // 32-bit words per vertex mask (m <= 32*mw)
  uint32_t T = 0;                   // threshold nodes
  uint32_t tw = 0;                  // 32-bit words per TN-satisfaction mask
  bool nonmonotone = false;         // a live TN has threshold 0: Jacobi != Gauss-Seidel
  std::vector<uint32_t> scc;        // local -> global vertex
  std::vector<int32_t> thr;         // [T][2] effective threshold (outside unavailable / available)
  std::vector<uint32_t> flags;      // [T] bit0 inverted test (count==0), bit1 extra terms
  std::vector<uint32_t> vmask;      // [T][mw] validator refs, multiplicity plane 0
  std::vector<uint32_t> cmask;      // [T][tw] child TN refs, multiplicity plane 0
  std::vector<uint32_t> extra_off;  // [T+1] extra planes: (src word, mask) terms
  std::vector<uint32_t> extra_src;  //   src < mw: vertex word, else TN-sat word src-mw
  std::vector<uint32_t> extra_mask;
  uint32_t R = 0;                   // distinct root TNs
  std::vector<uint32_t> root_tn;    // [R]
  std::vector<uint32_t> root_users; // [R][mw] vertices whose qset root is root_tn[r]
  uint32_t G = 0;                   // findBestNode column groups (identical in-edge columns)
  std::vector<uint32_t> grp_members;// [G][mw]
  std::vector<uint32_t> grp_col;    // [G][mw] in-edge sources, multiplicity plane 0
  std::vector<uint32_t> grp_extra_off;  // [G+1] extra multiplicity planes (mw words each)
  std::vector<uint32_t> grp_extra;
  // Smallest possible non-empty greatest fixpoint, per polarity (outside unavailable /
  // available): every survivor y needs the internal vertices of one of its slices, so
  // containsQuorum(X) is empty whenever |X| < qmin.  0 disables the test (threshold-0
  // sets make the slice predicate non-monotone).
  uint32_t qmin[2] = {0, 0};
  // Order-exact search (threshold-0 SCCs, qi_ordered_kernel.h): the root TN of each
  // vertex (NO_ROOT: never satisfied) and the out-edges inside the SCC in insertion
  // order with repetitions (findBestNode's in-degrees, cpp:222-247).
  static constexpr uint32_t NO_ROOT = 0xFFFFFFFFu;
  std::vector<uint32_t> vroot;      // [m]
  std::vector<uint32_t> ladj_off;   // [m+1]
  std::vector<uint32_t> ladj;
};
LocalFlat flatten_local(const Graph& g, const std::vector<uint32_t>& scc);

// ----------------------------------------------------------------------------------
// Text output used by the CLI (cpp:475-530, 532-613)
// ----------------------------------------------------------------------------------
void print_quorum(const std::vector<uint32_t>& quorum, const Graph& g, std::ostream& out);
void print_graphviz(const Graph& g, std::ostream& out, const Sccs& s);
std::vector<float> page_rank(const Graph& g, float m, float convergence, uint64_t max_iterations);
void print_page_rank(const Graph& g, std::ostream& out, const std::vector<float>& pr);

}  // namespace qi
