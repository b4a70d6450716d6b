// =====================================================================================
//  oracle/qi_oracle.cpp  --  TEST INFRASTRUCTURE ONLY (the checker, never the product)
// =====================================================================================
//  CPU restatement of /root/reference/quorum_intersection.cpp (fixxxedpoint/
//  quorum_intersection), written from the reference's behaviour, not copied from it.
//  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
//
//  The reference cannot be compiled here (Boost graph/log/program_options/property_tree
//  >= 1.58 are absent, CMakeLists.txt:8), so this file restates, function by function:
//    containsQuorumSlice   cpp:90-138     R1  recursive threshold test, size_t wrap quirks
//    containsQuorum        cpp:140-177    R2  Gauss-Seidel greatest fixpoint, mask restore
//    isMinimalQuorum       cpp:179-201    R3
//    findBestNode          cpp:203-250    R5  (tie-break: "random" = reference reservoir
//                                              sampling, "lowest" = lowest vertex index of
//                                              the argmax set, one of the reference's
//                                              possible outcomes, cpp:229-246)
//    iterateMinimalQuorums cpp:252-346    R6  exclusion branch first, |D|>|scc|/2 prune
//    checkMinimalQuorums   cpp:348-400    R4/R7 visitor with outside-SCC vertices available
//    parseQuorumSet/JSON   cpp:402-436    boost::property_tree JSON semantics (values as text)
//    buildDependencyGraph  cpp:438-473    unknown id -> vertex 0, duplicate keys append
//    printQuorum           cpp:475-490    -v text
//    NodeWriter/graphviz   cpp:492-530    -g text (boost::write_graphviz layout)
//    pageRank/print        cpp:532-613    -p
//    solve(Graph)          cpp:615-707    Tarjan numbering as boost::strong_components
//    main                  cpp:744-800    CLI (built as oracle/_build/qi_oracle)
//
//  Parity pinning: the four reference fixtures' verdicts (correct*.json -> true,
//  broken*.json -> false; README.md:25-28) are the only reference-held known answers.
//  Node/eval counts and witnesses are pinned under the deterministic "lowest" tie-break
//  and committed as golden vectors by tests/golden/make_golden.py.
//
//  Deliberate additions (instrumentation only, no behavioural change): a context that
//  counts search calls (the reference's static counter, cpp:258), fixpoint evaluations
//  (containsQuorum calls), minimal quorums visited (cpp:361), and an optional node budget
//  used by bench.py to time a bounded CPU sample.
// =====================================================================================
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iomanip>
#include <iostream>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace qio {

// ------------------------------------------------------------------------------------
// property_tree-like value tree: every scalar is kept as text, arrays are children with
// empty keys, objects keep duplicate keys in order (boost standard_callbacks behaviour).
// ------------------------------------------------------------------------------------
struct PTree {
  std::string data;
  std::vector<std::pair<std::string, PTree>> children;
  bool empty() const { return children.empty(); }
  const PTree* child(const std::string& key) const {
    for (const auto& c : children)
      if (c.first == key) return &c.second;
    return nullptr;
  }
};

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class JsonReader {
 public:
  JsonReader(const char* s, size_t n) : p_(s), e_(s + n) {}
  PTree parse() {
    PTree root;
    ws();
    value(root);
    ws();
    if (p_ != e_) throw ParseError("garbage after data");
    return root;
  }

 private:
  const char* p_;
  const char* e_;
  void ws() {
    while (p_ != e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  bool lit(const char* w) {
    size_t n = std::strlen(w);
    if ((size_t)(e_ - p_) >= n && std::memcmp(p_, w, n) == 0) {
      p_ += n;
      return true;
    }
    return false;
  }
  void value(PTree& t) {
    if (p_ == e_) throw ParseError("expected value");
    char c = *p_;
    if (c == '{') return object(t);
    if (c == '[') return array(t);
    if (c == '"') {
      t.data = str();
      return;
    }
    if (lit("true")) { t.data = "true"; return; }
    if (lit("false")) { t.data = "false"; return; }
    if (lit("null")) { t.data = "null"; return; }
    number(t);
  }
  void number(PTree& t) {
    const char* s = p_;
    if (p_ != e_ && *p_ == '-') ++p_;
    if (p_ == e_) throw ParseError("expected number");
    if (*p_ == '0') {
      ++p_;
    } else if (*p_ >= '1' && *p_ <= '9') {
      while (p_ != e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    } else {
      throw ParseError("expected value");
    }
    if (p_ != e_ && *p_ == '.') {
      ++p_;
      if (p_ == e_ || !(*p_ >= '0' && *p_ <= '9')) throw ParseError("need digits after '.'");
      while (p_ != e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    }
    if (p_ != e_ && (*p_ == 'e' || *p_ == 'E')) {
      ++p_;
      if (p_ != e_ && (*p_ == '+' || *p_ == '-')) ++p_;
      if (p_ == e_ || !(*p_ >= '0' && *p_ <= '9')) throw ParseError("need digits in exponent");
      while (p_ != e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    }
    t.data.assign(s, p_);
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) throw ParseError("invalid escape sequence");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else throw ParseError("invalid escape sequence");
    }
    return v;
  }
  std::string str() {
    ++p_;  // opening quote
    std::string out;
    for (;;) {
      if (p_ == e_) throw ParseError("unterminated string");
      unsigned char c = (unsigned char)*p_++;
      if (c == '"') break;
      if (c < 0x20) throw ParseError("invalid code sequence");
      if (c != '\\') {
        out += (char)c;
        continue;
      }
      if (p_ == e_) throw ParseError("invalid escape sequence");
      char x = *p_++;
      switch (x) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (!(e_ - p_ >= 2 && p_[0] == '\\' && p_[1] == 'u')) throw ParseError("invalid codepoint");
            p_ += 2;
            uint32_t lo = hex4();
            if (lo < 0xDC00 || lo > 0xDFFF) throw ParseError("invalid codepoint");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            throw ParseError("invalid codepoint");
          }
          utf8(out, cp);
          break;
        }
        default: throw ParseError("invalid escape sequence");
      }
    }
    return out;
  }
  void object(PTree& t) {
    ++p_;
    ws();
    if (p_ != e_ && *p_ == '}') { ++p_; return; }
    for (;;) {
      ws();
      if (p_ == e_ || *p_ != '"') throw ParseError("expected key string");
      std::string key = str();
      ws();
      if (p_ == e_ || *p_ != ':') throw ParseError("expected ':'");
      ++p_;
      ws();
      t.children.emplace_back(key, PTree());
      value(t.children.back().second);
      ws();
      if (p_ != e_ && *p_ == ',') { ++p_; continue; }
      if (p_ != e_ && *p_ == '}') { ++p_; return; }
      throw ParseError("expected ',' or '}'");
    }
  }
  void array(PTree& t) {
    ++p_;
    ws();
    if (p_ != e_ && *p_ == ']') { ++p_; return; }
    for (;;) {
      ws();
      t.children.emplace_back(std::string(), PTree());
      value(t.children.back().second);
      ws();
      if (p_ != e_ && *p_ == ',') { ++p_; continue; }
      if (p_ != e_ && *p_ == ']') { ++p_; return; }
      throw ParseError("expected ',' or ']'");
    }
  }
};

// property_tree::get<size_t>: stream extraction of the text, whole string must be used
// (stream_translator), else ptree_bad_data.  libstdc++ num_get accepts '-' for unsigned
// and wraps ("-1" -> SIZE_MAX, no failbit).
static size_t get_size_t(const PTree& t, const char* key) {
  const PTree* c = t.child(key);
  if (!c) throw ParseError(std::string("No such node (") + key + ")");
  std::istringstream iss(c->data);
  unsigned long v = 0;
  iss >> v;
  if (!iss.eof()) iss >> std::ws;
  if (iss.fail() || iss.bad() || iss.get() != std::char_traits<char>::eof())
    throw ParseError(std::string("conversion of data to type \"m\" failed (") + key + ")");
  return (size_t)v;
}

// ------------------------------------------------------------------------------------
// Data model (cpp:55-87)
// ------------------------------------------------------------------------------------
using NodeIx = size_t;
struct QSetS {  // GenericQuorumSet<NodeID>
  size_t threshold = 0;
  bool threshold_set = false;  // false for null/{} quorum sets (indeterminate in reference)
  std::vector<std::string> nodes;
  std::vector<QSetS> innerSets;
};
struct QSet {  // GenericQuorumSet<GraphQData>
  size_t threshold = 0;
  std::vector<NodeIx> nodes;
  std::vector<QSet> innerSets;
};
struct StellarNode {
  std::string nodeID, name;
  QSetS qSet;
};
struct Vertex {
  std::string nodeID, name;
  QSet qSet;
};
struct Graph {
  std::vector<Vertex> v;
  std::vector<std::vector<NodeIx>> adj;  // out-edges in insertion order (vecS)
  size_t size() const { return v.size(); }
};

// parseQuorumSet (cpp:402-418)
static QSetS parseQuorumSet(const PTree& value) {
  QSetS result;
  if (value.empty()) return result;
  result.threshold = get_size_t(value, "threshold");
  result.threshold_set = true;
  const PTree* vs = value.child("validators");
  if (!vs) throw ParseError("No such node (validators)");
  for (const auto& c : vs->children) result.nodes.push_back(c.second.data);
  const PTree* is = value.child("innerQuorumSets");
  if (!is) throw ParseError("No such node (innerQuorumSets)");
  for (const auto& c : is->children) result.innerSets.push_back(parseQuorumSet(c.second));
  return result;
}

// parseStellarConfigurationJSON (cpp:420-436)
static std::vector<StellarNode> parseStellarConfigurationJSON(const char* s, size_t n) {
  PTree root = JsonReader(s, n).parse();
  std::vector<StellarNode> result;
  for (const auto& node : root.children) {
    const PTree* pk = node.second.child("publicKey");
    if (!pk) throw ParseError("No such node (publicKey)");
    const PTree* nm = node.second.child("name");
    const PTree* qs = node.second.child("quorumSet");
    if (!qs) throw ParseError("No such node (quorumSet)");
    result.push_back(StellarNode{pk->data, nm ? nm->data : std::string(), parseQuorumSet(*qs)});
  }
  return result;
}

// buildDependencyGraph (cpp:438-473)
static Graph buildDependencyGraph(const std::vector<StellarNode>& nodes) {
  Graph g;
  std::unordered_map<std::string, NodeIx> idMap;
  for (const auto& node : nodes) {
    g.v.push_back(Vertex{node.nodeID, node.name, QSet{}});
    g.adj.emplace_back();
    idMap[node.nodeID] = g.v.size() - 1;
  }
  std::function<void(NodeIx, QSet&, const QSetS&)> addEdges = [&](NodeIx ix, QSet& q, const QSetS& orig) {
    q.threshold = orig.threshold;
    for (const auto& trust : orig.nodes) {
      NodeIx v = idMap[trust];  // unknown id default-inserts 0 (cpp:456)
      q.nodes.push_back(v);
      g.adj[ix].push_back(v);
    }
    for (const auto& inner : orig.innerSets) {
      q.innerSets.push_back({});
      addEdges(ix, q.innerSets.back(), inner);
    }
  };
  for (const auto& node : nodes) {
    NodeIx ix = idMap[node.nodeID];
    addEdges(ix, g.v[ix].qSet, node.qSet);
  }
  return g;
}

// ------------------------------------------------------------------------------------
// Search context: the reference's static counter (cpp:258), the visitor counter
// (cpp:355) and the RNG (cpp:207) made explicit, plus instrumentation.
// ------------------------------------------------------------------------------------
enum TieBreak { TIE_LOWEST = 0, TIE_RANDOM = 1 };
struct Ctx {
  TieBreak tie = TIE_LOWEST;
  std::default_random_engine rng;
  uint64_t nodes = 0;       // iterateMinimalQuorums calls
  uint64_t evals = 0;       // containsQuorum calls (all call sites)
  uint64_t scc_evals = 0;   // of which at cpp:658
  uint64_t minq = 0;        // visitor calls (minimal quorums of size <= |scc|/2)
  uint64_t zero_fallback = 0;  // findBestNode returned *quorum.begin() (no in-edges)
  uint64_t budget = 0;      // 0 = unlimited
  bool aborted = false;
  uint64_t depth = 0, max_depth = 0;  // recursion depth of iterateMinimalQuorums (root = 0)
};

// containsQuorumSlice (cpp:90-138)
static bool containsQuorumSlice(NodeIx node, const QSet& q, const std::vector<bool>& avail) {
  if (!avail[node]) return false;
  size_t threshold = q.threshold;
  size_t failLimit = (size_t)(q.nodes.size() + q.innerSets.size()) - threshold + 1;
  for (const auto& id : q.nodes) {
    if (avail[id]) threshold--;
    else failLimit--;
    if (threshold == 0) return true;
    if (failLimit == 0) return false;
  }
  for (const auto& inner : q.innerSets) {
    if (containsQuorumSlice(node, inner, avail)) threshold--;
    else failLimit--;
    if (threshold == 0) return true;
    if (failLimit == 0) return false;
  }
  return false;
}

// containsQuorum (cpp:140-177)
static std::vector<NodeIx> containsQuorum(Ctx& ctx, std::vector<NodeIx> nodes, std::vector<bool>& avail,
                                          const Graph& g) {
  ctx.evals++;
  std::vector<NodeIx> removed, filtered;
  size_t count = nodes.size();
  do {
    count = nodes.size();
    filtered.clear();
    std::copy_if(nodes.begin(), nodes.end(), std::back_inserter(filtered), [&](NodeIx node) {
      if (!containsQuorumSlice(node, g.v[node].qSet, avail)) {
        if (avail[node]) {
          avail[node] = false;
          removed.push_back(node);
        }
        return false;
      }
      return true;
    });
    nodes = filtered;
  } while (count != nodes.size());
  for (NodeIx n : removed) avail[n] = true;
  return nodes;
}

// isMinimalQuorum (cpp:179-201)
static bool isMinimalQuorum(Ctx& ctx, std::vector<NodeIx> nodes, std::vector<bool> avail, const Graph& g) {
  if (containsQuorum(ctx, nodes, avail, g).empty()) return false;
  for (NodeIx node : nodes) {
    avail[node] = false;
    if (!containsQuorum(ctx, nodes, avail, g).empty()) return false;
    avail[node] = true;
  }
  return true;
}

// findBestNode (cpp:203-250)
static NodeIx findBestNode(Ctx& ctx, const std::vector<NodeIx>& quorum, const std::vector<NodeIx>& restriction,
                           const Graph& g) {
  std::vector<bool> avail(g.size(), false);
  std::vector<uint64_t> inDegree(g.size(), 0);
  for (NodeIx n : quorum) avail[n] = true;
  for (NodeIx n : restriction) avail[n] = false;
  uint64_t maxValue = 0;
  int maxCount = 1;
  NodeIx bestNode = *quorum.begin();
  for (NodeIx node : quorum) {
    for (NodeIx w : g.adj[node]) {
      if (!avail[w]) continue;
      uint64_t d = ++inDegree[w];
      if (d >= maxValue) {
        if (d == maxValue) {
          if (ctx.tie == TIE_RANDOM) {
            maxCount += 1;
            int r = std::uniform_int_distribution<int>{1, maxCount}(ctx.rng);
            if (r != 1) continue;
          } else {
            if (w > bestNode) continue;  // lowest index among the argmax set
          }
        } else {
          maxCount = 1;
        }
        maxValue = d;
        bestNode = w;
      }
    }
  }
  if (maxValue == 0) ctx.zero_fallback++;
  return bestNode;
}

using Visitor = std::function<bool(const std::vector<NodeIx>&)>;

// iterateMinimalQuorums (cpp:252-346)
static bool iterateMinimalQuorumsBody(Ctx& ctx, std::vector<NodeIx> toRemove, std::vector<NodeIx> dontRemove,
                                      const Graph& g, const Visitor& visitor, const Visitor& currentVisitor);
static bool iterateMinimalQuorums(Ctx& ctx, std::vector<NodeIx> toRemove, std::vector<NodeIx> dontRemove,
                                  const Graph& g, const Visitor& visitor, const Visitor& currentVisitor) {
  ctx.max_depth = std::max(ctx.max_depth, ctx.depth);
  ++ctx.depth;
  const bool r = iterateMinimalQuorumsBody(ctx, std::move(toRemove), std::move(dontRemove), g, visitor, currentVisitor);
  --ctx.depth;
  return r;
}
static bool iterateMinimalQuorumsBody(Ctx& ctx, std::vector<NodeIx> toRemove, std::vector<NodeIx> dontRemove,
                                      const Graph& g, const Visitor& visitor, const Visitor& currentVisitor) {
  if (ctx.budget && ctx.nodes >= ctx.budget) {
    ctx.aborted = true;
    return true;  // unwind (instrumentation only)
  }
  ctx.nodes++;
  if (currentVisitor(dontRemove)) return false;
  if (toRemove.empty() && dontRemove.empty()) return false;
  std::vector<bool> avail(g.size(), false);
  std::vector<NodeIx> nodes;
  for (NodeIx n : dontRemove) {
    avail[n] = true;
    nodes.push_back(n);
  }
  if (!containsQuorum(ctx, nodes, avail, g).empty()) {
    if (isMinimalQuorum(ctx, dontRemove, avail, g)) return visitor(dontRemove);
    return false;
  }
  for (NodeIx n : toRemove) {
    avail[n] = true;
    nodes.push_back(n);
  }
  const auto quorum = containsQuorum(ctx, nodes, avail, g);
  if (quorum.empty()) return false;
  std::unordered_set<NodeIx> quorumNodes(quorum.begin(), quorum.end());
  for (NodeIx n : dontRemove)
    if (quorumNodes.find(n) == quorumNodes.end()) return false;
  const NodeIx bestNode = findBestNode(ctx, quorum, dontRemove, g);
  for (NodeIx n : dontRemove) quorumNodes.erase(n);
  if (quorumNodes.empty()) return false;
  toRemove.clear();
  std::copy_if(quorumNodes.begin(), quorumNodes.end(), std::back_inserter(toRemove),
               [&](NodeIx n) { return n != bestNode; });
  if (iterateMinimalQuorums(ctx, toRemove, dontRemove, g, visitor, currentVisitor)) return true;
  dontRemove.push_back(bestNode);
  return iterateMinimalQuorums(ctx, toRemove, dontRemove, g, visitor, currentVisitor);
}

// checkMinimalQuorums (cpp:348-400)
static bool checkMinimalQuorums(Ctx& ctx, const std::vector<NodeIx>& scc, const Graph& g,
                                std::vector<NodeIx>& q1, std::vector<NodeIx>& q2) {
  bool result = true;
  std::vector<bool> avail(g.size(), true);
  Visitor visitor = [&](const std::vector<NodeIx>& quorum) -> bool {
    ctx.minq++;
    for (NodeIx n : quorum) avail[n] = false;
    const auto disjoint = containsQuorum(ctx, scc, avail, g);
    if (!disjoint.empty()) {
      result = false;
      q1 = disjoint;
      q2 = std::vector<NodeIx>(quorum.begin(), quorum.end());
      return true;
    }
    for (NodeIx n : quorum) avail[n] = true;
    return false;
  };
  Visitor currentVisitor = [&](const std::vector<NodeIx>& c) -> bool { return c.size() > (scc.size() / 2); };
  iterateMinimalQuorums(ctx, scc, std::vector<NodeIx>(), g, visitor, currentVisitor);
  return result;
}

// boost::strong_components numbering: DFS roots 0..n-1, out-edges in insertion order,
// component ids in SCC completion order (cpp:621-622).
static std::vector<size_t> strongComponents(const Graph& g, size_t& count) {
  const size_t n = g.size();
  const size_t UNSET = (size_t)-1;
  std::vector<size_t> comp(n, UNSET), disc(n, UNSET), low(n, 0);
  std::vector<char> onstack(n, 0);
  std::vector<size_t> st;
  size_t t = 0;
  count = 0;
  struct Frame { size_t v, e; };
  std::vector<Frame> cs;
  for (size_t r = 0; r < n; ++r) {
    if (disc[r] != UNSET) continue;
    cs.push_back({r, 0});
    disc[r] = low[r] = t++;
    st.push_back(r);
    onstack[r] = 1;
    while (!cs.empty()) {
      Frame& f = cs.back();
      if (f.e < g.adj[f.v].size()) {
        size_t w = g.adj[f.v][f.e++];
        if (disc[w] == UNSET) {
          disc[w] = low[w] = t++;
          st.push_back(w);
          onstack[w] = 1;
          cs.push_back({w, 0});
        } else if (onstack[w]) {
          low[f.v] = std::min(low[f.v], disc[w]);
        }
        continue;
      }
      size_t v = f.v;
      cs.pop_back();
      if (!cs.empty()) low[cs.back().v] = std::min(low[cs.back().v], low[v]);
      if (low[v] == disc[v]) {
        size_t w;
        do {
          w = st.back();
          st.pop_back();
          onstack[w] = 0;
          comp[w] = count;
        } while (w != v);
        ++count;
      }
    }
  }
  return comp;
}

// printQuorum (cpp:475-490).  Null quorum sets print threshold 0 (the reference prints
// an indeterminate value there: parity unpinned).
static void printQuorum(const std::vector<NodeIx>& quorum, const Graph& g, std::ostream& out) {
  for (NodeIx node : quorum) {
    const auto& value = g.v[node];
    out << value.name << " " << value.nodeID << std::endl
        << "( quorumslice: "
        << "threshold = " << value.qSet.threshold << " ";
    for (NodeIx id : value.qSet.nodes) out << g.v[id].nodeID << " ";
    out << ") " << std::endl << std::endl;
  }
  out << std::endl;
}

// printGraphvizWithSccs + NodeWriter (cpp:492-530), boost::write_graphviz layout.
static void printGraphviz(const Graph& g, std::ostream& out, const std::vector<std::vector<NodeIx>>& sccs) {
  std::vector<unsigned> colors(g.size());
  for (unsigned it = 0; it < sccs.size(); it++)
    for (NodeIx v : sccs[it]) colors[v] = it;
  unsigned offset = sccs.empty() ? 0u : 0xFFFFFFu / (unsigned)sccs.size();
  out << "digraph G {" << std::endl;
  for (size_t v = 0; v < g.size(); ++v) {
    std::stringstream s;
    s << std::setfill('0') << std::setw(6) << std::hex << offset * colors[v];
    const std::string label = g.v[v].name.empty() ? g.v[v].nodeID : g.v[v].name;
    out << v << "[style=filled color=\"#" << s.str() << "\" label=\"" << label << "\" fontcolor=\"white\"]"
        << ";" << std::endl;
  }
  for (size_t v = 0; v < g.size(); ++v)
    for (NodeIx w : g.adj[v]) out << v << "->" << w << " " << ";" << std::endl;
  out << "}" << std::endl;
}

// pageRank (cpp:532-583)
static std::vector<float> pageRank(const Graph& g, float m, float convergence, uint64_t maxIterations) {
  const size_t n = g.size();
  std::vector<float> result(n, 0);
  if (n == 0) return result;
  result[0] = 1;
  float sum = 1;
  std::vector<float> tmp = result;
  float diff = convergence + 1;
  uint64_t iterations = 0;
  for (; diff > convergence && iterations < maxIterations; iterations++) {
    const float mS = m / n;
    sum = n * mS;
    std::fill(tmp.begin(), tmp.end(), mS);
    for (size_t v = 0; v < n; ++v) {
      const float outDegree = float(g.adj[v].size());
      if (0 == outDegree) continue;
      const float Ax_k = (1 - m) / outDegree * result[v];
      for (NodeIx w : g.adj[v]) {
        tmp[w] += Ax_k;
        sum += Ax_k;
      }
    }
    diff = 0;
    for (size_t v = 0; v < n; ++v) {
      diff += std::fabs(tmp[v] - result[v]);
      tmp[v] /= sum;
    }
    result = tmp;
  }
  return result;
}

// printPageRank (cpp:585-613)
static void printPageRank(const Graph& g, std::ostream& out, const std::vector<float>& pr) {
  std::vector<std::pair<std::string, float>> sorted;
  for (size_t v = 0; v < g.size(); ++v) {
    std::string label = g.v[v].name.empty() ? g.v[v].nodeID : g.v[v].name;
    sorted.push_back({label, pr[v]});
  }
  std::sort(sorted.begin(), sorted.end(), [](const std::pair<std::string, float>& a, const std::pair<std::string, float>& b) {
    if (a.second == b.second) return a.first < b.first;
    return a.second > b.second;
  });
  for (const auto& x : sorted) out << x.first << ": " << x.second << std::endl;
}

struct SolveInfo {
  bool verdict = false;
  size_t n = 0, sccCount = 0, withQuorum = 0;
  std::vector<NodeIx> front;
  std::vector<size_t> sccQuorumIds;  // component ids that contain a quorum
  std::vector<NodeIx> q1, q2;
  bool searched = false;
  double search_seconds = 0;
};

// solve(Graph) (cpp:615-707)
static SolveInfo solve(Ctx& ctx, const Graph& g, std::ostream& out, bool verbose, bool graphviz) {
  SolveInfo info;
  info.n = g.size();
  size_t sccCount = 0;
  std::vector<size_t> comp = strongComponents(g, sccCount);
  std::vector<std::vector<NodeIx>> sccs(sccCount);
  for (size_t v = 0; v < g.size(); ++v) sccs[comp[v]].push_back(v);
  info.sccCount = sccCount;
  if (graphviz) printGraphviz(g, out, sccs);
  if (verbose) out << "total number of strongly connected components: " << sccCount << std::endl;
  uint64_t nonIntersectingQs = 0;
  std::vector<bool> avail(g.size(), false);
  std::vector<NodeIx> nodes;
  for (size_t c = 0; c < sccs.size(); ++c) {
    nodes.clear();
    for (NodeIx v : sccs[c]) {
      avail[v] = true;
      nodes.push_back(v);
    }
    ctx.scc_evals++;
    const auto quorum = containsQuorum(ctx, nodes, avail, g);
    if (!quorum.empty()) {
      nonIntersectingQs++;
      info.sccQuorumIds.push_back(c);
      if (verbose) {
        out << "found quorum inside of a strongly connected component:" << std::endl;
        printQuorum(quorum, g, out);
      }
    }
    for (NodeIx v : sccs[c]) avail[v] = false;
  }
  info.withQuorum = nonIntersectingQs;
  if (!sccs.empty()) info.front = sccs.front();
  if (verbose && !sccs.empty()) {  // the reference dereferences front() of an empty vector (UB) here
    out << "number of strongly connected components containing some quorum: " << nonIntersectingQs << std::endl;
    out << "size of the main strongly connected component: " << sccs.front().size() << std::endl;
    out << "main strongly connected component (all minimal quorums are included in it; "
        << "small size means small resilience of the network):" << std::endl;
    printQuorum(sccs.front(), g, out);
  }
  if (nonIntersectingQs != 1) {
    if (verbose)
      out << "network's configuration is broken - more than one strongly connected component contains a quorum - "
          << nonIntersectingQs << std::endl;
    info.verdict = false;
    return info;
  }
  info.searched = true;
  auto t0 = std::chrono::steady_clock::now();
  bool ok = checkMinimalQuorums(ctx, sccs.front(), g, info.q1, info.q2);
  info.search_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (!ok) {
    if (verbose) {
      out << "found two non-intersecting quorums" << std::endl;
      out << "first quorum:" << std::endl;
      printQuorum(info.q1, g, out);
      out << "second quorum:" << std::endl;
      printQuorum(info.q2, g, out);
    }
    info.verdict = false;
    return info;
  }
  if (verbose) out << "all quorums are intersecting" << std::endl;
  info.verdict = true;
  return info;
}

static Graph loadGraph(const char* s, size_t n) { return buildDependencyGraph(parseStellarConfigurationJSON(s, n)); }

static std::string jsonEscape(const std::string& s) {
  std::string o;
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
    else if (c < 0x20) { char b[8]; std::snprintf(b, sizeof b, "\\u%04x", c); o += b; }
    else o += (char)c;
  }
  return o;
}

static std::string idxList(const std::vector<NodeIx>& v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i]);
  return s + "]";
}

}  // namespace qio

// =====================================================================================
// C-ABI used by tests/ and bench.py's cpu_baseline (ctypes).  Strings returned are
// malloc'd JSON; free with qio_free_str.
// =====================================================================================
extern "C" {

struct qio_handle {
  qio::Graph g;
};

static thread_local std::string g_qio_err;

const char* qio_last_error() { return g_qio_err.c_str(); }

void* qio_load(const char* json, size_t len) {
  try {
    auto* h = new qio_handle{qio::loadGraph(json, len)};
    return h;
  } catch (const std::exception& e) {
    g_qio_err = e.what();
    return nullptr;
  }
}

void qio_free(void* h) { delete (qio_handle*)h; }

void qio_free_str(char* s) { std::free(s); }

uint64_t qio_num_vertices(void* h) { return ((qio_handle*)h)->g.size(); }

// containsQuorum(nodes = X[0..nx), availableNodes = avail[0..n)) -> survivors (input order)
uint64_t qio_contains_quorum(void* h, const uint32_t* X, uint64_t nx, const uint8_t* avail, uint32_t* out) {
  auto& g = ((qio_handle*)h)->g;
  qio::Ctx ctx;
  std::vector<qio::NodeIx> nodes(X, X + nx);
  std::vector<bool> a(g.size());
  for (size_t i = 0; i < g.size(); ++i) a[i] = avail[i] != 0;
  auto r = qio::containsQuorum(ctx, nodes, a, g);
  for (size_t i = 0; i < r.size(); ++i) out[i] = (uint32_t)r[i];
  return r.size();
}

int qio_slice(void* h, uint32_t v, const uint8_t* avail) {
  auto& g = ((qio_handle*)h)->g;
  std::vector<bool> a(g.size());
  for (size_t i = 0; i < g.size(); ++i) a[i] = avail[i] != 0;
  return qio::containsQuorumSlice(v, g.v[v].qSet, a) ? 1 : 0;
}

// Graph description: {"n":..,"adj":[[..]..],"comp":[..],"nscc":..}
char* qio_graph_json(void* h) {
  auto& g = ((qio_handle*)h)->g;
  size_t cnt = 0;
  auto comp = qio::strongComponents(g, cnt);
  std::string s = "{\"n\":" + std::to_string(g.size()) + ",\"nscc\":" + std::to_string(cnt) + ",\"comp\":" +
                  qio::idxList(std::vector<qio::NodeIx>(comp.begin(), comp.end())) + ",\"adj\":[";
  for (size_t v = 0; v < g.size(); ++v) s += (v ? "," : "") + qio::idxList(g.adj[v]);
  s += "],\"ids\":[";
  for (size_t v = 0; v < g.size(); ++v) s += std::string(v ? "," : "") + "\"" + qio::jsonEscape(g.v[v].nodeID) + "\"";
  s += "]}";
  return strdup(s.c_str());
}

// Full solve (cpp:615-707) with counters.  tiebreak: 0 lowest, 1 random.
char* qio_solve(void* h, int tiebreak, uint64_t seed, uint64_t node_budget) {
  auto& g = ((qio_handle*)h)->g;
  qio::Ctx ctx;
  ctx.tie = tiebreak ? qio::TIE_RANDOM : qio::TIE_LOWEST;
  ctx.rng.seed((unsigned)seed);
  ctx.budget = node_budget;
  std::ostringstream sink;
  auto t0 = std::chrono::steady_clock::now();
  qio::SolveInfo info = qio::solve(ctx, g, sink, false, false);
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::string s = "{";
  s += "\"verdict\":" + std::string(info.verdict ? "true" : "false");
  s += ",\"aborted\":" + std::string(ctx.aborted ? "true" : "false");
  s += ",\"n\":" + std::to_string(info.n);
  s += ",\"nscc\":" + std::to_string(info.sccCount);
  s += ",\"scc_with_quorum\":" + std::to_string(info.withQuorum);
  s += ",\"scc_quorum_ids\":" + qio::idxList(info.sccQuorumIds);
  s += ",\"front\":" + qio::idxList(info.front);
  s += ",\"searched\":" + std::string(info.searched ? "true" : "false");
  s += ",\"nodes\":" + std::to_string(ctx.nodes);
  s += ",\"evals\":" + std::to_string(ctx.evals);
  s += ",\"scc_evals\":" + std::to_string(ctx.scc_evals);
  s += ",\"minq\":" + std::to_string(ctx.minq);
  s += ",\"zero_fallback\":" + std::to_string(ctx.zero_fallback);
  s += ",\"max_depth\":" + std::to_string(ctx.max_depth);
  s += ",\"q1\":" + qio::idxList(info.q1);
  s += ",\"q2\":" + qio::idxList(info.q2);
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.9f", secs);
  s += ",\"seconds\":" + std::string(buf);
  std::snprintf(buf, sizeof buf, "%.9f", info.search_seconds);
  s += ",\"search_seconds\":" + std::string(buf);
  s += "}";
  return strdup(s.c_str());
}

// CLI-equivalent text output of solve (-v / -g) for golden text tests.
char* qio_solve_text(void* h, int verbose, int graphviz) {
  auto& g = ((qio_handle*)h)->g;
  qio::Ctx ctx;
  std::ostringstream out;
  out << std::boolalpha;
  auto info = qio::solve(ctx, g, out, verbose != 0, graphviz != 0);
  out << info.verdict << std::endl;
  return strdup(out.str().c_str());
}

// Iteration order of std::unordered_set<size_t> built like cpp:308 from the keys of
// seq[0..n_seq) (keys[v] = global index of local vertex v); out = local vertices.
uint64_t qio_hash_order(const uint32_t* keys, uint32_t n_keys, const uint32_t* seq, uint32_t n_seq, uint32_t* out) {
  std::vector<size_t> v;
  std::unordered_map<size_t, uint32_t> local;
  for (uint32_t i = 0; i < n_keys; ++i) local[keys[i]] = i;
  for (uint32_t i = 0; i < n_seq; ++i) v.push_back(keys[seq[i]]);
  std::unordered_set<size_t> s(v.begin(), v.end());
  uint64_t n = 0;
  for (size_t k : s) out[n++] = local[k];
  return n;
}

// bucket_count() of that set after k distinct insertions, k = 1..nmax
void qio_hash_bucket_counts(uint32_t nmax, uint64_t* out) {
  std::vector<size_t> v;
  for (uint32_t k = 1; k <= nmax; ++k) {
    v.push_back(k * 7 + 3);
    std::unordered_set<size_t> s(v.begin(), v.end());
    out[k - 1] = s.bucket_count();
  }
}

char* qio_pagerank_text(void* h, float m, float conv, uint64_t iters) {
  auto& g = ((qio_handle*)h)->g;
  auto pr = qio::pageRank(g, m, conv, iters);
  std::ostringstream out;
  out << "PageRank:" << std::endl;
  qio::printPageRank(g, out, pr);
  return strdup(out.str().c_str());
}

}  // extern "C"

#ifdef QIO_MAIN
// main (cpp:744-800), minus Boost.program_options: the oracle binary accepts the same
// short/long flags.  Used only to produce golden CLI transcripts.
int main(int argc, char** argv) {
  bool help = false, verbose = false, graphviz = false, pagerankF = false;
  uint64_t maxIterations = 100000;
  float danglingFactor = 0.0001f, convergence = 0.0001f;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* name) -> std::string {
      if (i + 1 >= argc) { std::cout << "Invalid option!" << std::endl; std::exit(1); }
      (void)name;
      return argv[++i];
    };
    if (a == "-h" || a == "--help") help = true;
    else if (a == "-v" || a == "--verbose") verbose = true;
    else if (a == "-g" || a == "--graph") graphviz = true;
    else if (a == "-t" || a == "--trace") {}
    else if (a == "-p" || a == "--pagerank") pagerankF = true;
    else if (a == "-i" || a == "--max_iterations") maxIterations = std::stoull(val("i"));
    else if (a == "-m" || a == "--dangling_factor") danglingFactor = std::stof(val("m"));
    else if (a == "-c" || a == "--convergence") convergence = std::stof(val("c"));
    else { std::cout << "Invalid option!" << std::endl; return 1; }
  }
  if (help) { std::cout << "(help text: see product CLI)" << std::endl; return 0; }
  std::string in((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
  qio::Graph g;
  try {
    g = qio::loadGraph(in.data(), in.size());
  } catch (const std::exception& e) {
    std::cerr << "terminate called after throwing an instance of 'ptree_error'\n  what():  " << e.what() << std::endl;
    std::abort();
  }
  if (pagerankF) {
    auto pr = qio::pageRank(g, danglingFactor, convergence, maxIterations);
    std::cout << "PageRank:" << std::endl;
    qio::printPageRank(g, std::cout, pr);
    return 0;
  }
  std::cout << std::boolalpha;
  qio::Ctx ctx;
  auto info = qio::solve(ctx, g, std::cout, verbose, graphviz);
  std::cout << info.verdict << std::endl;
  return info.verdict ? 0 : 1;
}
#endif
