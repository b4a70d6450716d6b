// Stellarbeat JSON ingestion (replaces parseQuorumSet / parseStellarConfigurationJSON,
// quorum_intersection.cpp:402-436, which use boost::property_tree::read_json).
//
// property_tree semantics reproduced (they decide what the reference accepts):
//  * every scalar is stored as text: numbers verbatim, true/false/null as the words,
//    strings unescaped (\uXXXX -> UTF-8, surrogate pairs combined);
//  * arrays are children with empty keys; objects keep duplicate keys, get() takes the
//    first one; a top-level object is walked member by member like an array;
//  * get<size_t>("threshold") parses the text with operator>> and requires that the
//    whole text (up to trailing blanks) is consumed; libstdc++ num_get accepts a leading
//    '-' for unsigned and wraps ("-1" -> SIZE_MAX, no failbit), as property_tree does;
//  * a quorum set with no children (null, {}, [], "x", 3) is an empty quorum set;
//  * missing publicKey / quorumSet / threshold / validators / innerQuorumSets -> error.
// Errors are reported as qi::Error(QI_ERR_PARSE); the reference aborts (uncaught ptree_error).
#include <cstring>
#include <sstream>

#include "qi_internal.h"
#include "../../include/quorum_intersection.h"

namespace qi {
namespace {

// Arena DOM: node i has text + [first_child, child_count) into the kids array.
struct Dom {
  struct Node {
    std::string text;
    std::vector<std::pair<std::string, uint32_t>> kids;
  };
  std::vector<Node> nodes;
  uint32_t add() {
    nodes.emplace_back();
    return (uint32_t)nodes.size() - 1;
  }
  int child(uint32_t n, const char* key) const {
    for (const auto& k : nodes[n].kids)
      if (k.first == key) return (int)k.second;
    return -1;
  }
};

[[noreturn]] void fail(const std::string& what) { throw Error(QI_ERR_PARSE, what); }

class Parser {
 public:
  Parser(const char* s, size_t n, Dom& d) : s_(s), e_(s + n), d_(d) {}
  uint32_t document() {
    skip();
    uint32_t root = d_.add();
    value(root, 0);
    skip();
    if (s_ != e_) fail("json: garbage after data");
    return root;
  }

 private:
  const char* s_;
  const char* e_;
  Dom& d_;

  void skip() {
    while (s_ < e_ && (*s_ == ' ' || *s_ == '\n' || *s_ == '\r' || *s_ == '\t')) ++s_;
  }
  bool word(const char* w, size_t n) {
    if ((size_t)(e_ - s_) < n || std::memcmp(s_, w, n) != 0) return false;
    s_ += n;
    return true;
  }
  void value(uint32_t node, int depth) {
    if (depth > 4096) fail("json: nesting too deep");
    if (s_ >= e_) fail("json: expected value");
    switch (*s_) {
      case '{': object(node, depth); return;
      case '[': array(node, depth); return;
      case '"': d_.nodes[node].text = string(); return;
      default: break;
    }
    if (word("true", 4)) { d_.nodes[node].text = "true"; return; }
    if (word("false", 5)) { d_.nodes[node].text = "false"; return; }
    if (word("null", 4)) { d_.nodes[node].text = "null"; return; }
    number(node);
  }
  static bool digit(char c) { return c >= '0' && c <= '9'; }
  void number(uint32_t node) {
    const char* b = s_;
    if (s_ < e_ && *s_ == '-') ++s_;
    if (s_ >= e_ || !digit(*s_)) fail("json: expected value");
    if (*s_ == '0') ++s_;
    else while (s_ < e_ && digit(*s_)) ++s_;
    if (s_ < e_ && *s_ == '.') {
      ++s_;
      if (s_ >= e_ || !digit(*s_)) fail("json: expected digits after '.'");
      while (s_ < e_ && digit(*s_)) ++s_;
    }
    if (s_ < e_ && (*s_ == 'e' || *s_ == 'E')) {
      ++s_;
      if (s_ < e_ && (*s_ == '+' || *s_ == '-')) ++s_;
      if (s_ >= e_ || !digit(*s_)) fail("json: expected exponent digits");
      while (s_ < e_ && digit(*s_)) ++s_;
    }
    d_.nodes[node].text.assign(b, s_);
  }
  unsigned hex4() {
    if (e_ - s_ < 4) fail("json: invalid escape");
    unsigned v = 0;
    for (int i = 0; i < 4; ++i, ++s_) {
      char c = *s_;
      unsigned d;
      if (digit(c)) d = (unsigned)(c - '0');
      else if (c >= 'a' && c <= 'f') d = (unsigned)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') d = (unsigned)(c - 'A' + 10);
      else fail("json: invalid escape");
      v = v * 16 + d;
    }
    return v;
  }
  static void put_utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) { o.push_back((char)cp); return; }
    if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 63))); return; }
    if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 63)));
      o.push_back((char)(0x80 | (cp & 63)));
      return;
    }
    o.push_back((char)(0xF0 | (cp >> 18)));
    o.push_back((char)(0x80 | ((cp >> 12) & 63)));
    o.push_back((char)(0x80 | ((cp >> 6) & 63)));
    o.push_back((char)(0x80 | (cp & 63)));
  }
  std::string string() {
    ++s_;
    std::string o;
    const char* run = s_;
    for (;;) {
      if (s_ >= e_) fail("json: unterminated string");
      unsigned char c = (unsigned char)*s_;
      if (c == '"') {
        o.append(run, s_);
        ++s_;
        return o;
      }
      if (c < 0x20) fail("json: control character in string");
      if (c != '\\') { ++s_; continue; }
      o.append(run, s_);
      ++s_;
      if (s_ >= e_) fail("json: invalid escape");
      char x = *s_++;
      switch (x) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xDC00 && cp <= 0xDFFF) fail("json: invalid codepoint");
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (e_ - s_ < 2 || s_[0] != '\\' || s_[1] != 'u') fail("json: invalid codepoint");
            s_ += 2;
            unsigned lo = hex4();
            if (lo < 0xDC00 || lo > 0xDFFF) fail("json: invalid codepoint");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: fail("json: invalid escape");
      }
      run = s_;
    }
  }
  void object(uint32_t node, int depth) {
    ++s_;
    skip();
    if (s_ < e_ && *s_ == '}') { ++s_; return; }
    for (;;) {
      skip();
      if (s_ >= e_ || *s_ != '"') fail("json: expected member name");
      std::string key = string();
      skip();
      if (s_ >= e_ || *s_ != ':') fail("json: expected ':'");
      ++s_;
      skip();
      uint32_t c = d_.add();
      value(c, depth + 1);
      d_.nodes[node].kids.emplace_back(std::move(key), c);
      skip();
      if (s_ < e_ && *s_ == ',') { ++s_; continue; }
      if (s_ < e_ && *s_ == '}') { ++s_; return; }
      fail("json: expected ',' or '}'");
    }
  }
  void array(uint32_t node, int depth) {
    ++s_;
    skip();
    if (s_ < e_ && *s_ == ']') { ++s_; return; }
    for (;;) {
      skip();
      uint32_t c = d_.add();
      value(c, depth + 1);
      d_.nodes[node].kids.emplace_back(std::string(), c);
      skip();
      if (s_ < e_ && *s_ == ',') { ++s_; continue; }
      if (s_ < e_ && *s_ == ']') { ++s_; return; }
      fail("json: expected ',' or ']'");
    }
  }
};

// stream_translator<size_t>: iss >> v; iss >> ws; must reach EOF without failbit.
uint64_t to_size_t(const std::string& text, const char* key) {
  std::istringstream iss(text);
  unsigned long v = 0;
  iss >> v;
  if (!iss.eof()) iss >> std::ws;
  if (iss.fail() || iss.bad() || iss.get() != std::char_traits<char>::eof())
    fail(std::string("conversion of data to type failed: ") + key + "=\"" + text + "\"");
  return v;
}

QuorumSetIds quorum_set(const Dom& d, uint32_t n) {
  QuorumSetIds q;
  if (d.nodes[n].kids.empty()) return q;  // null / {} : empty set, threshold unset
  int t = d.child(n, "threshold");
  if (t < 0) fail("No such node (threshold)");
  q.threshold = to_size_t(d.nodes[t].text, "threshold");
  q.has_threshold = true;
  int v = d.child(n, "validators");
  if (v < 0) fail("No such node (validators)");
  for (const auto& k : d.nodes[v].kids) q.validators.push_back(d.nodes[k.second].text);
  int in = d.child(n, "innerQuorumSets");
  if (in < 0) fail("No such node (innerQuorumSets)");
  for (const auto& k : d.nodes[in].kids) q.inner.push_back(quorum_set(d, k.second));
  return q;
}

}  // namespace

std::vector<StellarNode> parse_stellar_json(const char* text, size_t len) {
  Dom d;
  d.nodes.reserve(len / 16 + 16);
  uint32_t root = Parser(text, len, d).document();
  std::vector<StellarNode> out;
  out.reserve(d.nodes[root].kids.size());
  for (const auto& k : d.nodes[root].kids) {
    uint32_t e = k.second;
    int pk = d.child(e, "publicKey");
    if (pk < 0) fail("No such node (publicKey)");
    int nm = d.child(e, "name");
    int qs = d.child(e, "quorumSet");
    if (qs < 0) fail("No such node (quorumSet)");
    StellarNode s;
    s.publicKey = d.nodes[pk].text;
    if (nm >= 0) s.name = d.nodes[nm].text;
    s.qset = quorum_set(d, (uint32_t)qs);
    out.push_back(std::move(s));
  }
  return out;
}

}  // namespace qi

// ----------------------------------------------------------------------------------
// Phase timing (qi_internal.h, namespace timing)
// ----------------------------------------------------------------------------------
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <utility>

namespace qi {
namespace timing {
namespace {
std::mutex g_mu;
std::vector<std::pair<std::string, double>> g_phases;
long long now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

bool enabled() {
  static const bool on = std::getenv("QI_TIMING") != nullptr;
  return on;
}

namespace {
void accumulate(const std::string& key, double v) {
  if (!enabled()) return;
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& p : g_phases)
    if (p.first == key) {
      p.second += v;
      return;
    }
  g_phases.emplace_back(key, v);
}
}  // namespace

void add(const char* phase, double ms) { accumulate(std::string(phase) + "_ms", ms); }
void count(const char* name, double n) { accumulate(name, n); }

std::string json() {
  std::lock_guard<std::mutex> g(g_mu);
  std::string o = "{";
  char buf[64];
  for (size_t i = 0; i < g_phases.size(); ++i) {
    std::snprintf(buf, sizeof buf, "%.3f", g_phases[i].second);
    o += (i ? ", \"" : "\"") + g_phases[i].first + "\": " + buf;
  }
  return o + "}";
}

Scope::Scope(const char* p) : phase(p), on(enabled()), t0(on ? now_ns() : 0) {}
Scope::~Scope() {
  if (on) add(phase, (double)(now_ns() - t0) * 1e-6);
}
}  // namespace timing
}  // namespace qi

