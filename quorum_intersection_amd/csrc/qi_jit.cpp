// Run-time specialisation of the search kernel (hipRTC).
//
// The search spends its time in containsQuorum (cpp:140-177) and findBestNode
// (cpp:203-250) over ONE flattened SCC.  The ahead-of-time kernel interprets the packed
// threshold-node table (scalar loads, loop control, flag tests per node: ~80% of the
// issued instructions in profile r01b).  Here the same kernel source
// (qi_search_kernel.h) is compiled once more with an evaluator generated for the given
// SCC: every threshold node becomes v_and_b32 + v_bcnt_u32_b32 on literal masks and a
// compare with a literal threshold, fully unrolled.  Code objects are cached on disk by
// a hash of their source.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "qi_jit.h"
#include "../../include/quorum_intersection.h"

#include "qi_search_kernel_src.inc"  // kSearchKernelSrc: qi_search_kernel.h as a string

namespace qi {
namespace {

std::string hex(uint32_t v) {
  char b[16];
  std::snprintf(b, sizeof b, "0x%08xu", v);
  return b;
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

std::string cache_dir() {
  if (const char* e = std::getenv("QI_JIT_CACHE")) return e;
  Dl_info info;
  if (dladdr((void*)&fnv1a, &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    auto k = p.rfind('/');
    if (k != std::string::npos) return p.substr(0, k) + "/jit_cache";
  }
  return "/tmp/qi_jit_cache";
}

}  // namespace

uint32_t jit_lds_ow(const LocalFlat& f) { return (f.m / 2 + 1 + 3) / 4; }

bool jit_eligible(const LocalFlat& f) {
  return f.T <= 1024 && f.G <= 1024 && f.extra_src.size() <= 4096 && f.grp_extra.size() <= 4096 * 8;
}

namespace {

// Sibling threshold nodes evaluated bit-sliced.  Leaf TNs (validators only, multiplicity 1)
// whose vertex masks are the same bit pattern at different positions of one mask word and
// whose thresholds agree -- the organisations of a tiered FBAS, "2 of 3" each -- are
// evaluated together: plane j = X >> o_j holds the j-th member of every sibling at the
// sibling's base bit, a bit-sliced adder counts the planes, and one boolean function of the
// count bits gives "count >= threshold" for all siblings at once (result bit = base bit).
// 10 siblings of 3 validators cost 2 shifts + 1 three-input bit operation + 1 AND instead of
// 10 x (AND, BCNT, compare, select).  Parents count satisfied siblings with one popcount.
struct SlicedGroup {
  uint32_t word = 0;              // vertex mask word the siblings live in
  std::vector<uint32_t> offs;     // bit offsets of the pattern (offs[0] == 0)
  int32_t t0 = 0, t1 = 0;         // thresholds (outside unavailable / available)
  std::vector<uint32_t> tns;      // member TNs
  uint32_t base_bits = 0;         // OR of 1 << base over the members
};

// Statements that leave in `out` the bitwise "at least k of the planes x[] are set".
std::string sliced_at_least(const std::vector<std::string>& x, int k, const std::string& out, const std::string& pfx) {
  const int n = (int)x.size();
  std::ostringstream o;
  auto join = [&](const char* op) {
    std::string e = x[0];
    for (int i = 1; i < n; ++i) e += std::string(" ") + op + " " + x[i];
    return e;
  };
  if (k <= 0) { o << "const uint32_t " << out << " = 0xFFFFFFFFu;"; return o.str(); }
  if (k > n) { o << "const uint32_t " << out << " = 0u;"; return o.str(); }
  if (k == 1) { o << "const uint32_t " << out << " = " << join("|") << ";"; return o.str(); }
  if (k == n) { o << "const uint32_t " << out << " = " << join("&") << ";"; return o.str(); }
  if (n == 3) {  // k == 2: majority
    o << "const uint32_t " << out << " = (" << x[0] << " & " << x[1] << ") | (" << x[2] << " & (" << x[0] << " | " << x[1] << "));";
    return o.str();
  }
  // column compression with full / half adders: cols[w] = bits of weight 2^w
  std::vector<std::vector<std::string>> cols(4);
  cols[0] = x;
  int tmp = 0;
  for (int w = 0; w < 3; ++w) {
    while (cols[w].size() > 1) {
      const std::string s_ = pfx + "s" + std::to_string(tmp), c_ = pfx + "c" + std::to_string(tmp);
      ++tmp;
      if (cols[w].size() >= 3) {
        const std::string a = cols[w][0], b = cols[w][1], c = cols[w][2];
        cols[w].erase(cols[w].begin(), cols[w].begin() + 3);
        o << "const uint32_t " << s_ << " = " << a << " ^ " << b << " ^ " << c << "; const uint32_t " << c_ << " = (" << a
          << " & " << b << ") | (" << c << " & (" << a << " | " << b << ")); ";
      } else {
        const std::string a = cols[w][0], b = cols[w][1];
        cols[w].erase(cols[w].begin(), cols[w].begin() + 2);
        o << "const uint32_t " << s_ << " = " << a << " ^ " << b << "; const uint32_t " << c_ << " = " << a << " & " << b
          << "; ";
      }
      cols[w].push_back(s_);
      cols[w + 1].push_back(c_);
    }
  }
  auto bit = [&](int w) -> std::string { return cols[w].empty() ? std::string("0u") : cols[w][0]; };
  const std::string b0 = bit(0), b1 = bit(1), b2 = bit(2);
  std::string e;
  switch (k) {  // count = 4*b2 + 2*b1 + b0 (n <= 7)
    case 2: e = b1 + " | " + b2; break;
    case 3: e = "(" + b1 + " & " + b0 + ") | " + b2; break;
    case 4: e = b2; break;
    case 5: e = b2 + " & (" + b1 + " | " + b0 + ")"; break;
    case 6: e = b2 + " & " + b1; break;
    default: e = b2 + " & " + b1 + " & " + b0; break;  // 7
  }
  o << "const uint32_t " << out << " = " << e << ";";
  return o.str();
}

std::vector<SlicedGroup> find_sliced_groups(const LocalFlat& f, std::vector<int>& grp_of, std::vector<uint32_t>& base_of) {
  grp_of.assign(f.T, -1);
  base_of.assign(f.T, 0);
  std::vector<SlicedGroup> groups;
  if (std::getenv("QI_JIT_NO_SLICE")) return groups;  // diagnostics: per-TN evaluation only
  for (uint32_t t = 0; t < f.T; ++t) {
    if (f.flags[t] & 3u) continue;  // inverted test or extra multiplicity planes
    bool leaf = true;
    for (uint32_t w = 0; w < f.tw; ++w) leaf = leaf && f.cmask[(size_t)t * f.tw + w] == 0;
    if (!leaf || f.extra_off[t] != f.extra_off[t + 1]) continue;
    int word = -1;
    bool one = true;
    for (uint32_t w = 0; w < f.mw; ++w)
      if (f.vmask[(size_t)t * f.mw + w]) {
        one = one && word < 0;
        word = (int)w;
      }
    if (word < 0 || !one) continue;
    const uint32_t m = f.vmask[(size_t)t * f.mw + word];
    const int n = __builtin_popcount(m);
    const int32_t t0 = f.thr[2 * t], t1 = f.thr[2 * t + 1];
    if (n > 7 || t0 < 1 || t0 > n || t1 < 1 || t1 > n) continue;
    const uint32_t base = (uint32_t)__builtin_ctz(m);
    std::vector<uint32_t> offs;
    for (uint32_t b = base; b < 32; ++b)
      if ((m >> b) & 1u) offs.push_back(b - base);
    int g = -1;
    for (size_t i = 0; i < groups.size(); ++i)
      if (groups[i].word == (uint32_t)word && groups[i].offs == offs && groups[i].t0 == t0 && groups[i].t1 == t1 &&
          !((groups[i].base_bits >> base) & 1u))
        g = (int)i;
    if (g < 0) {
      SlicedGroup ng;
      ng.word = (uint32_t)word;
      ng.offs = offs;
      ng.t0 = t0;
      ng.t1 = t1;
      groups.push_back(ng);
      g = (int)groups.size() - 1;
    }
    groups[g].tns.push_back(t);
    groups[g].base_bits |= 1u << base;
    grp_of[t] = g;
    base_of[t] = base;
  }
  // a group pays off from three siblings on; smaller ones stay per-TN
  std::vector<SlicedGroup> kept;
  std::vector<int> remap(groups.size(), -1);
  for (size_t i = 0; i < groups.size(); ++i)
    if (groups[i].tns.size() >= 3) {
      remap[i] = (int)kept.size();
      kept.push_back(groups[i]);
    }
  for (uint32_t t = 0; t < f.T; ++t)
    if (grp_of[t] >= 0) grp_of[t] = remap[grp_of[t]];
  return kept;
}

}  // namespace

std::string jit_source(const LocalFlat& f, int MW, int TW, int SMAX, bool stamps, bool tie_random) {
  std::ostringstream o;
  if (stamps) o << "#define QI_STAMPS 1\n";
  o << "#define QI_LDS_OW " << jit_lds_ow(f) << "\n";  // D-order words per lane: |D| <= m/2 + 1
  // diagnostics only (never set for measurements): QI_JIT_DEFINES="A,B=2" adds #defines
  // for A/B runs of the kernel's compile-time switches
  if (const char* e = std::getenv("QI_JIT_DEFINES")) {
    std::string d = e;
    size_t p = 0;
    while (p < d.size()) {
      size_t q = d.find(',', p);
      if (q == std::string::npos) q = d.size();
      std::string item = d.substr(p, q - p);
      const size_t eq = item.find('=');
      if (!item.empty()) o << "#define " << (eq == std::string::npos ? item + " 1" : item.substr(0, eq) + " " + item.substr(eq + 1)) << "\n";
      p = q + 1;
    }
  }
  o << kSearchKernelSrc << "\nnamespace qi {\nnamespace dev {\n";
  o << "// generated evaluator: m=" << f.m << " T=" << f.T << " R=" << f.R << " G=" << f.G << "\n";
  o << "struct SpecEval {\n";
  // ---------------- containsQuorum ----------------
  o << "  template <int POL>\n  static __device__ __forceinline__ bool gfp(const LocalDev&, uint32_t (&X)[" << MW
    << "], uint32_t pol, uint32_t& rounds) {\n    (void)pol;\n";
  // |X| < qmin => empty fixpoint (LocalFlat::qmin), before any round
  o << "    { const uint32_t c = __popc(X[0])";
  for (int w = 1; w < MW; ++w) o << " + __popc(X[" << w << "])";
  o << "; const uint32_t q = POL == 0 ? " << f.qmin[0] << "u : (POL == 1 ? " << f.qmin[1] << "u : (pol ? " << f.qmin[1]
    << "u : " << f.qmin[0] << "u));\n      if (c < q) {";
  for (int w = 0; w < MW; ++w) o << " X[" << w << "] = 0u;";
  o << " } }\n";
  o << "    for (;;) {\n      if (!(X[0]";
  for (int w = 1; w < MW; ++w) o << " | X[" << w << "]";
  o << ")) return false;\n      ++rounds;\n";
  for (int w = 0; w < TW; ++w) o << "      uint32_t sb" << w << " = 0u;\n";
  // sibling groups first (leaf TNs): R<g> bit `base` = sibling satisfied
  std::vector<int> grp_of;
  std::vector<uint32_t> base_of;
  const std::vector<SlicedGroup> sgroups = find_sliced_groups(f, grp_of, base_of);
  for (size_t g = 0; g < sgroups.size(); ++g) {
    const SlicedGroup& sg = sgroups[g];
    const std::string G = std::to_string(g);
    std::vector<std::string> planes;
    o << "      uint32_t R" << G << ";\n      {";
    for (size_t j = 0; j < sg.offs.size(); ++j) {
      const std::string nm = "p" + G + "_" + std::to_string(j);
      if (sg.offs[j] == 0) o << " const uint32_t " << nm << " = X[" << sg.word << "];";
      else o << " const uint32_t " << nm << " = X[" << sg.word << "] >> " << sg.offs[j] << "u;";
      planes.push_back(nm);
    }
    o << "\n        " << sliced_at_least(planes, sg.t0, "ge0_", "a" + G + "_") << "\n";
    if (sg.t1 != sg.t0) {
      o << "        " << sliced_at_least(planes, sg.t1, "ge1_", "b" + G + "_") << "\n";
      o << "        R" << G << " = (POL == 0 ? ge0_ : POL == 1 ? ge1_ : (pol ? ge1_ : ge0_)) & " << hex(sg.base_bits) << "; }\n";
    } else {
      o << "        R" << G << " = ge0_ & " << hex(sg.base_bits) << "; }\n";
    }
  }
  // popcount terms of a mask over TN-satisfaction word w: grouped children are counted in
  // their group's result word, the rest in sb<w>
  auto child_terms = [&](uint32_t w, uint32_t m, std::vector<std::string>& terms) {
    uint32_t rest = m;
    std::vector<uint32_t> sub(sgroups.size(), 0);
    for (uint32_t b = 0; b < 32; ++b) {
      const uint32_t c = 32 * w + b;
      if (((m >> b) & 1u) && c < f.T && grp_of[c] >= 0) {
        rest &= ~(1u << b);
        sub[grp_of[c]] |= 1u << base_of[c];
      }
    }
    if (rest) terms.push_back("__popc(sb" + std::to_string(w) + " & " + hex(rest) + ")");
    for (size_t g = 0; g < sgroups.size(); ++g)
      if (sub[g]) {
        if (sub[g] == sgroups[g].base_bits) terms.push_back("__popc(R" + std::to_string(g) + ")");
        else terms.push_back("__popc(R" + std::to_string(g) + " & " + hex(sub[g]) + ")");
      }
  };
  // 0/1 satisfaction of TN t as an expression
  auto sat_bit = [&](uint32_t t) -> std::string {
    if (grp_of[t] >= 0) return "((R" + std::to_string(grp_of[t]) + " >> " + std::to_string(base_of[t]) + "u) & 1u)";
    return "((sb" + std::to_string(t / 32) + " >> " + std::to_string(t % 32) + "u) & 1u)";
  };
  std::vector<std::vector<std::string>> extra(f.T);
  for (uint32_t t = 0; t < f.T; ++t)
    for (uint32_t e = f.extra_off[t]; e < f.extra_off[t + 1]; ++e) {
      const uint32_t src = f.extra_src[e];
      if (src < f.mw) extra[t].push_back("__popc(X[" + std::to_string(src) + "] & " + hex(f.extra_mask[e]) + ")");
      else child_terms(src - f.mw, f.extra_mask[e], extra[t]);
    }
  for (uint32_t t = 0; t < f.T; ++t) {
    if (grp_of[t] >= 0) continue;  // evaluated with its siblings above
    std::vector<std::string> terms;
    for (uint32_t w = 0; w < f.mw; ++w) {
      const uint32_t m = f.vmask[(size_t)t * f.mw + w];
      if (m) terms.push_back("__popc(X[" + std::to_string(w) + "] & " + hex(m) + ")");
    }
    for (uint32_t w = 0; w < f.tw; ++w) {
      const uint32_t m = f.cmask[(size_t)t * f.tw + w];
      if (m) child_terms(w, m, terms);
    }
    for (auto& x : extra[t]) terms.push_back(x);
    std::string c = terms.empty() ? std::string("0u") : terms[0];
    for (size_t i = 1; i < terms.size(); ++i) c += " + " + terms[i];
    const bool inv = (f.flags[t] & 1u) != 0;
    const int32_t t0 = f.thr[2 * t], t1 = f.thr[2 * t + 1];
    std::string bit;
    if (inv) {
      bit = "(c == 0u)";
    } else {
      auto cmp = [&](int32_t th) -> std::string {
        if (th <= 0) return "true";
        if (th == INT32_MAX) return "false";
        return "(c >= " + std::to_string(th) + "u)";
      };
      if (t0 == t1) bit = cmp(t0);
      else bit = "(POL == 0 ? " + cmp(t0) + " : POL == 1 ? " + cmp(t1) + " : (pol ? " + cmp(t1) + " : " + cmp(t0) + "))";
    }
    o << "      { const uint32_t c = " << c << "; (void)c; sb" << (t / 32) << " |= (uint32_t)(" << bit << ") << "
      << (t % 32) << "u; }\n";
  }
  // one root TN for every vertex of the SCC (a symmetric tier): all of X survives a round or
  // none does, so the first round decides and there is no loop
  bool one_root = f.R == 1;
  for (uint32_t w = 0; w < f.mw && one_root; ++w) {
    uint32_t all = 0;
    for (uint32_t v = 32 * w; v < f.m && v < 32 * w + 32; ++v) all |= 1u << (v & 31);
    one_root = f.root_users[w] == all;
  }
  if (one_root) {
    const uint32_t tn = f.root_tn[0];
    o << "#if QI_ONE_ROOT\n      { const bool s_ = " << sat_bit(tn) << " != 0u; if (!s_) {";
    for (int w = 0; w < MW; ++w) o << " X[" << w << "] = 0u;";
    o << " } return s_; }\n#endif\n";
  }
  for (int w = 0; w < MW; ++w) o << "      uint32_t n" << w << " = 0u;\n";
  for (uint32_t r = 0; r < f.R; ++r) {
    const uint32_t tn = f.root_tn[r];
    o << "      { const uint32_t s = 0u - " << sat_bit(tn) << ";";
    for (uint32_t w = 0; w < f.mw; ++w) {
      const uint32_t u = f.root_users[(size_t)r * f.mw + w];
      if (u) o << " n" << w << " |= " << hex(u) << " & s;";
    }
    o << " }\n";
  }
  o << "      bool same = true;\n";
  for (int w = 0; w < MW; ++w) o << "      n" << w << " &= X[" << w << "]; same &= (n" << w << " == X[" << w << "]);\n";
  o << "      if (same) return true;\n";
  for (int w = 0; w < MW; ++w) o << "      X[" << w << "] = n" << w << ";\n";
  o << "    }\n  }\n";
  // ---------------- findBestNode ----------------
  o << "  static __device__ __forceinline__ uint32_t best(const LocalDev&, const uint32_t (&Q)[" << MW
    << "], const uint32_t (&D)[" << MW << "], uint32_t& zero_fallback) {\n"
    << "    uint32_t bestdeg = 0u, bestv = 0xFFFFFFFFu;\n";
  for (uint32_t g = 0; g < f.G; ++g) {
    std::vector<std::string> terms;
    for (uint32_t w = 0; w < f.mw; ++w) {
      const uint32_t m = f.grp_col[(size_t)g * f.mw + w];
      if (m) terms.push_back("__popc(Q[" + std::to_string(w) + "] & " + hex(m) + ")");
    }
    for (uint32_t e = f.grp_extra_off[g]; e < f.grp_extra_off[g + 1]; ++e)
      for (uint32_t w = 0; w < f.mw; ++w) {
        const uint32_t m = f.grp_extra[(size_t)e * f.mw + w];
        if (m) terms.push_back("__popc(Q[" + std::to_string(w) + "] & " + hex(m) + ")");
      }
    std::string deg = terms.empty() ? std::string("0u") : terms[0];
    for (size_t i = 1; i < terms.size(); ++i) deg += " + " + terms[i];
    o << "    { const uint32_t deg = " << deg << "; uint32_t low = 0xFFFFFFFFu;";
    for (int w = (int)f.mw - 1; w >= 0; --w) {
      const uint32_t m = f.grp_members[(size_t)g * f.mw + w];
      if (!m) continue;
      o << " { const uint32_t c = Q[" << w << "] & ~D[" << w << "] & " << hex(m) << "; low = c ? " << (w * 32)
        << "u + (uint32_t)__builtin_ctz(c) : low; }";
    }
    o << "\n      const bool better = (low != 0xFFFFFFFFu) && (deg > bestdeg || (deg == bestdeg && low < bestv));"
      << " bestdeg = better ? deg : bestdeg; bestv = better ? low : bestv; }\n";
  }
  o << "    zero_fallback += (bestdeg == 0u) ? 1u : 0u;\n    return bestv;\n  }\n";
  // ---------------- minimality of |D| = qmin + 1 quorum leaves ----------------
  // With |D| = qmin + 1 every D \ {v} has qmin vertices, so it holds a quorum iff it is a
  // fixpoint itself (cpp:188-198 then finds it non-empty).  One removal-sensitivity pass
  // over the TN DAG (children first) decides all v at once: count c_t(X\{v}) = c_t(X) -
  // delta_t(v), where delta_t(v) sums v's direct multiplicity in t and the multiplicities of
  // satisfied children u with v in crit_u; crit_t = { v : delta_t(v) > c_t - thr_t }.
  // delta is kept as "at least 1 / 2 / 3" bit masks, so the pass is generated only when
  // no TN can reach delta 4 for any vertex (per-vertex bound over supports).
  {
    const uint32_t mw = f.mw, T = f.T;
    bool ok = !f.nonmonotone && f.qmin[0] > 0 && T <= 128 && mw <= 2;
    std::vector<std::vector<uint32_t>> supp(T, std::vector<uint32_t>(mw, 0));
    std::vector<std::vector<uint32_t>> childrefs(T);  // child TN per reference (with multiplicity)
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> vrefs(T);  // (word, mask) per plane
    for (uint32_t t = 0; t < T && ok; ++t) {
      if (f.flags[t] & 1u) ok = false;
      for (uint32_t w = 0; w < mw; ++w)
        if (f.vmask[(size_t)t * mw + w]) vrefs[t].push_back({w, f.vmask[(size_t)t * mw + w]});
      for (uint32_t w = 0; w < f.tw; ++w)
        for (uint32_t b = 0; b < 32; ++b)
          if ((f.cmask[(size_t)t * f.tw + w] >> b) & 1u) childrefs[t].push_back(32 * w + b);
      for (uint32_t e = f.extra_off[t]; e < f.extra_off[t + 1]; ++e) {
        const uint32_t src = f.extra_src[e], msk = f.extra_mask[e];
        if (src < mw) vrefs[t].push_back({src, msk});
        else
          for (uint32_t b = 0; b < 32; ++b)
            if ((msk >> b) & 1u) childrefs[t].push_back(32 * (src - mw) + b);
      }
      for (auto& pr : vrefs[t]) supp[t][pr.first] |= pr.second;
      for (uint32_t u : childrefs[t]) {
        if (u >= t) ok = false;  // children first
        else
          for (uint32_t w = 0; w < mw; ++w) supp[t][w] |= supp[u][w];
      }
      for (uint32_t v = 0; v < f.m && ok; ++v) {  // delta bound of vertex v at t
        const uint32_t w = v >> 5, bit = 1u << (v & 31);
        uint32_t d = 0;
        for (auto& pr : vrefs[t])
          if (pr.first == w && (pr.second & bit)) ++d;
        for (uint32_t u : childrefs[t])
          if (supp[u][w] & bit) ++d;
        if (d > 3) ok = false;
      }
    }
    o << "  static constexpr bool FASTMIN = " << (ok ? "true" : "false") << ";\n";
    o << "  static __device__ __forceinline__ void min_bad(const LocalDev&, const uint32_t (&X)[" << MW
      << "], uint32_t (&bad)[" << MW << "]) {\n";
    for (int w = 0; w < MW; ++w) o << "    bad[" << w << "] = 0u;\n";
    if (ok) {
      for (uint32_t w = 0; w < f.tw; ++w) o << "    uint32_t sb" << w << " = 0u;\n";
      for (uint32_t t = 0; t < T; ++t) {
        const int32_t th = f.thr[2 * t];
        o << "    uint32_t cr" << t << "_0 = 0u";
        for (uint32_t w = 1; w < mw; ++w) o << ", cr" << t << "_" << w << " = 0u";
        o << ";\n    {\n";
        // count as in gfp
        std::vector<std::string> terms;  // the count as in gfp: one popcount per mask word
        for (auto& pr : vrefs[t]) terms.push_back("__popc(X[" + std::to_string(pr.first) + "] & " + hex(pr.second) + ")");
        for (uint32_t w = 0; w < f.tw; ++w)
          if (f.cmask[(size_t)t * f.tw + w]) terms.push_back("__popc(sb" + std::to_string(w) + " & " + hex(f.cmask[(size_t)t * f.tw + w]) + ")");
        for (uint32_t e = f.extra_off[t]; e < f.extra_off[t + 1]; ++e)
          if (f.extra_src[e] >= mw)
            terms.push_back("__popc(sb" + std::to_string(f.extra_src[e] - mw) + " & " + hex(f.extra_mask[e]) + ")");
        std::string c = terms.empty() ? std::string("0u") : terms[0];
        for (size_t i = 1; i < terms.size(); ++i) c += " + " + terms[i];
        o << "      const uint32_t c = " << c << "; (void)c;\n";
        if (th <= 0) {
          o << "      sb" << (t / 32) << " |= 1u << " << (t % 32) << "u;\n";  // always satisfied, never critical
        } else if (th != INT32_MAX) {
          // branch-free (selects): every lane runs the same straight-line code.  The
          // "at least 2 / 3" masks are only built as far as this TN's delta bound needs.
          uint32_t dmax = 0;
          for (uint32_t v = 0; v < f.m; ++v) {
            const uint32_t w = v >> 5, bit = 1u << (v & 31);
            uint32_t d = 0;
            for (auto& pr : vrefs[t])
              if (pr.first == w && (pr.second & bit)) ++d;
            for (uint32_t u : childrefs[t])
              if (supp[u][w] & bit) ++d;
            dmax = std::max(dmax, d);
          }
          o << "      const bool s_ = c >= " << th << "u;\n      sb" << (t / 32) << " |= (uint32_t)s_ << " << (t % 32) << "u;\n";
          for (uint32_t w = 0; w < mw; ++w) o << "      uint32_t g1_" << w << " = 0u, g2_" << w << " = 0u, g3_" << w << " = 0u;\n";
          auto acc = [&](uint32_t w, const std::string& m) {
            o << "      { const uint32_t m_ = " << m << ";";
            if (dmax >= 3) o << " g3_" << w << " |= g2_" << w << " & m_;";
            if (dmax >= 2) o << " g2_" << w << " |= g1_" << w << " & m_;";
            o << " g1_" << w << " |= m_; }\n";
          };
          for (auto& pr : vrefs[t]) acc(pr.first, "X[" + std::to_string(pr.first) + "] & " + hex(pr.second));
          for (uint32_t u : childrefs[t])
            for (uint32_t w = 0; w < mw; ++w) acc(w, "cr" + std::to_string(u) + "_" + std::to_string(w));
          o << "      const uint32_t sl = c - " << th << "u;\n";
          for (uint32_t w = 0; w < mw; ++w) {
            o << "      cr" << t << "_" << w << " = s_ ? ((sl == 0u ? g1_" << w << " : ";
            if (dmax >= 2) o << "sl == 1u ? g2_" << w << " : ";
            if (dmax >= 3) o << "sl == 2u ? g3_" << w << " : ";
            o << "0u) & X[" << w << "]) : 0u;\n";
          }
        }
        o << "    }\n";
      }
      for (uint32_t r = 0; r < f.R; ++r) {
        const uint32_t tn = f.root_tn[r];
        o << "    {  // root " << r << "\n";
        std::string cnt = "0u";
        for (uint32_t w = 0; w < mw; ++w) {
          const uint32_t u = f.root_users[(size_t)r * mw + w];
          o << "      const uint32_t W" << w << " = X[" << w << "] & " << hex(u) << ";\n";
          cnt += " + __popc(W" + std::to_string(w) + ")";
        }
        o << "      const uint32_t n = " << cnt << ";\n      const bool s = (sb" << (tn / 32) << " >> " << (tn % 32)
          << "u) & 1u;\n      if (n) {\n";
        for (uint32_t w = 0; w < mw; ++w)
          o << "        bad[" << w << "] |= (s ? cr" << tn << "_" << w << " : X[" << w << "]) & ~(n == 1u ? W" << w << " : 0u);\n";
        o << "      }\n    }\n";
      }
    }
    o << "  }\n";
  }
  // the SCC mask and qmin as literals (no kernel-argument words held in SGPRs)
  o << "  static __device__ __forceinline__ uint32_t scc_word(const LocalDev&, int w) {\n    return ";
  for (int w = 0; w < MW; ++w) {
    uint32_t word = 0;
    for (uint32_t v = (uint32_t)w * 32; v < f.m && v < (uint32_t)w * 32 + 32; ++v) word |= 1u << (v & 31);
    o << (w + 1 < MW ? "w == " + std::to_string(w) + " ? " + hex(word) + " : " : hex(word));
  }
  o << ";\n  }\n";
  o << "  static __device__ __forceinline__ uint32_t qmin0(const LocalDev&) { return " << f.qmin[0] << "u; }\n};\n";
  o << "}  // namespace dev\n}  // namespace qi\n\n";
  o << "extern \"C\" __global__ __launch_bounds__(64) void qi_search_spec(qi::dev::SearchArgs a) {\n"
    << "  qi::dev::search_body<" << MW << ", " << TW << ", " << SMAX << ", qi::dev::SpecEval, " << (tie_random ? "true" : "false")
    << ">(a);\n}\n";
  return o.str();
}

std::string cache_path(const std::string& src) {
  char key[32];
  const char* xf = std::getenv("QI_JIT_FLAGS");
  std::snprintf(key, sizeof key, "%016llx", (unsigned long long)fnv1a(src + "|gfx950|-O3|v4|" + (xf ? xf : "")));
  return cache_dir() + "/" + key + ".co";
}

// A cache entry is the code object followed by an 16-byte trailer: "QICO" + its length +
// an FNV-1a hash of its bytes.  A file without a matching trailer (partly written, left by
// a crashed process, older format) is ignored and overwritten by the next compile.
std::vector<char> jit_cached(const std::string& src) {
  std::ifstream in(cache_path(src), std::ios::binary);
  if (!in) return {};
  std::vector<char> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (buf.size() < 16) return {};
  const size_t n = buf.size() - 16;
  uint32_t len = 0;
  uint64_t h = 0;
  std::memcpy(&len, &buf[n + 4], 4);
  std::memcpy(&h, &buf[n + 8], 8);
  if (std::memcmp(&buf[n], "QICO", 4) != 0 || len != n || h != fnv1a(std::string(buf.data(), n))) return {};
  buf.resize(n);
  return buf;
}

std::vector<char> jit_compile(const std::string& src, std::string* log) {
  if (const char* d = std::getenv("QI_JIT_DUMP")) {  // diagnostics: keep the generated source
    std::ofstream(d) << src;
  }
  const std::string dir = cache_dir();
  const std::string path = cache_path(src);
  {
    std::vector<char> code = jit_cached(src);
    if (!code.empty()) return code;
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "qi_search_spec.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    if (log) *log = "hiprtcCreateProgram failed";
    return {};
  }
  // the atomic optimizer rewrites every lane-0 atomic into a wave scan with an immediate
  // wait for its result; the kernel's lane-0 atomics are consumed an iteration later
  std::vector<std::string> optv = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-pragma-once-outside-header",
                                   "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
                                   // no packed FP32 VALU ops in device code (integer-only kernels)
                                   "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"};
  if (const char* e = std::getenv("QI_JIT_FLAGS")) {  // diagnostics: extra compiler flags (space separated)
    std::istringstream is(e);
    std::string t;
    while (is >> t) optv.push_back(t);
  }
  std::vector<const char*> opts;
  for (auto& o : optv) opts.push_back(o.c_str());
  const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  size_t n = 0;
  hiprtcGetProgramLogSize(prog, &n);
  std::string lg(n, '\0');
  if (n) hiprtcGetProgramLog(prog, &lg[0]);
  if (log) *log = lg;
  std::vector<char> code;
  if (rc == HIPRTC_SUCCESS) {
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.resize(cs);
    hiprtcGetCode(prog, code.data());
    ::mkdir(dir.c_str(), 0755);
    // unique per process AND thread (sharded solves compile on several threads at once)
    static std::atomic<uint32_t> seq{0};
    const std::string tmp = path + ".tmp" + std::to_string(::getpid()) + "." + std::to_string(seq.fetch_add(1));
    {
      std::ofstream out(tmp, std::ios::binary);
      out.write(code.data(), (std::streamsize)code.size());
      const uint32_t len = (uint32_t)code.size();
      const uint64_t h = fnv1a(std::string(code.data(), code.size()));
      out.write("QICO", 4);
      out.write((const char*)&len, 4);
      out.write((const char*)&h, 8);
    }
    std::rename(tmp.c_str(), path.c_str());
  }
  hiprtcDestroyProgram(&prog);
  return code;
}

}  // namespace qi
