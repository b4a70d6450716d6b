// `quorum_intersection` drop-in executable: the reference's main() (cpp:744-800) over the
// C-ABI.  Options follow boost::program_options' unix style as the reference configures
// it (cpp:755-765): short and long forms, "-i 5" / "-i5" / "--max_iterations=5",
// sticky short switches ("-vg"), unique long-option prefixes; anything else prints
// "Invalid option!" and the option table and exits 1.
//
// Multi-GPU and diagnostics come from the environment, so the option table stays the
// reference's:
//   QI_DEVICES = all | 0,2,5 | 0-7   GPUs of the search (default: device 0); the search
//                                    tree is sharded by branch prefix over them
//   QI_ENGINES = N                   search shards (default: one per device; N > 1 on one
//                                    device runs the same sharded path on one GPU)
//   QI_TIMING  = 1                   one JSON line on stderr: device init, then stdin to
//                                    verdict (parse + SCCs + checks + search) apart
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "../../include/quorum_intersection.h"

namespace {

const char* kHelp =
    "Allowed options:\n"
    "  -h [ --help ]                 print usage message\n"
    "  -v [ --verbose ]              print more details\n"
    "  -g [ --graph ]                print graphviz representation of network's \n"
    "                                configuration\n"
    "  -t [ --trace ]                enable tracing messages\n"
    "  -p [ --pagerank ]             compute the PageRank for the network\n"
    "  -i [ --max_iterations ] arg   maximal number of iterations for the PageRank \n"
    "                                algorithm\n"
    "  -m [ --dangling_factor ] arg  dangling factor parameter of the PageRank \n"
    "                                algorithm\n"
    "  -c [ --convergence ] arg      convergence parameter of the PageRank algorithm\n";

struct Opt {
  char s;
  const char* l;
  bool value;
};
const Opt kOpts[] = {{'h', "help", false},     {'v', "verbose", false}, {'g', "graph", false},
                     {'t', "trace", false},    {'p', "pagerank", false}, {'i', "max_iterations", true},
                     {'m', "dangling_factor", true}, {'c', "convergence", true}};

struct Parsed {
  bool help = false, verbose = false, graph = false, trace = false, pagerank = false;
  uint64_t max_iterations = 100000;
  float dangling = 0.0001f, convergence = 0.0001f;
};

bool parse_u64(const std::string& s, uint64_t* out) {
  if (s.empty() || s[0] == '-') return false;
  char* e = nullptr;
  errno = 0;
  unsigned long long v = std::strtoull(s.c_str(), &e, 10);
  if (errno || *e) return false;
  *out = v;
  return true;
}

bool parse_float(const std::string& s, float* out) {
  if (s.empty()) return false;
  char* e = nullptr;
  errno = 0;
  float v = std::strtof(s.c_str(), &e);
  if (errno || *e) return false;
  *out = v;
  return true;
}

bool apply(Parsed& p, const Opt& o, const std::string* val, std::vector<int>& seen) {
  int idx = (int)(&o - kOpts);
  if (o.value) {
    if (seen[idx]++) return false;  // multiple occurrences of a value option
    if (!val) return false;
    switch (o.s) {
      case 'i': return parse_u64(*val, &p.max_iterations);
      case 'm': return parse_float(*val, &p.dangling);
      case 'c': return parse_float(*val, &p.convergence);
    }
    return false;
  }
  if (val) return false;
  switch (o.s) {
    case 'h': p.help = true; break;
    case 'v': p.verbose = true; break;
    case 'g': p.graph = true; break;
    case 't': p.trace = true; break;
    case 'p': p.pagerank = true; break;
  }
  return true;
}

bool parse_args(int argc, char** argv, Parsed& p) {
  std::vector<int> seen(sizeof kOpts / sizeof kOpts[0], 0);
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
      std::string name = a.substr(2), val;
      bool has_val = false;
      size_t eq = name.find('=');
      if (eq != std::string::npos) {
        val = name.substr(eq + 1);
        name = name.substr(0, eq);
        has_val = true;
      }
      const Opt* hit = nullptr;
      int matches = 0;
      for (const auto& o : kOpts) {
        if (name == o.l) { hit = &o; matches = 1; break; }
        if (std::strncmp(o.l, name.c_str(), name.size()) == 0) { hit = &o; ++matches; }
      }
      if (!hit || matches != 1) return false;
      if (hit->value && !has_val) {
        if (i + 1 >= argc) return false;
        val = argv[++i];
        has_val = true;
      }
      if (!apply(p, *hit, has_val ? &val : nullptr, seen)) return false;
    } else if (a.size() >= 2 && a[0] == '-' && a[1] != '-') {
      for (size_t k = 1; k < a.size(); ++k) {
        const Opt* hit = nullptr;
        for (const auto& o : kOpts)
          if (o.s == a[k]) hit = &o;
        if (!hit) return false;
        if (hit->value) {
          std::string val = a.substr(k + 1);
          if (val.empty()) {
            if (i + 1 >= argc) return false;
            val = argv[++i];
          }
          if (!apply(p, *hit, &val, seen)) return false;
          break;
        }
        if (!apply(p, *hit, nullptr, seen)) return false;
      }
    } else {
      return false;  // no positional options are declared
    }
  }
  return true;
}

// QI_DEVICES -> device mask; returns false on a malformed value
bool parse_devices(const char* s, int ndev, uint32_t* mask) {
  *mask = 0;
  std::string v = s;
  if (v == "all") {
    for (int d = 0; d < ndev && d < 32; ++d) *mask |= 1u << d;
    return *mask != 0;
  }
  size_t p = 0;
  while (p < v.size()) {
    size_t q = v.find(',', p);
    if (q == std::string::npos) q = v.size();
    const std::string item = v.substr(p, q - p);
    const size_t dash = item.find('-');
    uint64_t a = 0, b = 0;
    if (dash == std::string::npos) {
      if (!parse_u64(item, &a)) return false;
      b = a;
    } else if (!parse_u64(item.substr(0, dash), &a) || !parse_u64(item.substr(dash + 1), &b) || b < a) {
      return false;
    }
    if (b >= 32) return false;
    for (uint64_t d = a; d <= b; ++d) *mask |= 1u << d;
    p = q + 1;
  }
  return *mask != 0;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

[[noreturn]] void die_parse(const char* what) {
  // the reference leaves the ptree_error uncaught: std::terminate -> SIGABRT
  std::cerr << "terminate called after throwing an instance of "
               "'boost::wrapexcept<boost::property_tree::ptree_error>'\n  what():  "
            << what << std::endl;
  std::abort();
}

}  // namespace

int main(int argc, char** argv) {
  Parsed p;
  if (!parse_args(argc, argv, p)) {
    std::cout << "Invalid option!" << std::endl;
    std::cout << kHelp;
    return EXIT_FAILURE;
  }
  if (p.help) {
    std::cout << kHelp << std::endl;
    return EXIT_SUCCESS;
  }
  const bool timing = std::getenv("QI_TIMING") != nullptr;
  qi_solve_opts opts;
  std::memset(&opts, 0, sizeof opts);
  opts.jit = 4;  // the specialised kernel only from the on-disk cache: no compile before the verdict
  int device = 0;
  if (const char* e = std::getenv("QI_DEVICES")) {
    if (!parse_devices(e, qi_device_count(), &opts.device_mask)) {
      std::cerr << "quorum_intersection: bad QI_DEVICES value '" << e << "'" << std::endl;
      return 3;
    }
    while (!((opts.device_mask >> device) & 1u)) ++device;  // per-SCC checks on the first
  }
  if (const char* e = std::getenv("QI_ENGINES")) {
    uint64_t n = 0;
    if (!parse_u64(e, &n) || n == 0 || n > 64) {
      std::cerr << "quorum_intersection: bad QI_ENGINES value '" << e << "'" << std::endl;
      return 3;
    }
    opts.engines = (uint32_t)n;
  }
  double init_ms = 0;
  if (timing && !p.pagerank) {  // HIP runtime + device context, reported apart
    if (qi_device_warmup(device, &init_ms) != QI_OK) {
      std::cerr << "quorum_intersection: " << qi_last_error() << std::endl;
      return 3;
    }
  }
  const auto t0 = std::chrono::steady_clock::now();  // stdin open -> verdict printed
  std::string in;  // all of stdin in large reads (a char-by-char istream copy took 25 ms per 500 KB)
  {
    char buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof buf, stdin)) > 0) in.append(buf, got);
  }
  const double read_ms = ms_since(t0);
  qi_fbas* f = nullptr;
  int rc = qi_fbas_from_json(in.data(), in.size(), device, &f);
  if (rc == QI_ERR_PARSE) die_parse(qi_last_error());
  if (rc != QI_OK) {
    std::cerr << "quorum_intersection: " << qi_last_error() << std::endl;
    return 3;
  }
  char* text = nullptr;
  if (p.pagerank) {
    rc = qi_pagerank_text(f, p.dangling, p.convergence, p.max_iterations, &text);
    if (rc != QI_OK) {
      std::cerr << "quorum_intersection: " << qi_last_error() << std::endl;
      return 3;
    }
    std::cout << text;
    qi_free(text);
    qi_fbas_destroy(f);
    return EXIT_SUCCESS;
  }
  int verdict = 0;
  const double parse_ms = ms_since(t0);
  rc = qi_solve_text_ex(f, p.verbose ? 1 : 0, p.graph ? 1 : 0, &opts, &text, &verdict);
  if (rc != QI_OK) {
    std::cerr << "quorum_intersection: " << qi_last_error() << std::endl;
    return 3;
  }
  const auto t_out = std::chrono::steady_clock::now();
  std::cout << text << std::flush;
  const double verdict_ms = ms_since(t0);
  const double text_ms = ms_since(t_out);
  qi_free(text);
  // After the verdict is out (printed and flushed): put the searched SCC's specialised kernel
  // into the on-disk cache (a no-op when it is there), so the next run of this network starts
  // with it.  The compile (~1 s) delays only the exit status of the first run on a network;
  // QI_NO_JIT_FILL=1 skips it.
  if (!std::getenv("QI_NO_JIT_FILL")) {
    const uint32_t n = qi_fbas_num_vertices(f);
    std::vector<uint32_t> comp(n ? n : 1);
    uint32_t front = 0;
    if (n && qi_fbas_scc_ids(f, comp.data()) == QI_OK)
      for (uint32_t v = 0; v < n; ++v) front += comp[v] == 0 ? 1u : 0u;
    if (front >= 8) (void)qi_fbas_jit_precompile(f, nullptr);
  }
  if (timing)
    std::fprintf(stderr,
                 "{\"device_init_ms\": %.3f, \"stdin_to_verdict_ms\": %.3f, \"read_parse_graph_ms\": %.3f, "
                 "\"read_stdin_ms\": %.3f, \"print_ms\": %.3f, \"devices_mask\": %u, \"engines\": %u, \"phases\": %s}\n",
                 init_ms, verdict_ms, parse_ms, read_ms, text_ms, opts.device_mask, opts.engines, qi_timing_json());
  qi_fbas_destroy(f);
  return verdict ? EXIT_SUCCESS : EXIT_FAILURE;
}
