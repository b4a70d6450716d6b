// `quorum_intersection` drop-in executable: the reference's main() (cpp:744-800) over the
// C-ABI.  Options follow boost::program_options' unix style as the reference configures
// it (cpp:755-765): short and long forms, "-i 5" / "-i5" / "--max_iterations=5",
// sticky short switches ("-vg"), unique long-option prefixes; anything else prints
// "Invalid option!" and the option table and exits 1.
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
  std::string in((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
  qi_fbas* f = nullptr;
  int rc = qi_fbas_from_json(in.data(), in.size(), 0, &f);
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
  rc = qi_solve_text(f, p.verbose ? 1 : 0, p.graph ? 1 : 0, &text, &verdict);
  if (rc != QI_OK) {
    std::cerr << "quorum_intersection: " << qi_last_error() << std::endl;
    return 3;
  }
  std::cout << text;
  qi_free(text);
  qi_fbas_destroy(f);
  return verdict ? EXIT_SUCCESS : EXIT_FAILURE;
}
