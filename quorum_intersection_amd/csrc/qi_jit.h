// Run-time specialisation of the search kernel (see qi_jit.cpp).
#pragma once

#include <string>
#include <vector>

#include "qi_internal.h"

namespace qi {

// Whether a generated evaluator stays a reasonable size for this SCC.
bool jit_eligible(const LocalFlat& f);
// LDS words of D order per lane in the specialised kernel (QI_LDS_OW): |D| <= m/2 + 1
uint32_t jit_lds_ow(const LocalFlat& f);
// Full hipRTC source: qi_search_kernel.h + generated SpecEval + extern "C" qi_search_spec.
std::string jit_source(const LocalFlat& f, int MW, int TW, int SMAX, bool stamps = false, bool tie_random = false);
// Compile for gfx950 (or read the on-disk cache); empty on failure, log in *log.
std::vector<char> jit_compile(const std::string& src, std::string* log);
// The code object from the on-disk cache only (no compile); empty when absent.
std::vector<char> jit_cached(const std::string& src);

}  // namespace qi
