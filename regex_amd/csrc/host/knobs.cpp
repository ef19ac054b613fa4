// The debug override table of knobs.hpp.
#include "knobs.hpp"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

namespace rure_amd {

namespace {

constexpr int kN = (int)Knob::kCount;

// names in Knob order
const char *const kNames[kN] = {
    "lit",        "sa",          "lex",        "lex4",       "lex_tail",   "kmer",       "runs",
    "ascii_shadow", "fb",        "prefix",     "big",        "big_bytes",  "lazy",       "lazy_rows",
    "lines",      "split",       "suffix_long", "suffix_iter", "iter_looks", "iter_chunk", "iter_lanes",
    "iter_bs",    "long_lanes",  "core_bs",    "core_lds",   "core_prof",  "scratch_cap", "timing",
    "replace_generic", "chain_seq", "shadow_sync", "iter_wave", "wave_cu", "wave_split", "wave_tables", "wave_lds",
};

std::atomic<long long> g_val[kN];
std::once_flag g_once;
std::mutex g_mu;

bool parse(const char *spec, long long *out) {
  for (int i = 0; i < kN; ++i) out[i] = -1;
  if (!spec) return true;
  std::string s(spec);
  size_t at = 0;
  while (at < s.size()) {
    size_t end = s.find(',', at);
    if (end == std::string::npos) end = s.size();
    const std::string item = s.substr(at, end - at);
    at = end + 1;
    if (item.empty()) continue;
    const size_t eq = item.find('=');
    if (eq == std::string::npos) return false;
    const std::string name = item.substr(0, eq), val = item.substr(eq + 1);
    int k = -1;
    for (int i = 0; i < kN; ++i)
      if (name == kNames[i]) k = i;
    char *e = nullptr;
    const long long v = strtoll(val.c_str(), &e, 10);
    if (k < 0 || val.empty() || *e || v < 0) return false;
    out[k] = v;
  }
  return true;
}

void store(const long long *v) {
  for (int i = 0; i < kN; ++i) g_val[i].store(v[i], std::memory_order_relaxed);
}

void init_once() {
  long long v[kN];
  const char *env = getenv("RURE_AMD_DEBUG");
  if (!parse(env, v)) {
    fprintf(stderr, "rure_amd: RURE_AMD_DEBUG=\"%s\" ignored (name=value,... of known knobs)\n", env);
    parse(nullptr, v);
  }
  store(v);
}

}  // namespace

long long knob(Knob k) {
  std::call_once(g_once, init_once);
  return g_val[(int)k].load(std::memory_order_relaxed);
}

bool knob_set(const char *spec) {
  std::call_once(g_once, init_once);
  long long v[kN];
  if (!parse(spec, v)) return false;
  std::lock_guard<std::mutex> g(g_mu);
  store(v);
  return true;
}

}  // namespace rure_amd
