// rure_amd: C ABI (include/rure_amd.h) over the host compiler + HIP kernels.
//
// Mirrors the reference C API regex-capi/src/rure.rs (compile 95-150,
// is_match 158-168, find 170-187, shortest_match 207-224, iter 308-360,
// options 13-19/67-74, set 470-572, errors regex-capi/src/error.rs) and the
// engine construction of src/exec.rs:273-327 (three programs per regex: NFA,
// forward DFA with `.*?`, reverse DFA).  All matching runs on the GPU.
#include "../../include/rure_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "host/dfa_build.hpp"
#include "host/nfa_build.hpp"
#include "host/literals.hpp"
#include "host/literal_sets.hpp"
#include "host/program.hpp"
#include "host/syntax.hpp"
#include "host/unicode_tables.h"
#include "kernels/dfa_scan.hpp"

using namespace rure_amd;

struct rure_error {
  std::string msg;
};

struct rure_options {
  size_t size_limit = 10u << 20;       // rure.rs:67-74, re_builder.rs:30-31
  size_t dfa_size_limit = 2u << 20;
};

namespace {

[[noreturn]] void die(const std::string &m) {
  fprintf(stderr, "rure_amd: %s\n", m.c_str());
  fprintf(stderr, "aborting\n");
  abort();
}

bool hip_ok(hipError_t e, std::string *err) {
  if (e == hipSuccess) return true;
  if (err) *err = std::string("HIP error: ") + hipGetErrorString(e);
  return false;
}

// Device copy of the automata of one regex on one device.
struct DevTables {
  void *blob = nullptr;
  FwdDfaDev f{};
  RevDfaDev r{};
  SetDfaDev s{};
  NfaDev n{};
  SetCoreDev c{};
  bool use_cores = false;   // sets: core-form kernel
  bool cores_adapted = false;
  void *core_blob = nullptr;  // re-ranked core tables (adapt_cores)
  bool has_dfa = false;     // the DFA materialised (else: Pike VM only)
  bool has_big = false;     // big (u32) forward / reverse automata: bf, br
  bool big_tried = false;   // big automata built (lazily, big_device) or found not to build
  void *big_blob = nullptr; // their device copy
  struct rure *owner = nullptr;  // the regex (big_device builds its automata on first need)
  BigDfaDev bf{}, br{};
  bool quit_possible = false;  // the DFA can quit (Unicode \b): Pike VM fallback pass
  bool anchored_rev = false;   // MatchType::DfaAnchoredReverse (exec.rs:1175-1177)
  // The reference's match type where its searches differ from a forward DFA
  // search (literal_sets.hpp): Literal(AnchoredStart), Literal(Unanchored)
  // chosen from complete suffixes (its prefix searcher may be Empty or
  // partial), DfaSuffix.  Those searches run match_types.hip / the wave
  // iteration with `m`.
  MatchDev m{-1, {}, {}, nullptr, 0};
  bool mt_lane = false;
  int cus = 256;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Packs a materialized forward (or set) DFA into the LDS image / full table.
struct PackedFwd {
  std::vector<uint8_t> lds;
  std::vector<uint8_t> lds_s;   // multi-byte (stride 2/4) fast table image, empty if stride 1
  uint32_t stride = 1, hot_s = 0, P = 1, sent = 0;
  std::vector<uint16_t> full;
  std::vector<uint8_t> eof;
  std::vector<uint64_t> eof_mask;
  std::vector<uint64_t> now_mask;
  std::vector<uint16_t> start;
  uint32_t hot = 0;
  uint32_t all = 0;       // the LDS rows are exact for every state (hot = nstates)
  uint32_t ustart1 = 0;   // 1 + the start state if every reachable flag set gives the same one
};

// 1 + the start state when all start flags a search can present (dfa.rs:
// 1415-1464: text start / empty text / line start / word before / word
// after, in the index layout of fwd_flag_index) map to one state — always
// so without look-around assertions; 0 otherwise.
uint32_t uniform_start(const DenseDfa &d) {
  int found = -1;
  for (int st = 0; st < 2; ++st)
    for (int en = 0; en < 2; ++en)
      for (int nl = 0; nl < 2; ++nl)
        for (int wl = 0; wl < 2; ++wl)
          for (int wn = 0; wn < 2; ++wn) {
            if (st && (wl || !nl)) continue;  // no byte before the text start
            if (nl && wl) continue;           // '\n' is not a word byte
            if (en && (wn || !st)) continue;  // empty text: no byte after, start == end
            const int idx = (st ? 1 : 0) | (en ? 2 : 0) | (nl ? 4 : 0) | (en ? 8 : 0) | (wl != wn ? 16 : 32) |
                            (wl ? 64 : 0);
            const int v = (int)d.start[idx];
            if (found < 0) found = v;
            else if (found != v) return 0;
          }
  return found < 0 ? 0 : (uint32_t)found + 1;
}

// Multi-byte fast table over the ASCII-hot sub-DFA (states [0, A)): bytes
// are grouped into K local classes (identical columns over the hot states,
// non-hot targets folded into the sentinel A); if K^stride is small the
// table maps (state, class_1..class_stride) -> next state in one lookup.
void build_stride_image(const DenseDfa &d, PackedFwd *p) {
  const int A = std::min(std::min(d.n_ascii, d.n_normal), 255);
  p->stride = 1;
  if (A <= 0) return;
  std::vector<int> cls(256, -1);
  std::vector<int> rep;
  std::map<std::vector<uint16_t>, int> seen;
  for (int b = 0; b < 256; ++b) {
    std::vector<uint16_t> col(A);
    for (int s = 0; s < A; ++s) {
      uint32_t t = d.trans[(size_t)s * 256 + b];
      col[s] = (uint16_t)(t < (uint32_t)A ? t : A);
    }
    auto it = seen.find(col);
    if (it == seen.end()) { it = seen.emplace(col, (int)rep.size()).first; rep.push_back(b); }
    cls[b] = it->second;
  }
  const int K = (int)rep.size();
  int stride = 1;
  const long budget = (16384 - 1024) / 2;  // u16 entries after the 1 KiB class tables
  if (K <= 4 && (long)(A + 1) * K * K * K * K <= budget) stride = 4;
  else if (K <= 16 && (long)(A + 1) * K * K <= budget) stride = 2;
  if (stride == 1) return;
  uint32_t P = 1;
  for (int i = 0; i < stride; ++i) P *= (uint32_t)K;
  std::vector<uint8_t> img(1024, 0);
  for (int pos = 0; pos < stride; ++pos) {
    uint32_t mul = 1;
    for (int i = pos + 1; i < stride; ++i) mul *= (uint32_t)K;
    for (int b = 0; b < 256; ++b) img[pos * 256 + b] = (uint8_t)(cls[b] * mul);
  }
  const size_t nent = (size_t)(A + 1) * P;
  std::vector<uint16_t> tab(nent);
  for (int s = 0; s <= A; ++s) {
    for (uint32_t combo = 0; combo < P; ++combo) {
      uint32_t t = (uint32_t)s;
      uint32_t c = combo, div = P / (uint32_t)K;
      for (int pos = 0; pos < stride; ++pos) {
        int k = (int)(c / div);
        c %= div;
        if (div > 1) div /= (uint32_t)K;
        if (t < (uint32_t)A) {
          uint32_t nx = d.trans[(size_t)t * 256 + rep[k]];
          t = nx < (uint32_t)A ? nx : (uint32_t)A;
        }
      }
      tab[(size_t)s * P + combo] = (uint16_t)(t * P);
    }
  }
  img.resize(1024 + nent * 2);
  memcpy(img.data() + 1024, tab.data(), nent * 2);
  img.resize((img.size() + 15) & ~(size_t)15, 0);
  p->lds_s = std::move(img);
  p->stride = (uint32_t)stride;
  p->hot_s = (uint32_t)A;
  p->P = P;
  p->sent = (uint32_t)A * P;
}

bool pack_forward(const DenseDfa &d, PackedFwd *p, std::string *err, bool all = false) {
  if (d.nstates > 65535) {
    if (err) *err = "DFA has too many states for u16 tables";
    return false;
  }
  p->ustart1 = uniform_start(d);
  if (all && d.nstates <= 255) {
    // small automata (find_iter / reverse scans): every state's exact row in
    // LDS, so match, dead and restart steps never touch the global table
    p->all = 1;
    p->hot = (uint32_t)d.nstates;
    p->lds.assign(((size_t)d.nstates * kRow + 15) & ~(size_t)15, 0);
    for (int st = 0; st < d.nstates; ++st)
      for (int b = 0; b < 256; ++b) p->lds[(size_t)st * kRow + b] = (uint8_t)d.trans[(size_t)st * 256 + b];
    p->full.resize((size_t)d.nstates * 256);
    for (size_t i = 0; i < p->full.size(); ++i) p->full[i] = (uint16_t)d.trans[i];
    p->eof.assign(d.eof_match.begin(), d.eof_match.end());
    p->start.resize(128);
    for (int i = 0; i < 128; ++i) p->start[i] = (uint16_t)d.start[i];
    return true;
  }
  // LDS fast table: the normal states reachable through ASCII bytes are
  // numbered first; hold them plus further BFS-order states in the smallest
  // of three table sizes (4 KiB / 16 KiB / 64 KiB) that fits the ASCII set,
  // so that several workgroups stay resident per CU.
  int need = std::min(d.n_ascii, d.n_normal);
  int cap = need + 1 <= 16 ? 15 : need + 1 <= 64 ? 63 : 255;
  uint32_t hot = (uint32_t)std::min(d.n_normal, cap);
  p->hot = hot;
  size_t lds_bytes = ((size_t)(hot + 1) * kRow + 15) & ~(size_t)15;
  p->lds.assign(lds_bytes, 0);
  for (uint32_t s = 0; s <= hot; ++s) {
    for (int b = 0; b < 256; ++b) {
      uint32_t t = (s < hot) ? d.trans[(size_t)s * 256 + b] : hot;
      p->lds[(size_t)s * kRow + b] = (uint8_t)(t < hot ? t : hot);
    }
    // column 256 (row padding): the identity, for the bytes outside a masked
    // head / tail block of the line kernel (dfa_line_kernel)
    p->lds[(size_t)s * kRow + kIdCol] = (uint8_t)s;
  }
  build_stride_image(d, p);
  p->full.resize((size_t)d.nstates * 256);
  for (size_t i = 0; i < p->full.size(); ++i) p->full[i] = (uint16_t)d.trans[i];
  p->eof.assign(d.eof_match.begin(), d.eof_match.end());
  p->eof_mask.assign(d.eof_mask.begin(), d.eof_mask.end());
  p->now_mask.assign(d.now_mask.begin(), d.now_mask.end());
  p->start.resize(128);
  for (int i = 0; i < 128; ++i) p->start[i] = (uint16_t)d.start[i];
  return true;
}

// Core form of a set DFA (kernel: set_core_kernel).  States whose rows and
// EOF masks agree differ only in the matches their entry reports; they share
// a core, and the report moves onto the transition (an output code).  Cores
// are numbered in BFS order over ASCII bytes from the start states; the first
// `hot` (as many as fit the LDS budget, at most 1023) are held in LDS.
struct CoreSet {
  bool ok = false;
  uint32_t K = 0, ncores = 0, hot = 0, dead = 0, quit = 0xFFFFFFFFu;
  std::vector<uint8_t> lds;       // class map (256 B), then (hot + 1) x K u16 entries
  std::vector<uint16_t> gcore;    // ncores x K
  std::vector<uint64_t> gout;     // ncores x K
  std::vector<uint64_t> eof;      // ncores
  uint16_t start[128];
  std::vector<uint32_t> order;    // rank -> core (in first-appearance numbering)
  bool profiled = false;
  // output codes: code c in 1..62 reports codemask[c] (the table is in the
  // LDS image at mt_off); 63 = look the mask up in gout.  mid (ncores x K)
  // = 1 + the index of gout's mask in `masks` (0: none), for the profile.
  uint64_t codemask[64] = {0};
  uint32_t mt_off = 0;
  uint64_t hot_visits = 0;        // with visit weights: the visits to the hot cores
  std::vector<uint64_t> masks;
  std::vector<uint16_t> mid;
};

// LDS budget of the core table (RURE_AMD_CORE_LDS overrides, tuning).
size_t core_lds_budget() {
  size_t b = 150 * 1024;
  if (const char *v = getenv("RURE_AMD_CORE_LDS")) b = std::max<size_t>(4096, std::min<size_t>(150 * 1024, atol(v)));
  return b;
}

// weights (optional, by core in first-appearance numbering): rank the cores
// by decreasing weight (measured visits), ties in BFS order.
// mask_weights: how often each reported mask occurred on a sample (the
// profile of adapt_cores); the 62 most frequent masks get the LDS codes.
// Without it, masks rank by the number of hot transitions reporting them.
bool build_set_cores(const DenseDfa &d, size_t lds_budget, CoreSet *cs,
                     const std::vector<uint64_t> *weights = nullptr,
                     const std::unordered_map<uint64_t, uint64_t> *mask_weights = nullptr,
                     const std::vector<uint64_t> *state_weights = nullptr) {
  const int S = d.nstates;
  std::unordered_map<std::string, uint32_t> key_core;
  std::vector<uint32_t> core_of(S);
  std::vector<int> rep;
  for (int s = 0; s < S; ++s) {
    std::string k((const char *)&d.trans[(size_t)s * 256], 256 * 4);
    k.append((const char *)&d.eof_mask[s], 8);
    auto it = key_core.emplace(k, (uint32_t)rep.size());
    if (it.second) rep.push_back(s);
    core_of[s] = it.first->second;
  }
  const uint32_t nc = (uint32_t)rep.size();
  if (nc >= 65535) return false;
  // BFS order over ASCII bytes from the start cores, then everything else
  std::vector<int32_t> rank(nc, -1);
  std::vector<uint32_t> order;
  std::deque<uint32_t> dq;
  auto push = [&](uint32_t c) { if (rank[c] < 0) { rank[c] = (int32_t)order.size(); order.push_back(c); dq.push_back(c); } };
  for (int i = 0; i < 128; ++i) push(core_of[d.start[i]]);
  while (!dq.empty()) {
    uint32_t c = dq.front(); dq.pop_front();
    for (int b = 0; b < 128; ++b) push(core_of[d.trans[(size_t)rep[c] * 256 + b]]);
  }
  for (uint32_t c = 0; c < nc; ++c) push(c);
  std::vector<uint64_t> sw;
  if (!weights && state_weights) {  // per-state visit counts summed per core
    sw.assign(nc, 0);
    for (int s2 = 0; s2 < S; ++s2) sw[core_of[s2]] += (*state_weights)[s2];
    weights = &sw;
  }
  if (weights) {
    std::vector<uint32_t> bfs = order;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b2) { return (*weights)[a] > (*weights)[b2]; });
    for (uint32_t r = 0; r < nc; ++r) rank[order[r]] = (int32_t)r;
    (void)bfs;
  }
  // byte classes: identical (next core, output) columns over all cores
  std::unordered_map<std::string, uint32_t> col_id;
  uint8_t cls[256];
  std::vector<int> col_rep;
  for (int b = 0; b < 256; ++b) {
    std::string k;
    k.reserve(nc * 12);
    for (uint32_t r = 0; r < nc; ++r) {
      const uint32_t nxt = d.trans[(size_t)rep[order[r]] * 256 + b];
      const uint32_t ncore = (uint32_t)rank[core_of[nxt]];
      k.append((const char *)&ncore, 4);
      k.append((const char *)&d.now_mask[nxt], 8);
    }
    auto it = col_id.emplace(k, (uint32_t)col_rep.size());
    if (it.second) col_rep.push_back(b);
    if (it.first->second > 255) return false;
    cls[b] = (uint8_t)it.first->second;
  }
  const uint32_t K = (uint32_t)col_rep.size();
  if (K > 127) return false;  // the kernel's LDS class map holds 2k in a byte
  if (lds_budget < 256 + 64 * 8 + 16 + 4 * (K + 1)) return false;
  // LDS rows have K + 1 entries: column K is the identity (same core, no
  // output), the class of the bytes outside a masked head / tail chunk
  const uint32_t KL = K + 1;
  // (the image: class map, (hot + 1) rows, the 64 code masks)
  uint32_t hot = (uint32_t)std::min<size_t>({(size_t)nc, 1023, (lds_budget - 256 - 64 * 8 - 16) / (2 * KL) - 1});
  cs->hot_visits = 0;
  if (weights)
    for (uint32_t r = 0; r < hot; ++r) cs->hot_visits += (*weights)[order[r]];
  cs->K = K;
  cs->ncores = nc;
  cs->hot = hot;
  cs->gcore.assign((size_t)nc * K, 0);
  cs->gout.assign((size_t)nc * K, 0);
  cs->eof.assign(nc, 0);
  cs->mid.assign((size_t)nc * K, 0);
  cs->masks.clear();
  std::unordered_map<uint64_t, uint32_t> mask_idx;
  std::unordered_map<uint64_t, uint64_t> hot_uses;
  for (uint32_t r = 0; r < nc; ++r) {
    const int s = rep[order[r]];
    cs->eof[r] = d.eof_mask[s];
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t nxt = d.trans[(size_t)s * 256 + col_rep[k]];
      const uint64_t out = d.now_mask[nxt];
      cs->gcore[(size_t)r * K + k] = (uint16_t)rank[core_of[nxt]];
      cs->gout[(size_t)r * K + k] = out;
      if (!out) continue;
      auto it = mask_idx.emplace(out, (uint32_t)cs->masks.size());
      if (it.second) cs->masks.push_back(out);
      if (cs->masks.size() >= 65535) return false;
      cs->mid[(size_t)r * K + k] = (uint16_t)(it.first->second + 1);
      if (r < hot) ++hot_uses[out];
    }
  }
  // output codes 1..62 for the most frequent masks (measured when profiled)
  std::vector<uint64_t> ranked = cs->masks;
  auto weight = [&](uint64_t m) -> uint64_t {
    if (mask_weights) {
      auto it = mask_weights->find(m);
      return it == mask_weights->end() ? 0 : it->second;
    }
    auto it = hot_uses.find(m);
    return it == hot_uses.end() ? 0 : it->second;
  };
  std::stable_sort(ranked.begin(), ranked.end(), [&](uint64_t a, uint64_t b2) { return weight(a) > weight(b2); });
  std::unordered_map<uint64_t, uint32_t> code_of;
  memset(cs->codemask, 0, sizeof(cs->codemask));
  for (uint32_t i = 0; i < ranked.size() && i < 62; ++i) {
    code_of[ranked[i]] = i + 1;
    cs->codemask[i + 1] = ranked[i];
  }
  const size_t t_end = 256 + (size_t)(hot + 1) * KL * 2;
  cs->mt_off = (uint32_t)((t_end + 7) & ~(size_t)7);
  cs->lds.assign(cs->mt_off + 64 * 8, 0);
  memcpy(cs->lds.data(), cls, 256);
  memcpy(cs->lds.data() + cs->mt_off, cs->codemask, 64 * 8);
  uint16_t *T = (uint16_t *)(cs->lds.data() + 256);
  for (uint32_t r = 0; r < hot; ++r) {
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t ncore = cs->gcore[(size_t)r * K + k];
      const uint64_t out = cs->gout[(size_t)r * K + k];
      uint32_t code = 0;
      if (out) {
        auto it = code_of.find(out);
        code = it == code_of.end() ? 63 : it->second;
      }
      const uint32_t tgt = ncore < hot ? ncore : hot;
      T[(size_t)r * KL + k] = (uint16_t)((tgt << 6) | (ncore < hot ? code : 0));
    }
    T[(size_t)r * KL + K] = (uint16_t)(r << 6);  // identity column
  }
  for (uint32_t k = 0; k < KL; ++k) T[(size_t)hot * KL + k] = (uint16_t)(hot << 6);  // sentinel row
  for (int i = 0; i < 128; ++i) cs->start[i] = (uint16_t)rank[core_of[d.start[i]]];
  cs->dead = (uint32_t)rank[core_of[d.dead]];
  cs->quit = d.quit >= 0 ? (uint32_t)rank[core_of[d.quit]] : 0xFFFFFFFFu;
  cs->lds.resize((cs->lds.size() + 15) & ~(size_t)15, 0);
  cs->order = order;
  cs->ok = true;
  return true;
}

struct Blob {
  std::vector<uint8_t> bytes;
  size_t add(const void *src, size_t n) {
    size_t off = align256(bytes.size());
    bytes.resize(off + align256(n));
    if (n) memcpy(bytes.data() + off, src, n);
    return off;
  }
};

// ---------------------------------------------------------- scratch cache
// See dfa_scan.hpp scratch_malloc.  Blocks are rounded up (4 KiB, then
// 64 KiB multiples) and come from hipMalloc.  A freed block is cached per
// device with an event recorded on the freeing stream; an allocation of at
// most half its size on any stream of that device waits for that event
// (hipStreamWaitEvent) and reuses it, so reuse is ordered after the previous
// user's kernels whatever stream either used (a destroyed and recreated
// stream handle, the per-thread default stream).  The cache holds at most
// max(kScratchMinCap, 2 x the peak of live scratch bytes), at most
// kScratchMaxCap (RURE_AMD_SCRATCH_CAP overrides, bytes); a block freed
// beyond that is returned to the driver once its event has completed.
// Cached blocks go back to the driver on rure_amd_release_scratch(), when the
// last rure / rure_set is freed, and before a retry when an allocation fails.
// (The stream-ordered pool of hipMallocAsync kept freed memory mapped even
// after hipMemPoolTrimTo on this ROCm, measured in round 3.)
constexpr size_t kScratchMinCap = 256ull << 20, kScratchMaxCap = 8ull << 30;
struct ScratchBlock {
  size_t n;
  int dev;
  hipEvent_t ev;   // recorded at the last free (nullptr: never freed yet)
  hipStream_t st;  // the stream of the last free
};
struct ScratchCache {
  std::mutex mu;
  std::map<int, std::multimap<size_t, std::pair<void *, ScratchBlock>>> free_blocks;
  std::unordered_map<void *, ScratchBlock> live;
  size_t cached = 0, live_bytes = 0, peak_live = 0;
};
ScratchCache &scratch_cache() {
  static ScratchCache *c = new ScratchCache();  // never destroyed: frees may run at exit
  return *c;
}
size_t scratch_round(size_t n) { return n <= 4096 ? 4096 : (n + 65535) & ~(size_t)65535; }
size_t scratch_cap(const ScratchCache &c) {
  if (const char *v = getenv("RURE_AMD_SCRATCH_CAP")) return (size_t)strtoull(v, nullptr, 10);
  return std::min(kScratchMaxCap, std::max(kScratchMinCap, 2 * c.peak_live));
}
// Returns a block to the driver after its last use.
void scratch_release_block(void *p, const ScratchBlock &b) {
  if (b.ev) {
    (void)hipEventSynchronize(b.ev);
    (void)hipEventDestroy(b.ev);
  }
  (void)hipFree(p);
}
// Returns every cached block (caller holds c.mu).
void scratch_drop_all(ScratchCache &c) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto &kv : c.free_blocks) {
    if (kv.second.empty()) continue;
    (void)hipSetDevice(kv.first);
    for (auto &blk : kv.second) scratch_release_block(blk.second.first, blk.second.second);
    kv.second.clear();
  }
  (void)hipSetDevice(cur);
  c.cached = 0;
}
std::atomic<long> g_live_handles{0};   // rure + rure_set objects alive
}  // namespace

hipError_t rure_amd::scratch_malloc(void **p, size_t bytes, hipStream_t st) {
  if (!p) return hipErrorInvalidValue;
  int d = 0;
  hipError_t e = hipGetDevice(&d);
  if (e != hipSuccess) return e;
  const size_t n = scratch_round(bytes);
  ScratchCache &c = scratch_cache();
  {
    std::lock_guard<std::mutex> g(c.mu);
    auto &fb = c.free_blocks[d];
    auto b = fb.lower_bound(n);
    if (b != fb.end() && b->first <= 2 * n) {
      void *q = b->second.first;
      ScratchBlock blk = b->second.second;
      fb.erase(b);
      c.cached -= blk.n;
      c.live[q] = blk;
      c.live_bytes += blk.n;
      c.peak_live = std::max(c.peak_live, c.live_bytes);
      *p = q;
      // Reuse on the stream that freed it is ordered by the stream itself
      // (hipStreamDestroy completes a stream's work before its handle can be
      // handed out again); the wait is a barrier packet that cost the
      // latency-bound C1 step ~5 us.  hipStreamPerThread names a different
      // stream on every thread, so it always waits.
      if (!blk.ev || (st == blk.st && st != hipStreamPerThread)) return hipSuccess;
      return hipStreamWaitEvent(st, blk.ev, 0);
    }
  }
  void *q = nullptr;
  e = hipMalloc(&q, n);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> g(c.mu);
      scratch_drop_all(c);
    }
    e = hipMalloc(&q, n);
  }
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(c.mu);
  c.live[q] = ScratchBlock{n, d, nullptr, nullptr};
  c.live_bytes += n;
  c.peak_live = std::max(c.peak_live, c.live_bytes);
  *p = q;
  return hipSuccess;
}

hipError_t rure_amd::scratch_free(void *p, hipStream_t st) {
  if (!p) return hipSuccess;
  ScratchCache &c = scratch_cache();
  ScratchBlock blk{0, 0, nullptr, nullptr};
  {
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return hipErrorInvalidValue;  // not a scratch block
    blk = it->second;
    c.live.erase(it);
    c.live_bytes -= blk.n;
    hipError_t e = hipSuccess;
    if (!blk.ev) e = hipEventCreateWithFlags(&blk.ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(blk.ev, st);
    blk.st = st;
    if (e == hipSuccess && c.cached + blk.n <= scratch_cap(c)) {
      c.free_blocks[blk.dev].emplace(blk.n, std::make_pair(p, blk));
      c.cached += blk.n;
      return hipSuccess;
    }
  }
  scratch_release_block(p, blk);
  return hipSuccess;
}

namespace {

void scratch_release() {
  ScratchCache &c = scratch_cache();
  std::lock_guard<std::mutex> g(c.mu);
  scratch_drop_all(c);
}

void handle_created() { g_live_handles.fetch_add(1); }
void handle_freed() {
  if (g_live_handles.fetch_sub(1) == 1) scratch_release();
}

}  // namespace

namespace {

int device_cus(int dev) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
  return prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
}

int grid_for(size_t count, uint32_t lds_bytes, int cus) {
  size_t blocks = (count + 255) / 256;
  uint32_t per_cu = 8;
  if (lds_bytes > 0) per_cu = std::max<uint32_t>(1, std::min<uint32_t>(8, (160u * 1024u) / lds_bytes));
  size_t cap = (size_t)cus * per_cu;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  return (int)blocks;
}

// A reusable host->device staging area for the single-haystack entry points.
struct Staging {
  int dev = -1;
  hipStream_t stream = nullptr;
  uint8_t *hay = nullptr;
  size_t cap = 0;
  uint64_t *res = nullptr;
  ~Staging() {
    if (hay) (void)hipFree(hay);
    if (res) (void)hipFree(res);
    if (stream) (void)hipStreamDestroy(stream);
  }
  bool ensure(int d, size_t n, std::string *err) {
    if (dev != d) {
      if (hay) (void)hipFree(hay);
      if (res) (void)hipFree(res);
      if (stream) (void)hipStreamDestroy(stream);
      hay = nullptr; res = nullptr; stream = nullptr; cap = 0;
      dev = d;
      if (!hip_ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), err)) return false;
      if (!hip_ok(hipMalloc(&res, 64 * sizeof(uint64_t)), err)) return false;
    }
    if (n + 16 > cap) {
      if (hay) (void)hipFree(hay);
      hay = nullptr;
      size_t c = std::max<size_t>(n + 16, 1 << 16);
      if (!hip_ok(hipMalloc(&hay, c), err)) return false;
      cap = c;
    }
    return true;
  }
};

}  // namespace

struct rure {
  std::string pattern;
  uint32_t flags = 0;
  rure_options opts;
  Expr expr;
  ExecLiterals xl;          // the reference's literal sets and MatchType (host/literal_sets.hpp)
  Program nfa, fwd, rev;
  std::mutex mu;
  bool built = false, dfa_ok = false;
  std::string dfa_err;
  DenseDfa dfwd, drev;
  PackedFwd pf, pr;   // forward / reverse hot tables
  // automata past the u16 tables (column form, u32; big_dfa.hip): batched
  // find / is_match / shortest_match only, when dfa_ok is false
  bool big_ok = false, big_built = false;
  DenseDfa bfwd, brev;
  NfaTables nt;
  bool nfa_ok = false;
  std::map<int, DevTables> dev;
  Staging stage;
  // find_iter: forward DFA with dotstar-stripped states (chunked iteration)
  bool iter_built = false, iter_ok = false;
  DenseDfa dfwd_iter;
  PackedFwd pf_iter;
  bool lit_ok = false;      // the regex is a finite string set (literal find_iter engine)
  bool lits_done = false;   // lit_ok / lits computed (build_iter_dfa or literal_engine)
  uint32_t fb_n = 0;        // first-byte start rule (first_byte_rule): |F| or 0
  uint8_t fb_bytes[4] = {0, 0, 0, 0};
  std::vector<uint8_t> lex;   // lexer table (build_lex), empty if none
  uint32_t lex_s0 = 0;
  LiteralSet lits;
  std::map<int, std::pair<void *, FwdDfaDev>> iter_dev;
};

struct rure_set {
  std::vector<std::string> patterns;
  uint32_t flags = 0;
  rure_options opts;
  std::vector<Expr> exprs;
  Program fwd;      // compile_many DFA program (compile.rs:162-198)
  Program nfa;      // compile_many NFA program (no `.*?`, no saves)
  std::mutex mu;
  bool built = false, dfa_ok = false;
  std::string dfa_err;
  DenseDfa dfa;
  PackedFwd pf;
  CoreSet cores;      // core form, used when the hot table cannot hold the set DFA
  NfaTables nt;
  bool nfa_ok = false;
  std::map<int, DevTables> dev;
  Staging stage;
  rure *single = nullptr;   // one-pattern sets compile with compile_one
  // Sets of more than 64 patterns: the device work runs in groups of 64
  // consecutive patterns (group g owns mask word g).  Which patterns match a
  // haystack does not depend on the other patterns of the set (every pattern
  // is searched to completion, dfa.rs:525-570, pikevm.rs:150-180), so the
  // groups' answers concatenated are the set's.  The combined programs are
  // still compiled (size limit, program export).
  std::vector<rure_set *> groups;
  struct MultiSet *multi = nullptr;   // the groups as one pass (build_multi)
};

namespace {
void free_multi(rure_set *rs);
}  // namespace

struct rure_captures {           // rure.rs Captures(Locations): 2 slots per group
  std::vector<uint64_t> slots;
};

struct rure_iter_capture_names {
  std::vector<std::string> names;
  size_t next = 0;
  std::vector<char *> owned;     // handed-out C strings, freed with the iterator
};

struct rure_iter {
  rure *re;
  size_t last_end = 0;
  bool has_last_match = false;
  size_t last_match = 0;
};

namespace {

void kmer_forget(const rure *re);  // k-mer table cache (below)

SyntaxFlags syntax_flags(uint32_t flags) {  // rure.rs:119-124
  SyntaxFlags f;
  f.casei = (flags & RURE_FLAG_CASEI) != 0;
  f.multi = (flags & RURE_FLAG_MULTI) != 0;
  f.dotnl = (flags & RURE_FLAG_DOTNL) != 0;
  f.swap_greed = (flags & RURE_FLAG_SWAP_GREED) != 0;
  f.ignore_space = (flags & RURE_FLAG_SPACE) != 0;
  f.unicode = (flags & RURE_FLAG_UNICODE) != 0;
  f.allow_bytes = true;  // bytes::RegexBuilder (re_builder.rs:171, exec.rs:225)
  return f;
}

// Builds the automata of a regex once: the DFAs (when they materialise
// within budget) and always the Pike VM closure tables.  Returns whether a
// search engine is available.
// Automata past the u16 tables (more than 65535 states): both directions in
// column form with the larger raw-state budget, for the big_dfa.hip kernels.
// Programs with a Unicode word boundary (quit states) keep the Pike VM, and
// so does a search the reference runs as DfaAnchoredReverse.
void build_big_dfas(rure *re) {
  re->big_ok = false;
  if (!re->nfa_ok) return;
  if (re->fwd.has_unicode_word_boundary || re->rev.has_unicode_word_boundary) return;
  if (!re->nfa.anchored_start && re->nfa.anchored_end) return;
  DfaBuildLimits lim;
  lim.max_raw_states = kBigDfaRawStates;
  lim.max_bytes = kBigDfaBytes;
  if (const char *v = getenv("RURE_AMD_BIG_BYTES")) lim.max_bytes = (size_t)std::max(1ll, atoll(v));
  lim.columns = true;
  lim.minimise = false;   // construction already shares step targets; refinement doubled the build time
  std::string e1, e2;
  bool rok = false;
  std::thread rt([&] { rok = build_dense_dfa(re->rev, lim, &re->brev, &e2); });
  const bool fok = build_dense_dfa(re->fwd, lim, &re->bfwd, &e1);
  rt.join();
  if (!fok || !rok || re->bfwd.quit >= 0 || re->brev.quit >= 0) {
    re->bfwd = DenseDfa();
    re->brev = DenseDfa();
    return;
  }
  re->big_ok = true;
}

bool build_regex(rure *re) {
  std::lock_guard<std::mutex> g(re->mu);
  if (re->built) return re->dfa_ok || re->nfa_ok;
  re->built = true;
  std::string nerr;
  re->nfa_ok = build_nfa_tables(re->nfa, &re->nt, &nerr);
  DfaBuildLimits lim;
  std::string err, rerr;
  // the forward and reverse automata are independent: build them on two threads
  bool rev_ok = false;
  std::thread rt([&] { rev_ok = build_dense_dfa(re->rev, lim, &re->drev, &rerr); });
  const bool fwd_ok = build_dense_dfa(re->fwd, lim, &re->dfwd, &err);
  rt.join();
  if (fwd_ok && !rev_ok) err = rerr;
  if (!fwd_ok || !rev_ok || !pack_forward(re->dfwd, &re->pf, &err) || !pack_forward(re->drev, &re->pr, &err, true)) {
    re->dfa_err = err.empty() ? "reverse DFA too large" : err;
    re->dfa_ok = false;   // the big automata are built on first need (big_device)
    if (!re->nfa_ok) re->dfa_err += "; " + nerr;
    return re->nfa_ok;
  }
  re->dfa_ok = true;
  return true;
}

bool build_regex_dfas(rure *re) {
  build_regex(re);
  return re->dfa_ok;
}

bool build_set(rure_set *rs) {
  std::lock_guard<std::mutex> g(rs->mu);
  if (rs->built) return rs->dfa_ok || rs->nfa_ok;
  rs->built = true;
  if (rs->exprs.empty()) { rs->dfa_ok = true; return true; }
  std::string nerr;
  rs->nfa_ok = build_nfa_tables(rs->nfa, &rs->nt, &nerr);
  if (!rs->groups.empty()) {  // searched group by group; no combined DFA
    rs->dfa_err = "set of more than 64 patterns: automata are built per 64-pattern group";
    return rs->nfa_ok;
  }
  DfaBuildLimits lim;
  std::string err;
  if (!build_dense_dfa(rs->fwd, lim, &rs->dfa, &err) || !pack_forward(rs->dfa, &rs->pf, &err)) {
    rs->dfa_err = err;
    rs->dfa_ok = false;
    if (!rs->nfa_ok) rs->dfa_err += "; " + nerr;
    return rs->nfa_ok;
  }
  // Large sets: the byte-row hot table holds at most 255 states; switch to
  // the core form when more normal or match-reporting states than that exist.
  if (rs->dfa.n_normal > 255 || rs->dfa.n_match_end - rs->dfa.n_normal > 255)
    build_set_cores(rs->dfa, core_lds_budget(), &rs->cores);
  rs->dfa_ok = true;
  return true;
}

bool build_set_dfa(rure_set *rs) {
  build_set(rs);
  return rs->dfa_ok;
}

// Appends the Pike VM tables to an upload blob; fix_nfa() then points the
// descriptor into the device copy.
struct NfaOffsets { size_t leaves, cl_off, entries, perlw, save_off, save_slot; };

NfaOffsets add_nfa(Blob &b, const NfaTables &nt) {
  NfaOffsets o;
  std::vector<uint32_t> lv(nt.leaves.size() * 3);
  for (size_t i = 0; i < nt.leaves.size(); ++i) {
    const NfaLeaf &l = nt.leaves[i];
    lv[3 * i] = (uint32_t)l.kind | ((uint32_t)l.lo << 8) | ((uint32_t)l.hi << 16);
    lv[3 * i + 1] = l.closure;
    lv[3 * i + 2] = l.slot;
  }
  o.leaves = b.add(lv.data(), lv.size() * 4);
  o.cl_off = b.add(nt.cl_off.data(), nt.cl_off.size() * 4);
  o.entries = b.add(nt.entries.data(), nt.entries.size() * 8);
  namespace U = rure_amd_unicode;
  o.perlw = b.add(U::kPairs + 2 * U::kPerlW.first, (size_t)U::kPerlW.count * 8);
  o.save_off = b.add(nt.save_off.data(), nt.save_off.size() * 4);
  o.save_slot = b.add(nt.save_slot.data(), nt.save_slot.size() * 2);
  return o;
}

void fix_nfa(NfaDev *n, uint8_t *base, const NfaOffsets &o, const NfaTables &nt, bool single) {
  n->leaves = (const uint32_t *)(base + o.leaves);
  n->cl_off = (const uint32_t *)(base + o.cl_off);
  n->entries = (const uint2 *)(base + o.entries);
  n->perlw = (const uint32_t *)(base + o.perlw);
  n->perlw_n = rure_amd_unicode::kPerlW.count;
  n->save_off = (const uint32_t *)(base + o.save_off);
  n->save_slot = (const uint16_t *)(base + o.save_slot);
  n->nleaves = (uint32_t)nt.leaves.size();
  n->root = nt.root;
  n->nmatch = nt.nmatch;
  n->anchored = nt.anchored_start ? 1 : 0;
  n->single = single ? 1 : 0;
  n->looks = nt.looks_used;
  n->unicode_wb = nt.unicode_wb ? 1 : 0;
}

bool upload_blob(const Blob &b, DevTables *t, std::string *err) {
  if (!hip_ok(hipMalloc(&t->blob, b.bytes.size()), err)) return false;
  if (!hip_ok(hipMemcpy(t->blob, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice), err)) {
    (void)hipFree(t->blob);
    t->blob = nullptr;
    return false;
  }
  return true;
}

// A literal list (bytes, n + 1 u32 offsets) into an upload blob.
struct LitOffsets { size_t bytes, off; uint32_t n; };
LitOffsets add_litlist(Blob &b, const Literals &l) {
  std::string cat;
  std::vector<uint32_t> off{0};
  for (const Lit &x : l.lits) {
    cat += x.v;
    off.push_back((uint32_t)cat.size());
  }
  cat.resize(cat.size() + 16, 0);
  LitOffsets o;
  o.bytes = b.add(cat.data(), cat.size());
  o.off = b.add(off.data(), off.size() * 4);
  o.n = (uint32_t)l.lits.size();
  return o;
}

// Whether the reference's match type makes this regex's searches differ from
// a forward DFA search (DevTables::mt_lane).
bool needs_mt_lane(const ExecLiterals &x) {
  return x.match_type == MT_DFA_SUFFIX || x.match_type == MT_LITERAL_ANCHORED_START ||
         (x.match_type == MT_LITERAL_UNANCHORED && !x.prefixes.complete);
}

// FwdDfaDev::pfx_*: the start-state prefix skip (dfa.rs:700-711), for a
// DFA whose start does not depend on look-behind, from the regex's prefix
// literals (dfa.prefixes, exec.rs:308-311; not for anchored starts,
// dfa.rs:1516-1522 has_prefix) when they have at most 4 first bytes.
// RURE_AMD_PREFIX=0 turns it off (A/B).
void set_prefix_skip(const rure *re, FwdDfaDev *f) {
  f->pfx_n = 0;
  const char *env = getenv("RURE_AMD_PREFIX");
  if ((env && env[0] == '0') || !f->ustart1 || re->nfa.anchored_start) return;
  const LitSearcher &p = re->xl.prefixes;
  if (p.matcher == 0 || p.lits.lits.empty()) return;
  bool seen[256] = {false};
  uint32_t n = 0;
  for (const Lit &l : p.lits.lits) {
    if (l.v.empty()) return;
    const uint8_t b = (uint8_t)l.v[0];
    if (seen[b]) continue;
    if (n == 4) return;
    seen[b] = true;
    f->pfx_rep[n++] = b * 0x01010101u;
  }
  f->pfx_n = n;
}

// Upload (once per device) and return device descriptors.
DevTables *regex_device(rure *re, std::string *err) {
  if (!build_regex(re)) { if (err) *err = re->dfa_err; return nullptr; }
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  std::lock_guard<std::mutex> g(re->mu);
  auto it = re->dev.find(d);
  if (it != re->dev.end()) return &it->second;
  Blob b;
  DevTables t;
  t.cus = device_cus(d);
  NfaOffsets no{};
  if (re->nfa_ok) no = add_nfa(b, re->nt);
  size_t o_lds = 0, o_lds_s = 0, o_full = 0, o_eof = 0, o_start = 0, o_rfull = 0, o_reof = 0, o_rstart = 0,
         o_rlds = 0;
  const PackedFwd &pf = re->pf;
  const DenseDfa &rv = re->drev;
  if (re->dfa_ok) {
    std::vector<uint16_t> rfull(rv.trans.size()), rstart(128);
    for (size_t i = 0; i < rv.trans.size(); ++i) rfull[i] = (uint16_t)rv.trans[i];
    for (int i = 0; i < 128; ++i) rstart[i] = (uint16_t)rv.start[i];
    o_lds = b.add(pf.lds.data(), pf.lds.size());
    o_lds_s = b.add(pf.lds_s.data(), pf.lds_s.size());
    o_full = b.add(pf.full.data(), pf.full.size() * 2);
    o_eof = b.add(pf.eof.data(), pf.eof.size());
    o_start = b.add(pf.start.data(), 256);
    o_rfull = b.add(rfull.data(), rfull.size() * 2);
    o_reof = b.add(rv.eof_match.data(), rv.eof_match.size());
    o_rstart = b.add(rstart.data(), 256);
    o_rlds = b.add(re->pr.lds.data(), re->pr.lds.size());
  }
  const bool mt_lane = needs_mt_lane(re->xl);
  LitOffsets lp{}, ls{};
  size_t o_lcs = 0;
  if (mt_lane) {
    lp = add_litlist(b, re->xl.prefixes.lits);
    ls = add_litlist(b, re->xl.suffixes.lits);
    std::string lcs = re->xl.suffixes.lcs;
    lcs.resize(lcs.size() + 16, 0);
    o_lcs = b.add(lcs.data(), lcs.size());
  }
  if (!upload_blob(b, &t, err)) return nullptr;
  uint8_t *base = (uint8_t *)t.blob;
  if (re->nfa_ok) fix_nfa(&t.n, base, no, re->nt, true);
  if (mt_lane) {
    t.mt_lane = true;
    t.m.mt = re->xl.match_type;
    t.m.pre = LitListDev{base + lp.bytes, (const uint32_t *)(base + lp.off), lp.n, re->xl.prefixes.matcher};
    t.m.suf = LitListDev{base + ls.bytes, (const uint32_t *)(base + ls.off), ls.n, re->xl.suffixes.matcher};
    t.m.lcs = base + o_lcs;
    t.m.lcs_len = (uint32_t)re->xl.suffixes.lcs.size();
  }
  if (re->dfa_ok) {
    const DenseDfa &fw = re->dfwd;
    t.has_dfa = true;
    t.quit_possible = fw.quit >= 0 || rv.quit >= 0;
    t.f.lds_image = base + o_lds;
    t.f.lds_bytes = (uint32_t)pf.lds.size();
    t.f.hot = pf.hot;
    t.f.lds_image_s = base + o_lds_s;
    t.f.lds_bytes_s = (uint32_t)pf.lds_s.size();
    t.f.stride = pf.stride;
    t.f.hot_s = pf.hot_s;
    t.f.P = pf.P;
    t.f.sent = pf.sent;
    t.f.cus = (uint32_t)t.cus;
    t.f.full = (const uint16_t *)(base + o_full);
    t.f.eof = base + o_eof;
    t.f.start = (const uint16_t *)(base + o_start);
    t.f.n_normal = fw.n_normal;
    t.f.n_match_end = fw.n_match_end;
    t.f.dead = fw.dead;
    t.f.quit = fw.quit < 0 ? 0xFFFFFFFFu : (uint32_t)fw.quit;
    t.r.lds_image = base + o_rlds;
    t.r.lds_bytes = (uint32_t)re->pr.lds.size();
    t.r.hot = re->pr.hot;
    t.r.full = (const uint16_t *)(base + o_rfull);
    t.r.eof = base + o_reof;
    t.r.start = (const uint16_t *)(base + o_rstart);
    t.r.n_normal = rv.n_normal;
    t.r.n_match_end = rv.n_match_end;
    t.r.dead = rv.dead;
    t.r.quit = rv.quit < 0 ? 0xFFFFFFFFu : (uint32_t)rv.quit;
    t.r.all = re->pr.all;
    t.r.ustart1 = re->pr.ustart1;
    t.f.ustart1 = pf.ustart1;
    t.f.nonempty = can_match_empty(re->nfa) ? 0 : 1;
    set_prefix_skip(re, &t.f);
    // a regex anchored at the end and not at the start runs the reverse DFA
    // from the end of the text (exec.rs:1175-1177, 671-688)
    t.anchored_rev = !re->nfa.anchored_start && re->nfa.anchored_end;
  }
  t.owner = re;
  if (t.quit_possible && !re->nfa_ok) {
    (void)hipFree(t.blob);
    if (err) *err = "the DFA can quit and the NFA tables could not be built";
    return nullptr;
  }
  return &(re->dev[d] = t);
}

// Automata past the u16 tables, built and uploaded on the first batch that
// would run them (big_batch): their construction can take seconds and
// hundreds of MB of host memory (bounded by kBigDfaBytes), which a regex
// searched on the Pike VM only (few long haystacks) never needs.  Returns
// whether t now has them.
bool big_device(const DevTables &tc) {
  DevTables &t = const_cast<DevTables &>(tc);  // the regex's own entry of rure::dev
  rure *re = t.owner;
  if (!re) return false;
  std::lock_guard<std::mutex> g(re->mu);
  if (t.big_tried) return t.has_big;
  t.big_tried = true;
  if (!re->big_built) {
    re->big_built = true;
    build_big_dfas(re);
  }
  if (!re->big_ok) return false;
  Blob b;
  size_t o_big[8];
  const DenseDfa *bd[2] = {&re->bfwd, &re->brev};
  for (int k = 0; k < 2; ++k) {
    o_big[4 * k] = b.add(bd[k]->ctrans.data(), bd[k]->ctrans.size() * 4);
    o_big[4 * k + 1] = b.add(bd[k]->colmap, 256);
    o_big[4 * k + 2] = b.add(bd[k]->eof_match.data(), bd[k]->eof_match.size());
    o_big[4 * k + 3] = b.add(bd[k]->start, 128 * 4);
  }
  DevTables tmp;
  std::string err;
  if (!upload_blob(b, &tmp, &err)) return false;
  uint8_t *base = (uint8_t *)tmp.blob;
  BigDfaDev *dst[2] = {&t.bf, &t.br};
  for (int k = 0; k < 2; ++k) {
    const DenseDfa &D = *bd[k];
    BigDfaDev &x = *dst[k];
    x.trans = (const uint32_t *)(base + o_big[4 * k]);
    x.colmap = base + o_big[4 * k + 1];
    x.eof = base + o_big[4 * k + 2];
    x.start = (const uint32_t *)(base + o_big[4 * k + 3]);
    x.ncol = D.ncol;
    x.nstates = (uint32_t)D.nstates;
    x.hot = k == 0 ? big_dfa_hot_rows(D.ncol, (uint32_t)D.nstates) : 0;
    x.n_normal = (uint32_t)D.n_normal;
    x.n_match_end = (uint32_t)D.n_match_end;
    x.dead = (uint32_t)D.dead;
    x.ustart1 = uniform_start(D);
  }
  t.big_blob = tmp.blob;
  t.has_big = true;
  return true;
}

DevTables *set_device(rure_set *rs, std::string *err) {
  if (!build_set(rs)) { if (err) *err = rs->dfa_err; return nullptr; }
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  std::lock_guard<std::mutex> g(rs->mu);
  auto it = rs->dev.find(d);
  if (it != rs->dev.end()) return &it->second;
  const PackedFwd &pf = rs->pf;
  Blob b;
  DevTables t;
  t.cus = device_cus(d);
  NfaOffsets no{};
  if (rs->nfa_ok) no = add_nfa(b, rs->nt);
  size_t o_lds = 0, o_full = 0, o_mask = 0, o_now = 0, o_start = 0;
  size_t c_lds = 0, c_core = 0, c_out = 0, c_eof = 0, c_start = 0;
  const CoreSet &cs = rs->cores;
  if (rs->dfa_ok && cs.ok) {
    c_lds = b.add(cs.lds.data(), cs.lds.size());
    c_core = b.add(cs.gcore.data(), cs.gcore.size() * 2);
    c_out = b.add(cs.gout.data(), cs.gout.size() * 8);
    c_eof = b.add(cs.eof.data(), cs.eof.size() * 8);
    c_start = b.add(cs.start, 256);
  }
  if (rs->dfa_ok) {
    o_lds = b.add(pf.lds.data(), pf.lds.size());
    o_full = b.add(pf.full.data(), pf.full.size() * 2);
    o_mask = b.add(pf.eof_mask.data(), pf.eof_mask.size() * 8);
    o_now = b.add(pf.now_mask.data(), pf.now_mask.size() * 8);
    o_start = b.add(pf.start.data(), 256);
  }
  if (!upload_blob(b, &t, err)) return nullptr;
  uint8_t *base = (uint8_t *)t.blob;
  // set programs: several Match instructions, no leftmost-first cut (pikevm.rs:196-212)
  if (rs->nfa_ok) fix_nfa(&t.n, base, no, rs->nt, rs->nt.nmatch <= 1);
  if (rs->dfa_ok) {
    const DenseDfa &fw = rs->dfa;
    t.has_dfa = true;
    t.quit_possible = fw.quit >= 0;
    t.s.lds_image = base + o_lds;
    t.s.lds_bytes = (uint32_t)pf.lds.size();
    t.s.hot = pf.hot;
    t.s.full = (const uint16_t *)(base + o_full);
    t.s.eof_mask = (const uint64_t *)(base + o_mask);
    t.s.now_mask = (const uint64_t *)(base + o_now);
    t.s.all = rs->exprs.size() >= 64 ? ~0ull : ((1ull << rs->exprs.size()) - 1);
    t.s.start = (const uint16_t *)(base + o_start);
    t.s.n_normal = fw.n_normal;
    t.s.n_match_end = fw.n_match_end;
    t.s.dead = fw.dead;
    t.s.quit = fw.quit < 0 ? 0xFFFFFFFFu : (uint32_t)fw.quit;
    if (cs.ok) {
      t.use_cores = true;
      t.c.lds_image = base + c_lds;
      t.c.lds_bytes = (uint32_t)cs.lds.size();
      t.c.hot = cs.hot;
      t.c.K = cs.K;
      t.c.gcore = (const uint16_t *)(base + c_core);
      t.c.gout = (const uint64_t *)(base + c_out);
      t.c.eof = (const uint64_t *)(base + c_eof);
      t.c.start = (const uint16_t *)(base + c_start);
      t.c.all = t.s.all;
      t.c.dead = cs.dead;
      t.c.quit = cs.quit;
      t.c.mt_off = cs.mt_off;
    }
  }
  if (t.quit_possible && !rs->nfa_ok) {
    (void)hipFree(t.blob);
    if (err) *err = "the DFA can quit and the NFA tables could not be built";
    return nullptr;
  }
  return &(rs->dev[d] = t);
}

int pike_grid(size_t count, bool fallback, const NfaDev &n, int cus) {
  size_t units = fallback ? (count + 63) / 64 : count;
  size_t wb = nfa_wave_bytes(n.nleaves);
  size_t per_cu = wb <= kNfaLdsMax ? std::max<size_t>(1, std::min<size_t>(32, (160u * 1024u) / wb)) : 4;
  size_t g = std::min(units, (size_t)cus * per_cu);
  return (int)std::max<size_t>(g, 1);
}

// Pike VM pass: all haystacks (no DFA) or only those the DFA quit on.
hipError_t run_pike(int mode, bool fallback, const BatchDev &b, const DevTables &t, void *out, hipStream_t st) {
  int grid = pike_grid(b.count, fallback, t.n, t.cus);
  size_t wb = nfa_wave_bytes(t.n.nleaves);
  if (wb <= kNfaLdsMax) return launch_pike(mode, fallback, b, t.n, out, nullptr, st, grid);
  void *scratch = nullptr;
  hipError_t e = scratch_malloc(&scratch, wb * (size_t)grid, st);
  if (e != hipSuccess) return e;
  e = launch_pike(mode, fallback, b, t.n, out, scratch, st, grid);
  hipError_t e2 = scratch_free(scratch, st);
  return e != hipSuccess ? e : e2;
}

// The first-byte start rule of FwdDfaDev::fb_n, decided on the find_iter DFA
// (with strip states, no look-around, flag-independent start).  F = the
// ASCII bytes on which the anchored start state strip[start] does not die
// (every match starts with a byte on which it does not die).  Every state
// reachable from it through F and then ASCII bytes, before a match-flag state
// is entered, must have no ASCII transition to `dead` or `quit`: an anchored
// run from an F byte over ASCII text then cannot fail except by reaching the
// end of the text.  So in a forward search (`.*?` prefix, leftmost-first)
// from p over ASCII text, the thread started at the first c >= p with text[c]
// in F stays alive until it has matched, the DFA reaches `dead` before the
// end only after that, and the match it reports starts at c (threads from
// earlier starts have priority, dfa.rs:910-1048).  The kernel applies the
// rule to a search only when every byte it loaded was ASCII (Unicode classes
// such as `[^\n]` die on invalid UTF-8).  Returns |F| (1..4) or 0.
static uint32_t first_byte_rule(const DenseDfa &d, uint32_t ustart1, bool nonempty, uint8_t bytes[4]) {
  if (!ustart1 || !nonempty || d.strip.empty() || d.quit >= 0) return 0;
  const uint32_t a0 = d.strip[ustart1 - 1];
  if ((int)a0 >= d.n_normal) return 0;
  uint32_t nf = 0;
  std::vector<uint32_t> todo;
  std::vector<uint8_t> seen(d.nstates, 0);
  for (int c = 0; c < 128; ++c) {
    const uint32_t t = d.trans[(size_t)a0 * 256 + c];
    if ((int)t == d.dead) continue;
    if (nf == 4) return 0;
    bytes[nf++] = (uint8_t)c;
    if ((int)t < d.n_normal && !seen[t]) { seen[t] = 1; todo.push_back(t); }
  }
  while (!todo.empty()) {  // pre-match states: normal states reached before a match flag
    const uint32_t x = todo.back();
    todo.pop_back();
    for (int c = 0; c < 128; ++c) {
      const uint32_t t = d.trans[(size_t)x * 256 + c];
      if ((int)t == d.dead) return 0;
      if ((int)t < d.n_normal && !seen[t]) { seen[t] = 1; todo.push_back(t); }
    }
  }
  return nf;
}

// The lexer table of FwdDfaDev::lex_image (iter_spec_lex_tile_kernel).
// Needs the first-byte start rule (a match's start is the first F byte of its
// search on ASCII text) and terminal match states: every state carrying the
// (one-byte delayed) match flag has only dead transitions, so entering one at
// byte x ends the search with the match [start, x), and the iteration's next
// search begins at x with the start state S0 (re_trait.rs:197-221; the regex
// is nonempty).  The table composes the two: the transition into a match
// state on byte b becomes S0's transition on b into a *twin* of its target
// (same row; entering a twin = a match ended here).  u8 state numbers, rows
// of kRow bytes (the forward kernels' LDS layout), numbered [other states,
// S0, twin(S0), other twins] so that one clamp of the state number gives the
// byte's flags (FwdDfaDev::lex_z).  Returns false if the rule does not hold
// or the states do not fit u8.
static bool build_lex(const DenseDfa &d, uint32_t ustart1, uint32_t fb_n, std::vector<uint8_t> *img,
                      uint32_t *s0_idx) {
  img->clear();
  if (!fb_n || !ustart1 || d.quit >= 0) return false;
  const uint32_t s0 = ustart1 - 1;
  for (int m = d.n_normal; m < d.n_match_end; ++m)
    for (int c = 0; c < 256; ++c)
      if ((int)d.trans[(size_t)m * 256 + c] != d.dead) return false;
  auto is_match = [&](uint32_t t) { return (int)t >= d.n_normal && (int)t < d.n_match_end; };
  // states reachable from S0 (match transitions replaced by restarts)
  std::vector<uint8_t> reach(d.nstates, 0);
  std::vector<uint32_t> todo{s0};
  reach[s0] = 1;
  while (!todo.empty()) {
    const uint32_t q = todo.back();
    todo.pop_back();
    for (int c = 0; c < 256; ++c) {
      uint32_t t = d.trans[(size_t)q * 256 + c];
      if (is_match(t)) t = d.trans[(size_t)s0 * 256 + c];
      if (is_match(t)) return false;  // S0 itself matching on one byte: an empty match
      if (!reach[t]) { reach[t] = 1; todo.push_back(t); }
    }
  }
  std::vector<int> plain(d.nstates, -1), twin(d.nstates, -1);
  std::vector<uint32_t> rows;  // DFA state of each lexer row
  for (int q = 0; q < d.nstates; ++q)
    if (reach[q] && (uint32_t)q != s0) { plain[q] = (int)rows.size(); rows.push_back(q); }
  plain[s0] = (int)rows.size();
  rows.push_back(s0);
  twin[s0] = (int)rows.size();
  rows.push_back(s0);
  for (int c = 0; c < 256; ++c) {
    const uint32_t t = d.trans[(size_t)s0 * 256 + c];
    if (twin[t] < 0) { twin[t] = (int)rows.size(); rows.push_back(t); }
  }
  if (rows.size() > kLexMaxRows || plain[s0] < 1) return false;
  // entries 4 row + code (dfa_scan.hpp FwdDfaDev::lex_image): codes 0 for the
  // rows below S0, 1 for S0, 2 for twin(S0), 3 for the other twins
  const uint32_t ps0 = (uint32_t)plain[s0];
  auto code = [&](uint32_t r) -> uint32_t { return r < ps0 ? 0 : r == ps0 ? 1 : r == ps0 + 1 ? 2 : 3; };
  auto entry = [&](uint32_t r) -> uint8_t { return (uint8_t)(4 * r + code(r)); };
  img->assign(((rows.size() - 1) * kRow + 3 * kLexUnit + 256 + 15) & ~(size_t)15, 0);
  for (size_t i = 0; i < rows.size(); ++i)
    for (int c = 0; c < 256; ++c) {
      const uint32_t t = d.trans[(size_t)rows[i] * 256 + c];
      const int to = is_match(t) ? twin[d.trans[(size_t)s0 * 256 + c]] : plain[t];
      (*img)[(size_t)entry((uint32_t)i) * kLexUnit + c] = entry((uint32_t)to);
    }
  *s0_idx = entry(ps0);
  return true;
}

bool build_iter_dfa(rure *re) {
  if (!build_regex_dfas(re)) return false;
  std::lock_guard<std::mutex> g(re->mu);
  if (!re->iter_built) {
    re->iter_built = true;
    DfaBuildLimits lim;
    lim.strip = true;
    std::string e;
    re->iter_ok = build_dense_dfa(re->fwd, lim, &re->dfwd_iter, &e) && pack_forward(re->dfwd_iter, &re->pf_iter, &e, true);
    if (!re->lits_done) re->lit_ok = extract_literals(re->nfa, kLitMax, kLitLen, &re->lits);
    re->lits_done = true;
    if (re->iter_ok)
      re->fb_n = first_byte_rule(re->dfwd_iter, re->pf_iter.ustart1, !can_match_empty(re->nfa), re->fb_bytes);
    if (re->iter_ok) build_lex(re->dfwd_iter, re->pf_iter.ustart1, re->fb_n, &re->lex, &re->lex_s0);
  }
  return re->iter_ok;
}


// Forward DFA with stripped states for the chunked find_iter (built and
// uploaded on first use).  Returns null if it does not materialise.
// The Shift-And image of a string set whose strings all have one length L
// (iter_spec_sa_kernel): strings equal but in one position are merged into
// class sequences (the union of that position's classes; the same language),
// until no pair merges; sequence x owns bits [x L, (x + 1) L) of the state.
// mask[b] bit i = byte b is in the class of bit position i.  Returns false
// (and leaves the outputs empty) unless the sequences fit 64 bits.
static bool build_shiftand(const LiteralSet &ls, std::vector<uint64_t> *mask, uint64_t *init, uint64_t *fin,
                           uint32_t *len, uint32_t *bits) {
  mask->clear();
  *init = *fin = 0;
  *len = *bits = 0;
  if (ls.lits.empty() || ls.minlen != ls.maxlen || ls.minlen < 1) return false;
  const size_t L = ls.minlen;
  using Cls = std::array<uint64_t, 4>;
  std::vector<std::vector<Cls>> seqs;
  for (const std::string &l : ls.lits) {
    std::vector<Cls> q(L, Cls{0, 0, 0, 0});
    for (size_t i = 0; i < L; ++i) q[i][(uint8_t)l[i] >> 6] |= 1ull << ((uint8_t)l[i] & 63);
    seqs.push_back(q);
  }
  for (bool merged = true; merged;) {
    merged = false;
    for (size_t x = 0; x < seqs.size() && !merged; ++x)
      for (size_t y = x + 1; y < seqs.size() && !merged; ++y) {
        int diff = -1, nd = 0;
        for (size_t i = 0; i < L && nd < 2; ++i)
          if (seqs[x][i] != seqs[y][i]) { diff = (int)i; ++nd; }
        if (nd == 1) {
          for (int w = 0; w < 4; ++w) seqs[x][diff][w] |= seqs[y][diff][w];
          seqs.erase(seqs.begin() + y);
          merged = true;
        }
      }
  }
  if (seqs.size() * L > 64) return false;
  *len = (uint32_t)L;
  *bits = (uint32_t)(seqs.size() * L);
  mask->assign(256, 0);
  for (size_t x = 0; x < seqs.size(); ++x) {
    *init |= 1ull << (x * L);
    *fin |= 1ull << (x * L + L - 1);
    for (size_t i = 0; i < L; ++i)
      for (int c = 0; c < 256; ++c)
        if ((seqs[x][i][c >> 6] >> (c & 63)) & 1) (*mask)[c] |= 1ull << (x * L + i);
  }
  return true;
}

const FwdDfaDev *iter_device(rure *re, const DevTables &t, std::string *err) {
  if (!build_iter_dfa(re)) return nullptr;
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  std::lock_guard<std::mutex> g(re->mu);
  auto it = re->iter_dev.find(d);
  if (it != re->iter_dev.end()) return &it->second.second;
  const PackedFwd &pf = re->pf_iter;
  const DenseDfa &fw = re->dfwd_iter;
  std::vector<uint16_t> strip(fw.strip.size());
  for (size_t i = 0; i < strip.size(); ++i) strip[i] = (uint16_t)fw.strip[i];
  Blob b;
  size_t o_lds = b.add(pf.lds.data(), pf.lds.size());
  size_t o_full = b.add(pf.full.data(), pf.full.size() * 2);
  size_t o_eof = b.add(pf.eof.data(), pf.eof.size());
  size_t o_start = b.add(pf.start.data(), 256);
  size_t o_strip = b.add(strip.data(), strip.size() * 2);
  std::vector<uint8_t> lit_img;
  uint32_t lit_k = 0;
  if (re->lit_ok) {
    // literal engine image (dfa_scan.hpp kLit*): prefix-hash bitmap, keys,
    // lengths, bytes
    lit_k = (uint32_t)std::min<size_t>(re->lits.minlen, 4);
    lit_img.assign(kLitImage, 0);
    uint32_t *bitmap = (uint32_t *)lit_img.data();
    for (size_t x = 0; x < re->lits.lits.size(); ++x) {
      const std::string &l = re->lits.lits[x];
      uint32_t key = 0;
      for (uint32_t j = 0; j < lit_k; ++j) key |= (uint32_t)(uint8_t)l[j] << (8 * j);
      const uint32_t h = lit_hash(key);
      bitmap[h >> 5] |= 1u << (h & 31);
      std::memcpy(lit_img.data() + kLitKeys + 4 * x, &key, 4);
      lit_img[kLitLens + x] = (uint8_t)l.size();
      std::memcpy(lit_img.data() + kLitBytes + kLitLen * x, l.data(), l.size());
      if (re->lits.minlen >= 8) {
        uint32_t key2 = 0;
        std::memcpy(&key2, l.data() + 4, 4);
        const uint32_t h2 = lit_hash(key2);
        ((uint32_t *)(lit_img.data() + kLitBitmap2))[h2 >> 5] |= 1u << (h2 & 31);
      }
    }
  }
  size_t o_lit = lit_img.empty() ? 0 : b.add(lit_img.data(), lit_img.size());
  // Shift-And image (build_shiftand)
  std::vector<uint64_t> sa_img;
  uint64_t sa_init = 0, sa_final = 0;
  uint32_t sa_len = 0, sa_bits = 0;
  if (re->lit_ok) build_shiftand(re->lits, &sa_img, &sa_init, &sa_final, &sa_len, &sa_bits);
  size_t o_sa = sa_img.empty() ? 0 : b.add(sa_img.data(), sa_img.size() * 8);
  size_t o_lex = re->lex.empty() ? 0 : b.add(re->lex.data(), re->lex.size());
  DevTables tmp;
  if (!upload_blob(b, &tmp, err)) return nullptr;
  uint8_t *base = (uint8_t *)tmp.blob;
  FwdDfaDev f{};
  f.lds_image = base + o_lds;
  f.lds_bytes = (uint32_t)pf.lds.size();
  f.hot = pf.hot;
  f.lds_image_s = nullptr;
  f.stride = 1;
  f.cus = (uint32_t)t.cus;
  f.full = (const uint16_t *)(base + o_full);
  f.eof = base + o_eof;
  f.start = (const uint16_t *)(base + o_start);
  f.strip = (const uint16_t *)(base + o_strip);
  f.n_normal = fw.n_normal;
  f.n_match_end = fw.n_match_end;
  f.dead = fw.dead;
  f.quit = fw.quit < 0 ? 0xFFFFFFFFu : (uint32_t)fw.quit;
  f.all = pf.all;
  f.ustart1 = pf.ustart1;
  f.nonempty = can_match_empty(re->nfa) ? 0 : 1;
  set_prefix_skip(re, &f);
  // RURE_AMD_FB=0 turns the first-byte start rule off (reverse scans)
  f.fb_n = getenv("RURE_AMD_FB") && getenv("RURE_AMD_FB")[0] == '0' ? 0 : re->fb_n;
  for (uint32_t i = 0; i < 4; ++i) f.fb_rep[i] = (i < re->fb_n ? re->fb_bytes[i] : re->fb_bytes[0]) * 0x01010101u;
  if (!lit_img.empty()) {
    f.lit_image = base + o_lit;
    f.lit_bytes = kLitImage;
    f.lit_n = (uint32_t)re->lits.lits.size();
    f.lit_k = lit_k;
    f.lit_minlen = (uint32_t)re->lits.minlen;
    f.lit_maxlen = (uint32_t)re->lits.maxlen;
    f.lit_k8 = re->lits.minlen >= 8 ? 1 : 0;
  }
  if (!re->lex.empty()) {
    f.lex_image = base + o_lex;
    f.lex_bytes = (uint32_t)re->lex.size();
    f.lex_s0 = re->lex_s0;
  }
  if (!sa_img.empty()) {
    f.sa_image = (const uint64_t *)(base + o_sa);
    f.sa_init = sa_init;
    f.sa_final = sa_final;
    f.sa_len = sa_len;
    f.sa_bits = sa_bits;
  }
  re->iter_dev[d] = {tmp.blob, f};
  return &re->iter_dev[d].second;
}

// The engine dispatch of exec.rs:473-514 / 382-420 for a batch: DFA, and the
// Pike VM where the DFA quits (or instead of it when it does not fit).
// Chunk sizes are an odd number of 128-byte lines: lanes that scan chunks in
// lockstep then read addresses with different low bits, instead of hammering
// the few HBM channels a power-of-two chunk would map them all to.
uint64_t odd_lines(uint64_t bytes) {
  uint64_t lines = (bytes + 127) / 128;
  if ((lines & 1) == 0) ++lines;
  return lines * 128;
}

// Few long haystacks: one lane per haystack would leave the chip idle, so the
// search is split into chunks (launch_long_scan).  Needs a DFA that cannot
// quit (the Pike VM fallback is per haystack).
bool long_batch(int mode, const BatchDev &b, const DevTables &t, uint64_t *chunk) {
  if (b.offs || !t.has_dfa || t.quit_possible || b.count == 0) return false;
  const uint64_t span = b.length > b.start ? b.length - b.start : 0;
  if (span < (256u << 10) || b.count >= (uint64_t)t.cus * 128) {
    // Small batches of medium haystacks (C1: 1024 x 1 KiB): one lane per
    // haystack runs count / 256 workgroups on a 256-CU chip, each lane a
    // dependent chain over its whole haystack; units of >= 128 B spread the
    // searches over about one wave per CU.  End-anchored regexes keep the
    // reverse scan (it reads O(match) bytes); single calls and batches of
    // fewer than 64 haystacks keep one lane each.  RURE_AMD_SPLIT=0 turns it off.
    // Only is_match: a unit stops at its first match there, while a find /
    // shortest_match unit scans on until the DFA dies, so a pattern that never
    // dies ([^\n]* over text without newlines) would cost every unit the rest
    // of its haystack (about units / 2 times the unsplit work).
    const char *sv = getenv("RURE_AMD_SPLIT");
    if ((sv && sv[0] == '0') || mode != MODE_ISMATCH || t.anchored_rev || span < 512 || b.count < 64 ||
        b.count > (uint64_t)t.cus * 16)
      return false;
    const uint64_t per_h = ((uint64_t)t.cus * 64 + b.count - 1) / b.count;
    const uint64_t c = odd_lines(std::max<uint64_t>(128, (span + per_h - 1) / per_h));
    if (c >= span) return false;
    *chunk = c;
    return true;
  }
  // 16 waves per CU: per-lane streams need latency hiding (RURE_AMD_LONG_LANES
  // per CU overrides, tuning)
  uint64_t per_cu = 1024;
  if (const char *v = getenv("RURE_AMD_LONG_LANES")) per_cu = std::max(64, atoi(v));
  const uint64_t target = (uint64_t)t.cus * per_cu;
  const uint64_t per_h = (target + b.count - 1) / b.count;
  uint64_t c = std::max<uint64_t>(16u << 10, (span + per_h - 1) / per_h);
  *chunk = odd_lines(c);
  return true;
}

// The DFA step of find / is_match / shortest_match (the quit marker where the
// DFA quit): the forward DFA (+ reverse for find), or for DfaAnchoredReverse
// regexes the reverse DFA from the end of each haystack.  Long haystacks
// searched from their start take the chunked forward scan for either (the
// two answer alike at start 0: only the look-behind at `start` differs).
hipError_t run_dfa_step(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st, int dfa_grid,
                        const FwdDfaDev *iter) {
  uint64_t chunk = 0;
  const bool long_fwd = iter && long_batch(mode, b, t, &chunk);
  if (t.anchored_rev && !(long_fwd && b.start == 0)) return launch_dfa_anchored_rev(mode, b, t.r, out, st, dfa_grid);
  if (long_fwd) return launch_long_scan(mode, b, *iter, t.r, chunk, out, st, t.cus);
  return launch_dfa_fwd(mode, b, t.f, t.r, out, st, dfa_grid);
}

// The Literal / DfaSuffix match types (DevTables::mt_lane): literal searches
// need no DFA; DfaSuffix steps the DFA tables (without them the reference's
// DFA would have quit too: the Pike VM answers).
bool lane_search_ok(const DevTables &t) { return t.mt_lane && (t.m.mt != MT_DFA_SUFFIX || t.has_dfa); }

hipError_t run_lane_search(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st) {
  if (!t.quit_possible || t.m.mt != MT_DFA_SUFFIX) return launch_lane_search(mode, b, t.m, t.f, t.r, out, st, t.cus);
  BatchDev bq = b;  // quit flag: see run_regex
  hipError_t e = scratch_malloc((void **)&bq.quit_flag, 4, st);
  if (e == hipSuccess) e = hipMemsetAsync(bq.quit_flag, 0, 4, st);
  if (e == hipSuccess) e = launch_lane_search(mode, bq, t.m, t.f, t.r, out, st, t.cus);
  if (e == hipSuccess) e = run_pike(mode, true, bq, t, out, st);
  if (bq.quit_flag) {
    hipError_t e2 = scratch_free(bq.quit_flag, st);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

// The big-DFA kernel runs one lane per haystack: for batches that fill the
// device (a handful of long haystacks stay on the Pike VM, which spreads one
// haystack over a wave).  RURE_AMD_BIG=2 forces it (tests), =0 keeps the
// Pike VM (A/B; read per call).
bool big_batch(const BatchDev &b, const DevTables &t) {
  const char *env = getenv("RURE_AMD_BIG");
  if (env && env[0] == '2') return true;
  if (env && env[0] == '0') return false;
  return b.count >= (uint64_t)t.cus * 64;
}

hipError_t run_regex(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st, int dfa_grid,
                     const FwdDfaDev *iter = nullptr) {
  if (lane_search_ok(t)) return run_lane_search(mode, b, t, out, st);
  if (!t.has_dfa && big_batch(b, t) && big_device(t)) return launch_big_dfa(mode, b, t.bf, t.br, out, st, t.cus);
  if (!t.has_dfa) return run_pike(mode, false, b, t, out, st);
  uint64_t chunk = 0;
  if (iter && long_batch(mode, b, t, &chunk) && !(t.anchored_rev && b.start != 0))
    return launch_long_scan(mode, b, *iter, t.r, chunk, out, st, t.cus);
  if (!t.quit_possible) return run_dfa_step(mode, b, t, out, st, dfa_grid, nullptr);
  // the DFA kernels flag a quit; the Pike VM fallback returns at once without
  BatchDev bq = b;
  hipError_t e = scratch_malloc((void **)&bq.quit_flag, 4, st);
  if (e == hipSuccess) e = hipMemsetAsync(bq.quit_flag, 0, 4, st);
  if (e == hipSuccess) e = run_dfa_step(mode, bq, t, out, st, dfa_grid, nullptr);
  if (e == hipSuccess) e = run_pike(mode, true, bq, t, out, st);
  if (bq.quit_flag) {
    hipError_t e2 = scratch_free(bq.quit_flag, st);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

// First batched use of a core-form set on a device: count core visits over a
// sample of the batch, re-rank the cores so the LDS table holds the visited
// ones, and upload the re-ranked tables.  Costs one host sync, once.
bool adapt_cores(rure_set *rs, DevTables *t, const BatchDev &b, hipStream_t st, std::string *err) {
  std::lock_guard<std::mutex> g(rs->mu);
  if (t->cores_adapted) return true;
  t->cores_adapted = true;
  const CoreSet &cs = rs->cores;
  const uint64_t sample = std::min<uint64_t>(b.count, 16384);
  // visits per core and reports per mask (mask ids: cs.mid) over a sample
  unsigned int *visits = nullptr;
  uint16_t *mid = nullptr;
  const size_t nm = cs.masks.size() + 1;
  if (!hip_ok(scratch_malloc((void **)&visits, (cs.ncores + nm) * 4, st), err)) return false;
  if (!hip_ok(scratch_malloc((void **)&mid, cs.mid.size() * 2, st), err)) return false;
  std::vector<unsigned int> h(cs.ncores + nm);
  SetCoreDev pc = t->c;
  pc.mid = mid;
  bool ok = hip_ok(hipMemsetAsync(visits, 0, (cs.ncores + nm) * 4, st), err) &&
            hip_ok(hipMemcpyAsync(mid, cs.mid.data(), cs.mid.size() * 2, hipMemcpyHostToDevice, st), err) &&
            hip_ok(launch_core_profile(b, pc, sample, visits, visits + cs.ncores, st, t->cus), err) &&
            hip_ok(hipMemcpyAsync(h.data(), visits, h.size() * 4, hipMemcpyDeviceToHost, st), err) &&
            hip_ok(scratch_free(visits, st), err) && hip_ok(scratch_free(mid, st), err) &&
            hip_ok(hipStreamSynchronize(st), err);
  if (!ok) return false;
  std::vector<uint64_t> w(cs.ncores, 0);
  for (uint32_t r = 0; r < cs.ncores; ++r) w[cs.order[r]] = h[r];
  std::unordered_map<uint64_t, uint64_t> mw;
  for (size_t i = 1; i < nm; ++i) mw[cs.masks[i - 1]] = h[cs.ncores + i];
  CoreSet c2;
  if (!build_set_cores(rs->dfa, core_lds_budget(), &c2, &w, &mw)) return true;  // keep the BFS ranking
  Blob bl;
  size_t c_lds = bl.add(c2.lds.data(), c2.lds.size());
  size_t c_core = bl.add(c2.gcore.data(), c2.gcore.size() * 2);
  size_t c_out = bl.add(c2.gout.data(), c2.gout.size() * 8);
  size_t c_eof = bl.add(c2.eof.data(), c2.eof.size() * 8);
  size_t c_start = bl.add(c2.start, 256);
  DevTables tmp;
  if (!upload_blob(bl, &tmp, err)) return false;
  uint8_t *base = (uint8_t *)tmp.blob;
  SetCoreDev c = t->c;
  c.lds_image = base + c_lds;
  c.lds_bytes = (uint32_t)c2.lds.size();
  c.hot = c2.hot;
  c.K = c2.K;
  c.gcore = (const uint16_t *)(base + c_core);
  c.gout = (const uint64_t *)(base + c_out);
  c.eof = (const uint64_t *)(base + c_eof);
  c.start = (const uint16_t *)(base + c_start);
  c.dead = c2.dead;
  c.quit = c2.quit;
  c.mt_off = c2.mt_off;
  if (t->core_blob) (void)hipFree(t->core_blob);
  t->core_blob = tmp.blob;
  t->c = c;
  return true;
}

// exec.rs:998-1038 many_matches_at for a batch.
hipError_t run_set(const BatchDev &b, const DevTables &t, uint64_t *out, hipStream_t st, int dfa_grid) {
  if (!t.has_dfa) return run_pike(MODE_SET, false, b, t, out, st);
  if (!t.quit_possible)
    return t.use_cores ? launch_set_cores(b, t.c, out, st, t.cus) : launch_dfa_set(b, t.s, out, st, dfa_grid);
  BatchDev bq = b;  // quit flag: see run_regex
  hipError_t e = scratch_malloc((void **)&bq.quit_flag, 4, st);
  if (e == hipSuccess) e = hipMemsetAsync(bq.quit_flag, 0, 4, st);
  if (e == hipSuccess)
    e = t.use_cores ? launch_set_cores(bq, t.c, out, st, t.cus) : launch_dfa_set(bq, t.s, out, st, dfa_grid);
  if (e == hipSuccess) e = run_pike(MODE_SET, true, bq, t, out, st);
  if (bq.quit_flag) {
    hipError_t e2 = scratch_free(bq.quit_flag, st);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

// exec.rs:524-596 read_captures_at for a batch.  One group (two slots): the
// plain find.  Otherwise the DFA's (start, end) per haystack (the quit marker
// kept, not resolved), then the Pike VM with slots: from the match start over
// the text up to two characters past the match end, or over the whole
// haystack where the DFA quit and for anchored-start programs.  A regex whose
// DFA does not materialise takes its bounds from the Pike VM (the reference's
// lazy DFA would have produced them).
hipError_t run_captures(const BatchDev &b, const DevTables &t, uint64_t *slots, uint32_t ns, hipStream_t st,
                        int dfa_grid) {
  if (ns <= 2) return run_regex(MODE_FIND, b, t, slots, st, dfa_grid);
  hipError_t e = hipSuccess;
  uint64_t *found = nullptr;
  if (!t.n.anchored) {
    if ((e = scratch_malloc((void **)&found, b.count * 16, st)) != hipSuccess) return e;
    e = lane_search_ok(t) ? launch_lane_search(MODE_FIND, b, t.m, t.f, t.r, found, st, t.cus)
        : t.has_dfa       ? run_dfa_step(MODE_FIND, b, t, found, st, dfa_grid, nullptr)
                          : run_pike(MODE_FIND, false, b, t, found, st);
  }
  const size_t wb = caps_wave_bytes(t.n.nleaves, ns);
  const bool in_lds = wb <= kNfaLdsMax;
  const size_t per_cu = in_lds ? std::max<size_t>(1, std::min<size_t>(32, (160u * 1024u) / wb)) : 4;
  size_t g = std::min<size_t>(b.count, (size_t)t.cus * per_cu);
  if (!in_lds) g = std::min<size_t>(g, (256u << 20) / wb);  // bound the scratch (wide programs: MiBs per wave)
  const int grid = (int)std::max<size_t>(1, g);
  void *scratch = nullptr;
  if (e == hipSuccess && !in_lds) e = scratch_malloc(&scratch, wb * (size_t)grid, st);
  if (e == hipSuccess) e = launch_captures(b, t.n, found, slots, ns, scratch, st, grid);
  if (scratch) { hipError_t e2 = scratch_free(scratch, st); if (e == hipSuccess) e = e2; }
  if (found) { hipError_t e2 = scratch_free(found, st); if (e == hipSuccess) e = e2; }
  return e;
}

bool to_batch(const rure_amd_batch *b, BatchDev *o) {
  if (!b || (!b->haystack && b->count > 0)) return false;
  o->hay = b->haystack;
  o->offs = b->offsets;
  o->stride = b->stride;
  o->length = b->length;
  o->count = b->count;
  o->start = b->start;
  o->quit_flag = nullptr;
  return true;
}

const uint64_t kQuit = ~0ull - 1;

// Runs one regex over one host haystack on the GPU (single-call entry points).
// mode: MODE_FIND / MODE_ISMATCH / MODE_SHORTEST.  Returns false if no match.
bool single_call(rure *re, int mode, const uint8_t *hay, size_t len, size_t start, uint64_t *r0, uint64_t *r1) {
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) die(err);
  uint64_t chunk;
  BatchDev probe{nullptr, nullptr, len, len, 1, start};
  const FwdDfaDev *iter = long_batch(mode, probe, *t, &chunk) ? iter_device(re, *t, &err) : nullptr;  // locks re->mu
  std::lock_guard<std::mutex> g(re->mu);
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), &err)) die(err);
  if (!re->stage.ensure(d, len, &err)) die(err);
  hipStream_t st = re->stage.stream;
  if (len && !hip_ok(hipMemcpyAsync(re->stage.hay, hay, len, hipMemcpyHostToDevice, st), &err)) die(err);
  BatchDev b{re->stage.hay, nullptr, len, len, 1, start};
  if (!hip_ok(run_regex(mode, b, *t, re->stage.res, st, 1, iter), &err)) die(err);
  uint64_t out[2] = {~0ull, ~0ull};
  size_t nbytes = mode == MODE_FIND ? 16 : mode == MODE_SHORTEST ? 8 : 1;
  if (!hip_ok(hipMemcpyAsync(out, re->stage.res, nbytes, hipMemcpyDeviceToHost, st), &err)) die(err);
  if (!hip_ok(hipStreamSynchronize(st), &err)) die(err);
  if (mode == MODE_ISMATCH) {
    uint8_t v = (uint8_t)(out[0] & 0xFF);
    if (v > 1) die("internal error: unresolved DFA quit");
    return v == 1;
  }
  if (out[0] == kQuit || (mode == MODE_FIND && out[1] == kQuit)) die("internal error: unresolved DFA quit");
  if (out[0] == ~0ull) return false;
  *r0 = out[0];
  if (r1) *r1 = out[1];
  return true;
}

uint64_t set_single_call(rure_set *rs, const uint8_t *hay, size_t len, size_t start) {
  std::string err;
  DevTables *t = set_device(rs, &err);
  if (!t) die(err);
  std::lock_guard<std::mutex> g(rs->mu);
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), &err)) die(err);
  if (!rs->stage.ensure(d, len, &err)) die(err);
  hipStream_t st = rs->stage.stream;
  if (len && !hip_ok(hipMemcpyAsync(rs->stage.hay, hay, len, hipMemcpyHostToDevice, st), &err)) die(err);
  BatchDev b{rs->stage.hay, nullptr, 0, len, 1, start};
  if (!hip_ok(run_set(b, *t, rs->stage.res, st, 1), &err)) die(err);
  uint64_t out = 0;
  if (!hip_ok(hipMemcpyAsync(&out, rs->stage.res, 8, hipMemcpyDeviceToHost, st), &err)) die(err);
  if (!hip_ok(hipStreamSynchronize(st), &err)) die(err);
  if (out == kQuit) die("internal error: unresolved DFA quit");
  return out;
}

void fill_prog_info(const Program &p, rure_amd_prog_info *info) {
  info->ninsts = (uint32_t)p.insts.size();
  info->start = p.start;
  info->nmatches = (uint32_t)p.matches.size();
  info->ncaptures = (uint32_t)p.capture_names.size();
  info->anchored_start = p.anchored_start;
  info->anchored_end = p.anchored_end;
  info->has_unicode_word_boundary = p.has_unicode_word_boundary;
  info->is_reverse = p.is_reverse;
  memcpy(info->byte_classes, p.byte_classes, 256);
}

int64_t export_prog(const Program &p, rure_amd_prog_info *info, rure_amd_inst *insts, size_t cap) {
  if (info) fill_prog_info(p, info);
  if (insts) {
    size_t n = std::min(cap, p.insts.size());
    for (size_t i = 0; i < n; ++i) {
      const Inst &in = p.insts[i];
      insts[i] = rure_amd_inst{in.op, in.look, in.lo, in.hi, in.x, in.y};
    }
  }
  return (int64_t)p.insts.size();
}

void fill_info(const DenseDfa &d, const Program &p, uint32_t hot, rure_amd_dfa_info *info, const PackedFwd *pf = nullptr) {
  info->ok = 1;
  info->states = d.nstates;
  info->raw_states = d.raw_states;
  info->normal = d.n_normal;
  info->match_end = d.n_match_end;
  info->dead = d.dead;
  info->quit = d.quit;
  info->hot = (int32_t)hot;
  info->byte_classes = p.num_byte_classes();
  info->insts = (int32_t)p.insts.size();
  info->fast_stride = pf ? (int32_t)pf->stride : 1;
  uint32_t k = 1;
  if (pf && pf->stride > 1) while (true) { uint32_t q = 1; for (uint32_t i = 0; i < pf->stride; ++i) q *= k; if (q >= pf->P) break; ++k; }
  info->fast_classes = pf && pf->stride > 1 ? (int32_t)k : 0;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ errors
rure_error *rure_error_new(void) { return new rure_error(); }
void rure_error_free(rure_error *err) { delete err; }
const char *rure_error_message(rure_error *err) { return err ? err->msg.c_str() : ""; }

// ----------------------------------------------------------------- options
rure_options *rure_options_new(void) { return new rure_options(); }
void rure_options_free(rure_options *o) { delete o; }
void rure_options_size_limit(rure_options *o, size_t limit) { if (o) o->size_limit = limit; }
void rure_options_dfa_size_limit(rure_options *o, size_t limit) { if (o) o->dfa_size_limit = limit; }

// ----------------------------------------------------------------- compile
rure *rure_compile(const uint8_t *pattern, size_t length, uint32_t flags, rure_options *options,
                   rure_error *error) {
  std::string pat((const char *)pattern, length);
  {
    size_t i = 0;
    while (i < length) {  // rure.rs:101-112: the pattern must be UTF-8
      uint32_t cp; size_t l;
      if (!decode_utf8(pattern + i, length - i, &cp, &l)) {
        if (error) error->msg = "pattern is not valid UTF-8 (invalid byte at offset " + std::to_string(i) + ")";
        return nullptr;
      }
      i += l;
    }
  }
  std::unique_ptr<rure> re(new rure());
  re->pattern = pat;
  re->flags = flags;
  if (options) re->opts = *options;
  std::string err;
  if (!parse_regex(pat, syntax_flags(flags), &re->expr, &err)) {
    if (error) error->msg = err;
    return nullptr;
  }
  std::vector<Expr> es{re->expr};
  CompileOptions o;
  o.size_limit = re->opts.size_limit;
  // exec.rs:288-306: nfa (bytes), dfa (.*? prefixed), dfa_reverse
  if (!compile_program(es, o, &re->nfa, &err)) { if (error) error->msg = err; return nullptr; }
  o.dfa = true;
  if (!compile_program(es, o, &re->fwd, &err)) { if (error) error->msg = err; return nullptr; }
  o.reverse = true;
  if (!compile_program(es, o, &re->rev, &err)) { if (error) error->msg = err; return nullptr; }
  re->fwd.dfa_size_limit = re->rev.dfa_size_limit = re->opts.dfa_size_limit;
  re->xl = exec_literals(re->expr);
  handle_created();
  return re.release();
}

rure *rure_compile_must(const char *pattern) {  // rure.rs:76-91
  rure_error err;
  rure *re = rure_compile((const uint8_t *)pattern, strlen(pattern), RURE_DEFAULT_FLAGS, nullptr, &err);
  if (!re) {
    fprintf(stderr, "%s\naborting from rure_compile_must\n", err.msg.c_str());
    abort();
  }
  return re;
}

void rure_free(rure *re) {
  if (!re) return;
  kmer_forget(re);
  for (auto &kv : re->iter_dev) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(kv.first);
    (void)hipFree(kv.second.first);
    (void)hipSetDevice(cur);
  }
  for (auto &kv : re->dev) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(kv.first);
    (void)hipFree(kv.second.blob);
    if (kv.second.big_blob) (void)hipFree(kv.second.big_blob);
    (void)hipSetDevice(cur);
  }
  delete re;
  handle_freed();
}

// ---------------------------------------------------------------- searches
bool rure_is_match(rure *re, const uint8_t *hay, size_t len, size_t start) {
  uint64_t a;
  return single_call(re, MODE_ISMATCH, hay, len, start, &a, nullptr);
}

bool rure_find(rure *re, const uint8_t *hay, size_t len, size_t start, rure_match *m) {
  uint64_t s, e;
  if (!single_call(re, MODE_FIND, hay, len, start, &s, &e)) return false;
  if (m) { m->start = (size_t)s; m->end = (size_t)e; }
  return true;
}

bool rure_shortest_match(rure *re, const uint8_t *hay, size_t len, size_t start, size_t *end) {
  uint64_t e;
  if (!single_call(re, MODE_SHORTEST, hay, len, start, &e, nullptr)) return false;
  if (end) *end = (size_t)e;
  return true;
}

rure_iter *rure_iter_new(rure *re) {
  rure_iter *it = new rure_iter();
  it->re = re;
  return it;
}
void rure_iter_free(rure_iter *it) { delete it; }

bool rure_iter_next(rure_iter *it, const uint8_t *hay, size_t len, rure_match *m) {  // rure.rs:322-360
  while (true) {
    if (it->last_end > len) return false;
    uint64_t s, e;
    if (!single_call(it->re, MODE_FIND, hay, len, it->last_end, &s, &e)) return false;
    if (s == e) {
      it->last_end += 1;
      if (it->has_last_match && it->last_match == e) continue;
    } else {
      it->last_end = e;
    }
    it->has_last_match = true;
    it->last_match = e;
    if (m) { m->start = (size_t)s; m->end = (size_t)e; }
    return true;
  }
}

// ----------------------------------------------------------------- captures
namespace {

uint32_t capture_slots(rure *re) {
  if (!build_regex(re)) die(re->dfa_err);
  return (uint32_t)(2 * re->nfa.capture_names.size());
}

// One haystack through run_captures (staged like single_call).  slots: ns.
bool captures_call(rure *re, const uint8_t *hay, size_t len, size_t start, uint64_t *slots, uint32_t ns) {
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) die(err);
  if (ns > 2 && !re->nfa_ok) die("captures need the NFA tables, which could not be built");
  std::lock_guard<std::mutex> g(re->mu);
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), &err)) die(err);
  if (!re->stage.ensure(d, len, &err)) die(err);
  hipStream_t st = re->stage.stream;
  if (len && !hip_ok(hipMemcpyAsync(re->stage.hay, hay, len, hipMemcpyHostToDevice, st), &err)) die(err);
  BatchDev b{re->stage.hay, nullptr, len, len, 1, start};
  uint64_t *dev = re->stage.res;
  if (ns > 64 && !hip_ok(scratch_malloc((void **)&dev, (size_t)ns * 8, st), &err)) die(err);
  if (!hip_ok(run_captures(b, *t, dev, ns, st, 1), &err)) die(err);
  if (!hip_ok(hipMemcpyAsync(slots, dev, (size_t)ns * 8, hipMemcpyDeviceToHost, st), &err)) die(err);
  if (dev != re->stage.res && !hip_ok(scratch_free(dev, st), &err)) die(err);
  if (!hip_ok(hipStreamSynchronize(st), &err)) die(err);
  if (slots[0] == kQuit || slots[1] == kQuit) die("internal error: unresolved DFA quit");
  return slots[0] != ~0ull && slots[1] != ~0ull;
}

}  // namespace

rure_captures *rure_captures_new(rure *re) {
  rure_captures *c = new rure_captures();
  c->slots.assign(capture_slots(re), ~0ull);
  return c;
}
void rure_captures_free(rure_captures *c) { delete c; }
size_t rure_captures_len(rure_captures *c) { return c->slots.size() / 2; }

bool rure_captures_at(rure_captures *c, size_t i, rure_match *m) {  // rure.rs:413-433 (Locations::pos)
  if (2 * i + 1 >= c->slots.size()) return false;
  const uint64_t s = c->slots[2 * i], e = c->slots[2 * i + 1];
  if (s == ~0ull || e == ~0ull) return false;
  if (m) { m->start = (size_t)s; m->end = (size_t)e; }
  return true;
}

bool rure_find_captures(rure *re, const uint8_t *hay, size_t len, size_t start, rure_captures *c) {
  std::fill(c->slots.begin(), c->slots.end(), ~0ull);
  return captures_call(re, hay, len, start, c->slots.data(), (uint32_t)c->slots.size());
}

bool rure_iter_next_captures(rure_iter *it, const uint8_t *hay, size_t len, rure_captures *c) {  // rure.rs:363-397
  while (true) {
    if (it->last_end > len) return false;
    if (!rure_find_captures(it->re, hay, len, it->last_end, c)) return false;
    const size_t s = (size_t)c->slots[0], e = (size_t)c->slots[1];
    if (s == e) {
      it->last_end += 1;
      if (it->has_last_match && it->last_match == e) continue;
    } else {
      it->last_end = e;
    }
    it->has_last_match = true;
    it->last_match = e;
    return true;
  }
}

int32_t rure_capture_name_index(rure *re, const char *name) {  // rure.rs:233-240
  if (!build_regex(re)) die(re->dfa_err);
  const auto &names = re->nfa.capture_names;
  for (size_t i = 0; i < names.size(); ++i)
    if (re->nfa.capture_has_name[i] && names[i] == name) return (int32_t)i;
  return -1;
}

rure_iter_capture_names *rure_iter_capture_names_new(rure *re) {
  if (!build_regex(re)) die(re->dfa_err);
  rure_iter_capture_names *it = new rure_iter_capture_names();
  it->names = re->nfa.capture_names;
  return it;
}

void rure_iter_capture_names_free(rure_iter_capture_names *it) {
  for (char *p : it->owned) free(p);
  delete it;
}

bool rure_iter_capture_names_next(rure_iter_capture_names *it, char **name) {  // rure.rs:267-301
  if (!name || it->next >= it->names.size()) return false;
  char *p = strdup(it->names[it->next++].c_str());
  if (!p) return false;
  it->owned.push_back(p);
  *name = p;
  return true;
}

// --------------------------------------------------------------------- sets
rure_set *rure_compile_set(const uint8_t **patterns, const size_t *lens, size_t count, uint32_t flags,
                           rure_options *options, rure_error *error) {
  std::unique_ptr<rure_set> rs(new rure_set());
  rs->flags = flags;
  if (options) rs->opts = *options;
  for (size_t i = 0; i < count; ++i) {
    std::string pat((const char *)patterns[i], lens[i]);
    size_t k = 0;
    while (k < pat.size()) {
      uint32_t cp; size_t l;
      if (!decode_utf8((const uint8_t *)pat.data() + k, pat.size() - k, &cp, &l)) {
        if (error) error->msg = "pattern is not valid UTF-8";
        return nullptr;
      }
      k += l;
    }
    Expr e;
    std::string err;
    if (!parse_regex(pat, syntax_flags(flags), &e, &err)) { if (error) error->msg = err; return nullptr; }
    rs->patterns.push_back(pat);
    rs->exprs.push_back(std::move(e));
  }
  if (rs->exprs.size() == 1) {
    rs->single = rure_compile((const uint8_t *)rs->patterns[0].data(), rs->patterns[0].size(), flags,
                              options, error);
    if (!rs->single) return nullptr;
  } else if (!rs->exprs.empty()) {
    CompileOptions o;
    o.size_limit = rs->opts.size_limit;
    o.dfa = true;
    std::string err;
    if (!compile_program(rs->exprs, o, &rs->fwd, &err)) { if (error) error->msg = err; return nullptr; }
    o.dfa = false;
    if (!compile_program(rs->exprs, o, &rs->nfa, &err)) { if (error) error->msg = err; return nullptr; }
  }
  for (size_t lo = 0; count > 64 && lo < count; lo += 64) {
    rure_set *g = rure_compile_set(patterns + lo, lens + lo, std::min<size_t>(64, count - lo), flags, options, error);
    if (!g) {
      for (rure_set *x : rs->groups) rure_set_free(x);
      rs->groups.clear();
      return nullptr;
    }
    rs->groups.push_back(g);
  }
  handle_created();
  return rs.release();
}

void rure_set_free(rure_set *rs) {
  if (!rs) return;
  free_multi(rs);
  if (rs->single) rure_free(rs->single);
  for (rure_set *g : rs->groups) rure_set_free(g);
  for (auto &kv : rs->dev) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(kv.first);
    (void)hipFree(kv.second.blob);
    if (kv.second.core_blob) (void)hipFree(kv.second.core_blob);
    (void)hipSetDevice(cur);
  }
  delete rs;
  handle_freed();
}

void rure_amd_release_scratch(void) { scratch_release(); }
void rure_amd_scratch_stats(size_t *cached, size_t *live, long *handles) {
  ScratchCache &c = scratch_cache();
  std::lock_guard<std::mutex> g(c.mu);
  if (cached) *cached = c.cached;
  if (live) *live = c.live_bytes;
  if (handles) *handles = g_live_handles.load();
}

size_t rure_set_len(rure_set *rs) { return rs->exprs.size(); }

static uint64_t set_mask_single(rure_set *rs, const uint8_t *hay, size_t len, size_t start) {
  if (rs->exprs.empty()) return 0;  // MatchType::Nothing (exec.rs:276-286)
  if (rs->single) return rure_is_match(rs->single, hay, len, start) ? 1 : 0;  // dfa.rs:556-558
  return set_single_call(rs, hay, len, start);
}

bool rure_set_is_match(rure_set *rs, const uint8_t *hay, size_t len, size_t start) {
  for (rure_set *g : rs->groups)
    if (rure_set_is_match(g, hay, len, start)) return true;
  if (!rs->groups.empty()) return false;
  return set_mask_single(rs, hay, len, start) != 0;
}

bool rure_set_matches(rure_set *rs, const uint8_t *hay, size_t len, size_t start, bool *matches) {
  size_t n = rs->exprs.size();
  for (size_t i = 0; i < n; ++i) matches[i] = false;  // rure.rs:557-562
  if (!rs->groups.empty()) {
    bool any = false;
    for (size_t g = 0; g < rs->groups.size(); ++g) any |= rure_set_matches(rs->groups[g], hay, len, start, matches + 64 * g);
    return any;
  }
  uint64_t m = set_mask_single(rs, hay, len, start);
  for (size_t i = 0; i < n; ++i) matches[i] = (m >> i) & 1;
  return m != 0;
}

// ------------------------------------------------------------------ batches
// MatchType::Literal (exec.rs:1148-1166 -> find_literals, exec.rs:601-625):
// a regex that is a finite string set can answer find / is_match from its
// literals instead of the DFA.  On the GPU that wins for a few literals
// (tools/lit_find_bench.py, find over 262144 x 2000 B of sherlock text,
// literal engine vs DFA: 1 word 0.19 vs 0.22 ms, 3 words 0.19 vs 0.32,
// 4 words 0.24 vs 0.30, 8 words 0.24 vs 0.29, 2 rare words 0.29 vs 0.29;
// 16 words 0.30 vs 0.25 and 64 words 0.76 vs 0.63 favour the DFA, whose
// lookups stay one LDS read per byte while candidate verification grows with
// the literal count), so by default it runs for at most kLitFindMax
// literals, on batches of many haystacks (few long ones keep the chunked DFA
// scan).  RURE_AMD_LIT=1 / 0 forces it on / off.
static constexpr size_t kLitFindMax = 8;
static const FwdDfaDev *literal_engine(int mode, rure *re, DevTables &t, const BatchDev &b) {
  uint64_t chunk;
  const char *env = getenv("RURE_AMD_LIT");
  if (env && env[0] != '1') return nullptr;
  if (t.mt_lane) return nullptr;  // the reference's literal searcher differs from the regex's strings
  if (!env && long_batch(mode, b, t, &chunk)) return nullptr;  // RURE_AMD_LIT=1 forces the literal engine
  {
    // the literal set alone (cheap) before any find_iter DFA is built
    std::lock_guard<std::mutex> g(re->mu);
    if (!re->iter_built && !re->lits_done) re->lit_ok = extract_literals(re->nfa, kLitMax, kLitLen, &re->lits);
    re->lits_done = true;
    if (!re->lit_ok || (!env && re->lits.lits.size() > kLitFindMax)) return nullptr;
  }
  std::string err;
  const FwdDfaDev *fi = iter_device(re, t, &err);
  return fi && fi->lit_n ? fi : nullptr;
}

int rure_amd_find_batch(rure *re, const rure_amd_batch *batch, rure_match *out, void *stream) {
  static_assert(sizeof(rure_match) == 16, "rure_match layout");
  BatchDev b;
  if (!re || !to_batch(batch, &b) || (!out && b.count)) return RURE_AMD_ERR_ARG;
  if (b.count == 0) return RURE_AMD_OK;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  if (const FwdDfaDev *lit = literal_engine(MODE_FIND, re, *t, b))
    return launch_lit_find(MODE_FIND, b, *lit, out, (hipStream_t)stream) == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
  int grid = grid_for(b.count, t->f.lds_bytes, t->cus);
  uint64_t chunk;
  const FwdDfaDev *iter = long_batch(MODE_FIND, b, *t, &chunk) ? iter_device(re, *t, &err) : nullptr;
  if (run_regex(MODE_FIND, b, *t, out, (hipStream_t)stream, grid, iter) != hipSuccess) return RURE_AMD_ERR_HIP;
  return RURE_AMD_OK;
}

int rure_amd_compact_matches(const rure_match *found, size_t n, uint64_t base, uint64_t *records, size_t capacity,
                             uint64_t *count, void *stream) {
  if ((!found && n) || (!records && capacity) || !count) return RURE_AMD_ERR_ARG;
  return launch_compact_matches((const uint64_t *)found, n, base, records, capacity, count, (hipStream_t)stream) ==
                 hipSuccess
             ? RURE_AMD_OK
             : RURE_AMD_ERR_HIP;
}

size_t rure_amd_captures_len(rure *re) { return re ? capture_slots(re) / 2 : 0; }

int rure_amd_captures_batch(rure *re, const rure_amd_batch *batch, size_t *slots, void *stream) {
  static_assert(sizeof(size_t) == 8, "64-bit slots");
  BatchDev b;
  if (!re || !to_batch(batch, &b) || (!slots && b.count)) return RURE_AMD_ERR_ARG;
  if (b.count == 0) return RURE_AMD_OK;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  const uint32_t ns = capture_slots(re);
  if (ns > 2 && !re->nfa_ok) return RURE_AMD_ERR_DFA;
  int grid = grid_for(b.count, t->f.lds_bytes, t->cus);
  if (run_captures(b, *t, (uint64_t *)slots, ns, (hipStream_t)stream, grid) != hipSuccess) return RURE_AMD_ERR_HIP;
  return RURE_AMD_OK;
}

int rure_amd_is_match_batch(rure *re, const rure_amd_batch *batch, uint8_t *out, void *stream) {
  BatchDev b;
  if (!re || !to_batch(batch, &b) || (!out && b.count)) return RURE_AMD_ERR_ARG;
  if (b.count == 0) return RURE_AMD_OK;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  if (const FwdDfaDev *lit = literal_engine(MODE_ISMATCH, re, *t, b))
    return launch_lit_find(MODE_ISMATCH, b, *lit, out, (hipStream_t)stream) == hipSuccess ? RURE_AMD_OK
                                                                                      : RURE_AMD_ERR_HIP;
  int grid = grid_for(b.count, t->f.lds_bytes, t->cus);
  uint64_t chunk;
  const FwdDfaDev *iter = long_batch(MODE_ISMATCH, b, *t, &chunk) ? iter_device(re, *t, &err) : nullptr;
  if (run_regex(MODE_ISMATCH, b, *t, out, (hipStream_t)stream, grid, iter) != hipSuccess) return RURE_AMD_ERR_HIP;
  return RURE_AMD_OK;
}

int rure_amd_shortest_match_batch(rure *re, const rure_amd_batch *batch, size_t *end, void *stream) {
  BatchDev b;
  if (!re || !to_batch(batch, &b) || (!end && b.count)) return RURE_AMD_ERR_ARG;
  if (b.count == 0) return RURE_AMD_OK;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  int grid = grid_for(b.count, t->f.lds_bytes, t->cus);
  uint64_t chunk;
  const FwdDfaDev *iter = long_batch(MODE_SHORTEST, b, *t, &chunk) ? iter_device(re, *t, &err) : nullptr;
  if (run_regex(MODE_SHORTEST, b, *t, end, (hipStream_t)stream, grid, iter) != hipSuccess) return RURE_AMD_ERR_HIP;
  return RURE_AMD_OK;
}

namespace {

// One set of at most 64 patterns (>= 2) into one mask word per haystack.
int set_batch_word(rure_set *rs, const BatchDev &b, uint64_t *mask, hipStream_t stream) {
  std::string err;
  DevTables *t = set_device(rs, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  if (t->use_cores && !t->cores_adapted && !adapt_cores(rs, t, b, stream, &err)) return RURE_AMD_ERR_HIP;
  int grid = grid_for(b.count, t->s.lds_bytes, t->cus);
  if (run_set(b, *t, mask, stream, grid) != hipSuccess) return RURE_AMD_ERR_HIP;
  return RURE_AMD_OK;
}

// Group g (patterns [64 g, 64 g + len)) into word g of mask (words per haystack).
// ------------------------------------------------- sets as one pass (groups)
// A set of more than 64 patterns is searched as its 64-pattern groups
// (rure_set::groups), one pass over the batch per group.  With
// RURE_AMD_SET_MULTI=1, build_multi puts every group's core-form automaton
// in one LDS image and set_multi.hip steps all of them over each haystack
// read once; RURE_AMD_SET_CHAINS=G (2..4) splits a set of at most 64
// patterns into G groups the same way.  Measured (tools/bigset_bench.py,
// DESIGN.md §4.3): the chains share the VALU and LDS issue slots the single
// chain already saturates, and the split LDS holds fewer hot cores, so one
// pass is slower (C4 as 2 chains 1.50 vs 0.64 ms; 100 patterns 4.95 vs
// 1.39 ms per-group) though it reads the text once; per-group passes stay
// the default.
}  // namespace
struct MultiSet {
  bool built = false, ok = false;
  std::vector<rure_set *> owned;   // split groups (RURE_AMD_SET_CHAINS), freed with the set
  std::vector<rure_set *> parts;
  std::vector<uint32_t> word, shift;
  std::vector<CoreSet> cores;
  std::vector<uint8_t> lds;
  MultiCoreDev proto{};            // offsets and scalars; pointers filled per device
  bool quit = false;               // some group can quit: Pike VM fallback passes
  double coverage = 1.0;           // smallest share of sampled visits in a group's hot cores
  std::map<int, std::pair<void *, MultiCoreDev>> dev;
};
namespace {

int set_chains() {
  const char *v = getenv("RURE_AMD_SET_CHAINS");
  return v ? std::max(1, std::min(kMultiMaxGroups, atoi(v))) : 1;
}

int device_cus_cached() {
  int d = 0;
  (void)hipGetDevice(&d);
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(d);
  if (it != cache.end()) return it->second;
  return cache[d] = device_cus(d);
}

void free_multi(rure_set *rs) {
  MultiSet *m = rs->multi;
  if (!m) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto &kv : m->dev) {
    (void)hipSetDevice(kv.first);
    (void)hipFree(kv.second.first);
  }
  (void)hipSetDevice(cur);
  for (rure_set *x : m->owned) rure_set_free(x);
  delete m;
  rs->multi = nullptr;
}

bool multi_fail(int why) {  // diagnostic (RURE_AMD_MULTI_DEBUG): which rule declined one pass
  if (getenv("RURE_AMD_MULTI_DEBUG")) fprintf(stderr, "set_multi: not built (%d)\n", why);
  return false;
}

bool build_multi_locked(rure_set *rs, MultiSet *m, std::string *err, const std::vector<std::string> *sample,
                        size_t sample_start) {
  const char *on = getenv("RURE_AMD_SET_MULTI");
  if (!(on && on[0] == '1')) return multi_fail(1);
  if (!rs->groups.empty()) {
    for (size_t g = 0; g < rs->groups.size(); ++g) {
      m->parts.push_back(rs->groups[g]);
      m->word.push_back((uint32_t)g);
      m->shift.push_back(0);
    }
  } else {
    const int G = set_chains();
    const size_t n = rs->exprs.size();
    if (G < 2 || n < (size_t)G) return multi_fail(2);
    const size_t per = (n + G - 1) / G;
    for (size_t lo = 0; lo < n; lo += per) {
      const size_t cnt = std::min(per, n - lo);
      std::vector<const uint8_t *> ps;
      std::vector<size_t> ls;
      for (size_t i = lo; i < lo + cnt; ++i) {
        ps.push_back((const uint8_t *)rs->patterns[i].data());
        ls.push_back(rs->patterns[i].size());
      }
      rure_error e;
      rure_set *x = rure_compile_set(ps.data(), ls.data(), cnt, rs->flags, &rs->opts, &e);
      if (!x) { if (err) *err = e.msg; return multi_fail(3); }
      m->owned.push_back(x);
      m->parts.push_back(x);
      m->word.push_back(0);
      m->shift.push_back((uint32_t)lo);
    }
  }
  const int G = (int)m->parts.size();
  if (G < 2 || G > kMultiMaxGroups) return multi_fail(4);
  for (rure_set *x : m->parts)
    if (x->single || !build_set_dfa(x)) return multi_fail(5);
  // quit states (Unicode \b): the Pike VM redoes the words a lane quit in,
  // with each group's NFA (one word each) or the whole set's (split sets)
  if (rs->groups.empty() && !rs->nfa_ok) return multi_fail(6);  // (built by multi_device before the lock)
  // which cores the batch visits (the hot LDS rows) and which masks it
  // reports (the 62 LDS codes): each group's DFA run on the host over a
  // sample of the first batch (one copy + sync, once per set, like
  // adapt_cores)
  std::vector<std::vector<uint64_t>> sw(G);
  std::vector<std::unordered_map<uint64_t, uint64_t>> mw(G);
  if (sample && !sample->empty()) {
    for (int g = 0; g < G; ++g) {
      const DenseDfa &d = m->parts[g]->dfa;
      sw[g].assign(d.nstates, 0);
      for (const std::string &line : *sample) {
        const uint8_t *tx = (const uint8_t *)line.data();
        const size_t len = line.size();
        if (sample_start > len) continue;
        uint32_t c = d.start[start_flag_index_fwd(tx, len, sample_start)];
        for (size_t i = sample_start; i < len && (int)c != d.dead && (int)c != d.quit; ++i) {
          c = d.trans[(size_t)c * 256 + tx[i]];
          ++sw[g][c];
          if (d.now_mask[c]) ++mw[g][d.now_mask[c]];
        }
      }
    }
  }
  // one LDS image for all groups: each group's share of 159 KiB, shrunk
  // until the image fits (class map 512 B, rows, code masks 512 B, start
  // cores 256 B, hot EOF masks 8 B per hot core)
  const size_t L = 159 * 1024;
  size_t bud = L / G;
  m->cores.assign(G, CoreSet());
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  for (int tries = 0;; ++tries) {
    size_t total = 0;
    for (int g = 0; g < G; ++g) {
      m->cores[g] = CoreSet();
      const bool prof = sample && !sample->empty();
      if (!build_set_cores(m->parts[g]->dfa, bud, &m->cores[g], nullptr, prof ? &mw[g] : nullptr,
                           prof ? &sw[g] : nullptr))
        return multi_fail(7);
      const CoreSet &cs = m->cores[g];
      total += 512 + al16((size_t)(cs.hot + 1) * (cs.K + 1) * 2) + 512 + 256 + al16(8 * (size_t)cs.hot);
    }
    if (total <= L) break;
    if (tries > 16 || bud < 16 * 1024) return multi_fail(8);
    bud -= 4 * 1024;
  }
  // The share of the sample's visits that stays in every group's LDS cores
  // (the LDS is split between the groups), for rure_amd_set_multi_info.
  m->coverage = 1.0;
  if (sample && !sample->empty()) {
    for (int g = 0; g < G; ++g) {
      uint64_t tot = 0;
      for (uint64_t v : sw[g]) tot += v;
      const double cov = tot ? (double)m->cores[g].hot_visits / (double)tot : 1.0;
      m->coverage = std::min(m->coverage, cov);
    }
  }
  MultiCoreDev &P = m->proto;
  P = MultiCoreDev{};
  P.G = (uint32_t)G;
  P.split = rs->groups.empty() ? 1u : 0u;
  size_t cur = 0;
  for (int g = 0; g < G; ++g) {
    const CoreSet &cs = m->cores[g];
    MultiGroupDev &d = P.g[g];
    const size_t rows = (size_t)(cs.hot + 1) * (cs.K + 1) * 2;
    d.K = cs.K;
    d.hot = cs.hot;
    d.dead = cs.dead;
    d.quit = cs.quit;
    if (cs.quit != 0xFFFFFFFFu) m->quit = true;
    d.cls_off = (uint32_t)cur;
    d.rows_off = (uint32_t)(cur + 512);
    d.mt_off = (uint32_t)(d.rows_off + al16(rows));
    d.st_off = d.mt_off + 512;
    d.he_off = d.st_off + 256;
    d.word = m->word[g];
    d.shift = m->shift[g];
    const size_t np = m->parts[g]->exprs.size();
    d.all = np >= 64 ? ~0ull : ((1ull << np) - 1);
    cur = d.he_off + al16(8 * (size_t)cs.hot);
    m->lds.resize(cur, 0);
    uint16_t *cm = (uint16_t *)(m->lds.data() + d.cls_off);
    for (int b = 0; b < 256; ++b) cm[b] = (uint16_t)(2 * cs.lds[b]);
    memcpy(m->lds.data() + d.rows_off, cs.lds.data() + 256, rows);
    memcpy(m->lds.data() + d.mt_off, cs.codemask, 512);
    memcpy(m->lds.data() + d.st_off, cs.start, 256);
    memcpy(m->lds.data() + d.he_off, cs.eof.data(), 8 * (size_t)cs.hot);
  }
  m->lds.resize(al16(m->lds.size()), 0);
  P.lds_bytes = (uint32_t)m->lds.size();
  uint32_t words = 0;
  for (int g = 0; g < G; ++g) words = std::max(words, P.g[g].word + 1);
  P.words = words;
  return true;
}

// Host copy of the first haystacks of the batch (the profile sample): at most
// 4096 of them, each cut to its first 4 KiB, at most 4 MiB in all (so a few
// huge haystacks cost a bounded copy).
std::vector<std::string> batch_sample(const BatchDev &b, hipStream_t st) {
  std::vector<std::string> out;
  const uint64_t n = std::min<uint64_t>(b.count, 4096);
  if (!n) return out;
  constexpr uint64_t kPerHay = 4096, kTotal = 4u << 20;
  std::vector<uint64_t> offs(n + 1);
  if (b.offs) {
    if (hipMemcpyAsync(offs.data(), b.offs, (n + 1) * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return out;
  } else {
    for (uint64_t i = 0; i <= n; ++i) offs[i] = i * b.stride;
  }
  std::vector<uint8_t> buf;
  uint64_t total = 0;
  for (uint64_t i = 0; i < n && total < kTotal; ++i) {
    const uint64_t len = b.offs ? offs[i + 1] - offs[i] : b.length;
    const uint64_t take = std::min<uint64_t>({len, kPerHay, kTotal - total});
    buf.resize(take);
    if (take && (hipMemcpyAsync(buf.data(), b.hay + offs[i], take, hipMemcpyDeviceToHost, st) != hipSuccess ||
                 hipStreamSynchronize(st) != hipSuccess))
      return out;
    out.emplace_back((const char *)buf.data(), take);
    total += take;
  }
  return out;
}

const MultiCoreDev *multi_device(rure_set *rs, std::string *err, const BatchDev &b, hipStream_t st) {
  if (rs->groups.empty()) build_set(rs);  // split sets: the whole set's NFA (quit fallback); takes rs->mu
  std::lock_guard<std::mutex> g(rs->mu);
  if (!rs->multi) rs->multi = new MultiSet();
  MultiSet *m = rs->multi;
  if (!m->built) {
    m->built = true;
    // opt-in (RURE_AMD_SET_MULTI=1): the default path never samples
    const char *on = getenv("RURE_AMD_SET_MULTI");
    if (!(on && on[0] == '1')) {
      m->ok = false;
      return nullptr;
    }
    const std::vector<std::string> sample = batch_sample(b, st);
    m->ok = build_multi_locked(rs, m, err, &sample, b.start);
  }
  if (!m->ok) return nullptr;
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  auto it = m->dev.find(d);
  if (it != m->dev.end()) return &it->second.second;
  Blob bl;
  const int G = (int)m->parts.size();
  size_t o_core[kMultiMaxGroups], o_out[kMultiMaxGroups], o_eof[kMultiMaxGroups];
  for (int k = 0; k < G; ++k) {
    const CoreSet &cs = m->cores[k];
    o_core[k] = bl.add(cs.gcore.data(), cs.gcore.size() * 2);
    o_out[k] = bl.add(cs.gout.data(), cs.gout.size() * 8);
    o_eof[k] = bl.add(cs.eof.data(), cs.eof.size() * 8);
  }
  const size_t o_lds = bl.add(m->lds.data(), m->lds.size());
  DevTables tmp;
  if (!upload_blob(bl, &tmp, err)) return nullptr;
  uint8_t *base = (uint8_t *)tmp.blob;
  MultiCoreDev f = m->proto;
  f.lds_image = base + o_lds;
  for (int k = 0; k < G; ++k) {
    f.g[k].gcore = (const uint16_t *)(base + o_core[k]);
    f.g[k].gout = (const uint64_t *)(base + o_out[k]);
    f.g[k].eof = (const uint64_t *)(base + o_eof[k]);
  }
  auto &slot = m->dev[d];
  slot = std::make_pair(tmp.blob, f);
  return &slot.second;
}

// The one-pass kernel, then (only where a lane quit: the Pike kernels read
// the flag first) the Pike VM over the words marked QUITMARK.
int run_set_multi(rure_set *rs, const BatchDev &b, const MultiCoreDev &f, uint64_t *mask, hipStream_t st) {
  MultiSet *m = rs->multi;
  const int cus = device_cus_cached();
  if (getenv("RURE_AMD_MULTI_DEBUG")) {  // diagnostic: the combined image's layout
    fprintf(stderr, "set_multi: G %u words %u split %u lds %u quit %d\n", f.G, f.words, f.split, f.lds_bytes,
            (int)m->quit);
    for (uint32_t g = 0; g < f.G; ++g)
      fprintf(stderr, "  group %u: K %u hot %u dead %u quit %u cls %u rows %u mt %u st %u he %u word %u shift %u\n", g,
              f.g[g].K, f.g[g].hot, f.g[g].dead, f.g[g].quit, f.g[g].cls_off, f.g[g].rows_off, f.g[g].mt_off,
              f.g[g].st_off, f.g[g].he_off, f.g[g].word, f.g[g].shift);
  }
  if (!m->quit) return launch_set_multi(b, f, mask, st, cus) == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
  std::string err;
  BatchDev bq = b;
  hipError_t e = scratch_malloc((void **)&bq.quit_flag, 4, st);
  if (e == hipSuccess) e = hipMemsetAsync(bq.quit_flag, 0, 4, st);
  if (e == hipSuccess) e = launch_set_multi(bq, f, mask, st, cus);
  if (e == hipSuccess && f.split) {
    const DevTables *t = set_device(rs, &err);
    e = t ? run_pike(MODE_SET, true, bq, *t, mask, st) : hipErrorInvalidValue;
  } else {
    for (size_t g = 0; e == hipSuccess && g < m->parts.size(); ++g) {
      const DevTables *t = set_device(m->parts[g], &err);
      if (!t) { e = hipErrorInvalidValue; break; }
      BatchDev bg = bq;
      bg.out_stride = f.words;
      e = run_pike(MODE_SET, true, bg, *t, mask + f.g[g].word, st);
    }
  }
  if (bq.quit_flag) {
    hipError_t e2 = scratch_free(bq.quit_flag, st);
    if (e == hipSuccess) e = e2;
  }
  return e == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
}

int set_batch_group(rure_set *g, const rure_amd_batch *batch, const BatchDev &b, uint64_t *mask, size_t words,
                    size_t w, hipStream_t st) {
  void *tmp = nullptr;
  const bool single = g->single != nullptr;
  if (scratch_malloc(&tmp, b.count * (single ? 1 : 8), st) != hipSuccess) return RURE_AMD_ERR_HIP;
  int rc = single ? rure_amd_is_match_batch(g->single, batch, (uint8_t *)tmp, st)
                  : set_batch_word(g, b, (uint64_t *)tmp, st);
  if (rc == RURE_AMD_OK &&
      launch_mask_column(single ? (const uint8_t *)tmp : nullptr, single ? nullptr : (const uint64_t *)tmp, b.count,
                         mask, words, w, st) != hipSuccess)
    rc = RURE_AMD_ERR_HIP;
  if (scratch_free(tmp, st) != hipSuccess && rc == RURE_AMD_OK) rc = RURE_AMD_ERR_HIP;
  return rc;
}

}  // namespace

int rure_amd_set_matches_batch_words(rure_set *rs, const rure_amd_batch *batch, uint64_t *mask, size_t words,
                                     void *stream) {
  BatchDev b;
  if (!rs || !to_batch(batch, &b) || (!mask && b.count)) return RURE_AMD_ERR_ARG;
  const size_t n = rs->exprs.size();
  if (words < std::max<size_t>(1, (n + 63) / 64)) return RURE_AMD_ERR_ARG;
  if (b.count == 0) return RURE_AMD_OK;
  hipStream_t st = (hipStream_t)stream;
  if (words <= (size_t)kMultiMaxGroups && (!rs->groups.empty() || set_chains() > 1)) {
    std::string err;
    if (const MultiCoreDev *md = multi_device(rs, &err, b, st)) {
      MultiCoreDev f = *md;
      f.words = (uint32_t)words;
      return run_set_multi(rs, b, f, mask, st);
    }
  }
  if (words == 1 && n >= 2) return set_batch_word(rs, b, mask, st);
  if (hipMemsetAsync(mask, 0, b.count * words * 8, st) != hipSuccess) return RURE_AMD_ERR_HIP;
  if (n == 0) return RURE_AMD_OK;  // MatchType::Nothing (exec.rs:276-286)
  if (rs->groups.empty()) return set_batch_group(rs, batch, b, mask, words, 0, st);
  for (size_t g = 0; g < rs->groups.size(); ++g) {
    int rc = set_batch_group(rs->groups[g], batch, b, mask, words, g, st);
    if (rc != RURE_AMD_OK) return rc;
  }
  return RURE_AMD_OK;
}

int rure_amd_set_multi_info(rure_set *rs, uint32_t *groups, uint32_t *lds_bytes, double *coverage) {
  if (!rs) return RURE_AMD_ERR_ARG;
  std::lock_guard<std::mutex> g(rs->mu);
  const MultiSet *m = rs->multi;
  const bool ok = m && m->built && m->ok;
  if (groups) *groups = ok ? m->proto.G : 0;
  if (lds_bytes) *lds_bytes = ok ? m->proto.lds_bytes : 0;
  if (coverage) *coverage = m && m->built ? m->coverage : 0.0;
  return RURE_AMD_OK;
}

int rure_amd_set_matches_batch(rure_set *rs, const rure_amd_batch *batch, uint64_t *mask, void *stream) {
  if (rs && rs->exprs.size() > 64) return RURE_AMD_ERR_ARG;  // use rure_amd_set_matches_batch_words
  return rure_amd_set_matches_batch_words(rs, batch, mask, 1, stream);
}

namespace {

// The batched find_iter (re_trait.rs:197-221) on one stream.
hipError_t run_find_iter(rure *re, DevTables *t, const BatchDev &b, const IterOut &o, hipStream_t st,
                         std::string *err, const IterSpan *sp = nullptr) {
  // DfaAnchoredReverse regexes match only at the end of the text, so the
  // iteration (re_trait.rs:197-221) yields at most the first search's match
  // (the next search starts at the end, where an empty match is the one just
  // reported or skipped).  Searched from `start` > 0, that first search is
  // the reverse DFA over text[start..] (its look-behind differs from the
  // forward scan's); from 0 the chunked path below answers the same.
  if (!sp && t->anchored_rev && b.start > 0 && b.count) {
    uint64_t *found = nullptr;
    hipError_t e = scratch_malloc((void **)&found, b.count * 16, st);
    if (e != hipSuccess) return e;
    e = run_regex(MODE_FIND, b, *t, found, st, grid_for(b.count, t->r.lds_bytes, t->cus));
    if (e == hipSuccess) e = launch_find_to_iter(found, b.count, o.counts, o.matches, o.cap, o.total, st);
    hipError_t e2 = scratch_free(found, st);
    return e != hipSuccess ? e : e2;
  }
  // The reference's Literal / DfaSuffix searches (DevTables::mt_lane): every
  // search of the iteration is one of those, on a wave per haystack (lane 0
  // searches, the wave runs the Pike VM where a DfaSuffix scan quits).
  if (lane_search_ok(*t) && re->nfa_ok)
    return launch_find_iter(b, t->has_dfa ? &t->f : nullptr, t->r, &t->n, false, 0, o, st, t->cus, sp, &t->m);
  // Chunked speculative iteration needs a DFA that cannot quit and a pattern
  // without assertions (see iter_scan.hip); otherwise one wave per haystack.
  const FwdDfaDev *fi = nullptr;
  if (t->has_dfa && !t->quit_possible && re->nfa_ok && re->nt.looks_used == 0) fi = iter_device(re, *t, err);
  if (fi) {
    uint64_t chunk = ~0ull >> 2;
    const uint64_t lim = sp ? std::min<uint64_t>(b.length, sp->hi) : b.length;
    if (!b.offs && lim > b.start && b.count) {
      const uint64_t span = lim - b.start;
      // lanes in flight: 16 waves per CU (tools/iter_sweep.py);
      // RURE_AMD_ITER_LANES (per CU) overrides (tuning)
      uint64_t per_cu = 1024;
      if (const char *v = getenv("RURE_AMD_ITER_LANES")) per_cu = std::max(64, atoi(v));
      const uint64_t target = (uint64_t)t->cus * per_cu;
      const uint64_t per_h = (target + b.count - 1) / b.count;
      chunk = odd_lines(std::max<uint64_t>(4096, (span + per_h - 1) / per_h));
    }
    return launch_find_iter(b, fi, t->r, &t->n, true, chunk, o, st, t->cus, sp);
  }
  if (!re->nfa_ok) return hipErrorInvalidValue;
  return launch_find_iter(b, t->has_dfa ? &t->f : nullptr, t->r, &t->n, false, 0, o, st, t->cus, sp);
}

// find_iter into internal device buffers: counts (n + 1, last 0), their
// exclusive sums moff (n + 1) and the match records; reads the total on the
// host (one sync) and reruns once with an exact buffer if the guess was short.
struct IterBufs {
  uint64_t *counts = nullptr, *moff = nullptr, *m = nullptr, *total = nullptr;
  uint64_t nm = 0;
  hipStream_t st = nullptr;
  ~IterBufs() {
    if (counts) (void)scratch_free(counts, st);
    if (moff) (void)scratch_free(moff, st);
    if (m) (void)scratch_free(m, st);
    if (total) (void)scratch_free(total, st);
  }
};

hipError_t iter_to_device(rure *re, DevTables *t, const BatchDev &b, hipStream_t st, IterBufs *ib, std::string *err) {
  ib->st = st;
  hipError_t e;
  const size_t n = b.count;
  if ((e = scratch_malloc((void **)&ib->counts, (n + 1) * 8, st)) != hipSuccess) return e;
  if ((e = scratch_malloc((void **)&ib->moff, (n + 1) * 8, st)) != hipSuccess) return e;
  if ((e = scratch_malloc((void **)&ib->total, 8, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(ib->counts, 0, (n + 1) * 8, st)) != hipSuccess) return e;
  const uint64_t bytes = b.offs ? 0 : (uint64_t)b.count * b.length;
  uint64_t cap = std::max<uint64_t>(1024, bytes / 64 + 2 * n);
  for (int pass = 0; pass < 2; ++pass) {
    if ((e = scratch_malloc((void **)&ib->m, cap * 16, st)) != hipSuccess) return e;
    IterOut o{ib->counts, ib->m, cap, ib->total};
    if ((e = run_find_iter(re, t, b, o, st, err)) != hipSuccess) return e;
    uint64_t tot = 0;
    if ((e = hipMemcpyAsync(&tot, ib->total, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    ib->nm = tot;
    if (tot <= cap) break;
    (void)scratch_free(ib->m, st);
    ib->m = nullptr;
    cap = tot;
  }
  return exclusive_scan_u64(ib->counts, ib->moff, n + 1, st);
}

}  // namespace

int rure_amd_find_iter_batch(rure *re, const rure_amd_batch *batch, uint64_t *counts, rure_match *matches,
                             size_t capacity, uint64_t *total, void *stream) {
  BatchDev b;
  if (!re || !to_batch(batch, &b) || (!counts && b.count) || !total || (!matches && capacity))
    return RURE_AMD_ERR_ARG;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  if (!t->has_dfa && !re->nfa_ok) return RURE_AMD_ERR_DFA;
  IterOut o{counts, (uint64_t *)matches, capacity, total};
  return run_find_iter(re, t, b, o, (hipStream_t)stream, &err) == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
}

int64_t rure_amd_literals_export(rure *re, uint32_t *lens, uint8_t *bytes, size_t cap) {
  if (!re) return RURE_AMD_ERR_ARG;
  build_iter_dfa(re);
  std::lock_guard<std::mutex> g(re->mu);
  if (!re->lit_ok) return 0;
  const auto &L = re->lits.lits;
  for (size_t x = 0; x < L.size() && x < cap; ++x) {
    if (lens) lens[x] = (uint32_t)L[x].size();
    if (bytes) std::memcpy(bytes + kLitLen * x, L[x].data(), L[x].size());
  }
  return (int64_t)L.size();
}

int64_t rure_amd_shiftand_export(rure *re, uint64_t *mask, uint64_t *init, uint64_t *fin, uint32_t *len) {
  if (!re) return RURE_AMD_ERR_ARG;
  build_iter_dfa(re);
  std::lock_guard<std::mutex> g(re->mu);
  std::vector<uint64_t> m;
  uint64_t i0 = 0, f0 = 0;
  uint32_t l0 = 0, b0 = 0;
  if (!re->lit_ok || !build_shiftand(re->lits, &m, &i0, &f0, &l0, &b0)) return 0;
  if (mask) std::memcpy(mask, m.data(), 256 * 8);
  if (init) *init = i0;
  if (fin) *fin = f0;
  if (len) *len = l0;
  return (int64_t)b0;
}

int rure_amd_find_iter_span(rure *re, const uint8_t *haystack, size_t length, size_t lo, size_t hi,
                            const rure_amd_iter_state *entry, uint64_t *count, rure_match *matches,
                            size_t capacity, rure_amd_iter_state *exit, void *stream) {
  if (!re || (!haystack && length) || lo > hi || hi > length || !count || !exit || (!matches && capacity))
    return RURE_AMD_ERR_ARG;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  if (!t->has_dfa && !re->nfa_ok) return RURE_AMD_ERR_DFA;
  BatchDev b;
  b.hay = haystack;
  b.offs = nullptr;
  b.stride = length;
  b.length = length;
  b.count = 1;
  b.start = lo;
  // hi == length: the span runs to the end of the text, so the iteration
  // may also own the empty match at the very end (re_trait.rs:205-214)
  IterSpan sp{hi == length ? ~0ull : (uint64_t)hi, (const uint64_t *)entry, (uint64_t *)exit,
              hi == length ? (uint64_t)length : ~0ull};
  IterOut o{count, (uint64_t *)matches, capacity, count};
  hipStream_t st = (hipStream_t)stream;
  return run_find_iter(re, t, b, o, st, &err, &sp) == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
}

namespace {
// k-mer probe tables of a regex list (KmerDev), built once per list and
// device: every regex a finite set of strings of one length L <= 8 over an
// alphabet of at most 4 bytes with distinct codes (b >> shift) & 3.
struct KmerCacheEntry {
  std::vector<const rure *> res;
  int dev;
  void *blob;
  KmerDev km;
};
std::mutex g_kmer_mu;
std::vector<KmerCacheEntry> g_kmer;

bool build_kmer(rure *const *res, size_t n, std::vector<uint32_t> *bitmap, std::vector<uint16_t> *mask, KmerDev *km) {
  if (n == 0 || n > 16) return false;
  size_t L = 0;
  bool seen[256] = {false};
  std::vector<uint8_t> alpha;
  for (size_t i = 0; i < n; ++i) {
    rure *re = res[i];
    if (!re->lit_ok || re->lits.lits.empty() || re->lits.minlen != re->lits.maxlen) return false;
    if (L == 0) L = re->lits.minlen;
    if (re->lits.minlen != L) return false;
    for (const std::string &l : re->lits.lits)
      for (unsigned char c : l)
        if (!seen[c]) {
          seen[c] = true;
          alpha.push_back(c);
        }
  }
  if (L == 0 || L > 8 || alpha.size() > 4) return false;
  int shift = -1;
  for (int sh = 0; sh <= 6 && shift < 0; ++sh) {
    uint32_t used = 0;
    bool ok = true;
    for (uint8_t c : alpha) {
      const uint32_t code = (c >> sh) & 3u;
      if (used & (1u << code)) ok = false;
      used |= 1u << code;
    }
    if (ok) shift = sh;
  }
  if (shift < 0) return false;
  km->shift = (uint32_t)shift;
  km->lut = 0;
  km->present = 0;
  for (uint8_t c : alpha) {
    const uint32_t code = (c >> shift) & 3u;
    km->lut |= (uint32_t)c << (8 * code);
    km->present |= 1u << code;
  }
  km->len = L;
  km->cmask = (uint32_t)((1ull << (2 * L)) - 1);
  bitmap->assign(2048, 0);
  mask->assign((size_t)1 << (2 * L), 0);
  for (size_t i = 0; i < n; ++i)
    for (const std::string &l : res[i]->lits.lits) {
      uint32_t code = 0;
      for (size_t j = 0; j < L; ++j) code |= (((uint8_t)l[j] >> shift) & 3u) << (2 * j);
      (*bitmap)[code >> 5] |= 1u << (code & 31);
      (*mask)[code] |= (uint16_t)(1u << i);
    }
  return true;
}

// The cached device tables for this regex list, copied into *out while the
// cache lock is held (an entry's address does not outlive the lock: another
// thread's push_back or kmer_forget moves the vector).  False: not eligible.
bool kmer_device(rure *const *res, size_t n, KmerDev *out) {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return false;
  std::lock_guard<std::mutex> g(g_kmer_mu);
  for (const KmerCacheEntry &e : g_kmer)
    if (e.dev == d && e.res.size() == n && std::equal(e.res.begin(), e.res.end(), res)) {
      if (e.blob) *out = e.km;
      return e.blob != nullptr;
    }
  KmerCacheEntry ent;
  ent.res.assign(res, res + n);
  ent.dev = d;
  ent.blob = nullptr;
  std::vector<uint32_t> bm;
  std::vector<uint16_t> mk;
  if (build_kmer(res, n, &bm, &mk, &ent.km)) {
    Blob b;
    const size_t ob = b.add(bm.data(), bm.size() * 4), om = b.add(mk.data(), mk.size() * 2);
    DevTables tmp;
    std::string err;
    if (upload_blob(b, &tmp, &err)) {
      ent.blob = tmp.blob;
      ent.km.bitmap = (const uint32_t *)((uint8_t *)tmp.blob + ob);
      ent.km.mask = (const uint16_t *)((uint8_t *)tmp.blob + om);
    }
  }
  g_kmer.push_back(ent);
  if (ent.blob) *out = ent.km;
  return ent.blob != nullptr;
}

// rure_free: drop the k-mer tables of lists holding this regex.
void kmer_forget(const rure *re) {
  std::lock_guard<std::mutex> g(g_kmer_mu);
  for (size_t i = 0; i < g_kmer.size();) {
    if (std::find(g_kmer[i].res.begin(), g_kmer[i].res.end(), re) != g_kmer[i].res.end()) {
      if (g_kmer[i].blob) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(g_kmer[i].dev);
        (void)hipFree(g_kmer[i].blob);
        (void)hipSetDevice(cur);
      }
      g_kmer.erase(g_kmer.begin() + i);
    } else {
      ++i;
    }
  }
}
}  // namespace

int rure_amd_find_iter_span_multi(rure *const *res, size_t n, const uint8_t *haystack, size_t length, size_t lo,
                                  size_t hi, const rure_amd_iter_state *const *entry, uint64_t *const *count,
                                  rure_match *const *matches, const size_t *capacity,
                                  rure_amd_iter_state *const *exit, void *stream) {
  if (!res || !count || !exit || (!matches && n) || (!capacity && n) || (!haystack && length) || lo > hi ||
      hi > length)
    return RURE_AMD_ERR_ARG;
  for (size_t i = 0; i < n; ++i)
    if (!res[i] || !count[i] || !exit[i] || (!matches[i] && capacity[i])) return RURE_AMD_ERR_ARG;
  if (n == 0) return RURE_AMD_OK;
  hipStream_t st = (hipStream_t)stream;
  BatchDev b;
  b.hay = haystack;
  b.offs = nullptr;
  b.stride = length;
  b.length = length;
  b.count = 1;
  b.start = lo;
  const uint64_t hcut = hi == length ? ~0ull : (uint64_t)hi, tail = hi == length ? (uint64_t)length : ~0ull;
  // the fused pass: every regex on the chunked Shift-And path
  std::vector<const FwdDfaDev *> fs(n);
  std::vector<const RevDfaDev *> rs(n);
  std::vector<IterOut> os(n);
  std::vector<IterSpan> sps(n);
  std::string err;
  bool fused = n > 1 && hi > lo;
  int cus = 0;
  for (size_t i = 0; i < n && fused; ++i) {
    DevTables *t = regex_device(res[i], &err);
    if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
    const FwdDfaDev *fi = nullptr;
    // a regex the reference searches with its own match type (Literal /
    // DfaSuffix, lane_search_ok) iterates on its own path, as in
    // rure_amd_find_iter_span: the fused pass is a forward-DFA iteration
    if (lane_search_ok(*t)) { fused = false; break; }
    if (t->has_dfa && !t->quit_possible && res[i]->nfa_ok && res[i]->nt.looks_used == 0) fi = iter_device(res[i], *t, &err);
    if (!fi || !fi->sa_len) { fused = false; break; }
    fs[i] = fi;
    rs[i] = &t->r;
    cus = t->cus;
    os[i] = IterOut{count[i], (uint64_t *)matches[i], capacity[i], count[i]};
    sps[i] = IterSpan{hcut, entry ? (const uint64_t *)entry[i] : nullptr, (uint64_t *)exit[i], tail};
  }
  if (fused) {
    // the unit size of run_find_iter (one haystack: the span over the lanes in flight)
    const uint64_t span = std::min<uint64_t>(length, hcut) - lo;
    uint64_t per_cu = 1024;
    if (const char *v = getenv("RURE_AMD_ITER_LANES")) per_cu = std::max(64, atoi(v));
    const uint64_t chunk = odd_lines(std::max<uint64_t>(4096, (span + (uint64_t)cus * per_cu - 1) / ((uint64_t)cus * per_cu)));
    KmerDev kmv;
    const KmerDev *km = kmer_device(res, n, &kmv) ? &kmv : nullptr;
    hipError_t e = launch_find_iter_multi(b, (int)n, fs.data(), rs.data(), chunk, os.data(), st, cus, sps.data(), km);
    if (e == hipSuccess) return RURE_AMD_OK;
    if (e != hipErrorNotSupported) return RURE_AMD_ERR_HIP;
  }
  for (size_t i = 0; i < n; ++i) {
    int rc = rure_amd_find_iter_span(res[i], haystack, length, lo, hi, entry ? entry[i] : nullptr, count[i],
                                     matches[i], capacity[i], exit[i], stream);
    if (rc != RURE_AMD_OK) return rc;
  }
  return RURE_AMD_OK;
}

int rure_amd_replace_batch(rure *re, const rure_amd_batch *batch, const uint8_t *rep, size_t rep_len, size_t limit,
                           uint8_t *out, uint64_t *out_offsets, size_t out_capacity, uint64_t *total, void *stream) {
  BatchDev b;
  if (!re || !to_batch(batch, &b) || !out_offsets || !total || (!out && out_capacity) || (!rep && rep_len))
    return RURE_AMD_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (b.count == 0) return hipMemsetAsync(out_offsets, 0, 8, st) == hipSuccess &&
                           hipMemsetAsync(total, 0, 8, st) == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  if (!t->has_dfa && !re->nfa_ok) return RURE_AMD_ERR_DFA;
  IterBufs ib;
  int64_t *shift = nullptr;
  uint64_t *olen = nullptr;
  uint8_t *drep = nullptr;
  const uint64_t lim = limit == 0 ? ~0ull : (uint64_t)limit;  // replacen: 0 = all
  hipError_t e = iter_to_device(re, t, b, st, &ib, &err);
  if (e == hipSuccess) e = scratch_malloc((void **)&shift, std::max<uint64_t>(ib.nm, 1) * 8, st);
  if (e == hipSuccess) e = scratch_malloc((void **)&olen, (b.count + 1) * 8, st);
  if (e == hipSuccess) e = scratch_malloc((void **)&drep, std::max<size_t>(rep_len, 1), st);
  if (e == hipSuccess && rep_len) e = hipMemcpyAsync(drep, rep, rep_len, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemsetAsync(olen + b.count, 0, 8, st);
  if (e == hipSuccess)
    e = launch_replace_plan(b, ib.counts, ib.moff, ib.m, lim, rep_len, shift, olen, st, t->cus, ib.nm);
  if (e == hipSuccess) e = exclusive_scan_u64(olen, out_offsets, b.count + 1, st);
  if (e == hipSuccess) e = hipMemcpyAsync(total, out_offsets + b.count, 8, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess && out_capacity) {
    const uint64_t hint = b.offs ? out_capacity : std::min<uint64_t>(out_capacity, b.count * b.length + ib.nm * rep_len);
    e = launch_replace_copy(b, out_offsets, ib.counts, ib.moff, ib.m, shift, lim, drep, rep_len, out, out_capacity,
                            hint, st, t->cus);
  }
  if (shift) (void)scratch_free(shift, st);
  if (olen) (void)scratch_free(olen, st);
  if (drep) (void)scratch_free(drep, st);
  return e == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
}

int rure_amd_split_batch(rure *re, const rure_amd_batch *batch, size_t limit, uint64_t *counts, rure_match *pieces,
                         size_t capacity, uint64_t *total, void *stream) {
  BatchDev b;
  if (!re || !to_batch(batch, &b) || (!counts && b.count) || !total || (!pieces && capacity))
    return RURE_AMD_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (b.count == 0) return hipMemsetAsync(total, 0, 8, st) == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
  std::string err;
  DevTables *t = regex_device(re, &err);
  if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
  if (!t->has_dfa && !re->nfa_ok) return RURE_AMD_ERR_DFA;
  IterBufs ib;
  uint64_t *fields = nullptr, *foff = nullptr;
  hipError_t e = iter_to_device(re, t, b, st, &ib, &err);
  if (e == hipSuccess) e = scratch_malloc((void **)&fields, (b.count + 1) * 8, st);
  if (e == hipSuccess) e = scratch_malloc((void **)&foff, (b.count + 1) * 8, st);
  if (e == hipSuccess) e = hipMemsetAsync(fields + b.count, 0, 8, st);
  if (e == hipSuccess)
    e = launch_split(b, ib.counts, ib.moff, ib.m, (uint64_t)limit, fields, foff, (uint64_t *)pieces, capacity, ib.nm,
                     st, t->cus);
  if (e == hipSuccess) e = hipMemcpyAsync(counts, fields, b.count * 8, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(total, foff + b.count, 8, hipMemcpyDeviceToDevice, st);
  if (fields) (void)scratch_free(fields, st);
  if (foff) (void)scratch_free(foff, st);
  return e == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
}

// ------------------------------------------------------------- diagnostics
int rure_amd_dfa_info_get(rure *re, int which, rure_amd_dfa_info *info) {
  if (!re || !info) return RURE_AMD_ERR_ARG;
  memset(info, 0, sizeof(*info));
  if (which == 3 || which == 4) {  // the big (u32 column form) automata
    if (!build_regex(re) || re->dfa_ok) { info->ok = 0; return RURE_AMD_ERR_DFA; }  // only where the u16 DFA fails
    {
      std::lock_guard<std::mutex> g(re->mu);
      if (!re->big_built) {
        re->big_built = true;
        build_big_dfas(re);
      }
    }
    if (!re->big_ok) { info->ok = 0; return RURE_AMD_ERR_DFA; }
    fill_info(which == 3 ? re->bfwd : re->brev, which == 3 ? re->fwd : re->rev, 0, info);
    info->byte_classes = (int32_t)(which == 3 ? re->bfwd.ncol : re->brev.ncol);
    return RURE_AMD_OK;
  }
  if (!build_regex_dfas(re)) { info->ok = 0; return RURE_AMD_ERR_DFA; }
  if (which == 0) fill_info(re->dfwd, re->fwd, re->pf.hot, info, &re->pf);
  else if (which == 1) fill_info(re->drev, re->rev, re->pr.hot, info);
  else {
    if (!build_iter_dfa(re)) { info->ok = 0; return RURE_AMD_ERR_DFA; }
    fill_info(re->dfwd_iter, re->fwd, re->pf_iter.hot, info, &re->pf_iter);
  }
  return RURE_AMD_OK;
}

int rure_amd_set_dfa_info_get(rure_set *rs, rure_amd_dfa_info *info) {
  if (!rs || !info) return RURE_AMD_ERR_ARG;
  memset(info, 0, sizeof(*info));
  if (!build_set_dfa(rs)) { info->ok = 0; return RURE_AMD_ERR_DFA; }
  if (rs->exprs.empty()) return RURE_AMD_OK;
  fill_info(rs->dfa, rs->fwd, rs->pf.hot, info);
  return RURE_AMD_OK;
}

int64_t rure_amd_program_export(rure *re, int which, rure_amd_prog_info *info, rure_amd_inst *insts,
                                size_t cap) {
  if (!re) return RURE_AMD_ERR_ARG;
  const Program &p = which == 0 ? re->fwd : which == 1 ? re->rev : re->nfa;
  return export_prog(p, info, insts, cap);
}

int64_t rure_amd_set_program_export(rure_set *rs, int which, rure_amd_prog_info *info, rure_amd_inst *insts,
                                    size_t cap) {
  if (!rs) return RURE_AMD_ERR_ARG;
  if (rs->single) return rure_amd_program_export(rs->single, which, info, insts, cap);
  if (which == 1) return RURE_AMD_ERR_ARG;
  return export_prog(which == 0 ? rs->fwd : rs->nfa, info, insts, cap);
}

int rure_amd_set_dfa_export(rure_set *rs, uint32_t *trans, uint64_t *eof_mask, uint64_t *now_mask,
                            uint32_t *start) {
  if (!rs) return RURE_AMD_ERR_ARG;
  if (rs->single || rs->exprs.size() < 2) return RURE_AMD_ERR_ARG;
  if (!build_set_dfa(rs)) return RURE_AMD_ERR_DFA;
  const DenseDfa &d = rs->dfa;
  if (trans) memcpy(trans, d.trans.data(), d.trans.size() * 4);
  if (eof_mask) memcpy(eof_mask, d.eof_mask.data(), d.eof_mask.size() * 8);
  if (now_mask) memcpy(now_mask, d.now_mask.data(), d.now_mask.size() * 8);
  if (start) memcpy(start, d.start, sizeof(d.start));
  return RURE_AMD_OK;
}

int rure_amd_set_core_export(rure_set *rs, rure_amd_core_info *info, uint8_t *lds, uint16_t *gcore,
                             uint64_t *gout, uint64_t *eof, uint16_t *start) {
  if (!rs || rs->single || rs->exprs.size() < 2) return RURE_AMD_ERR_ARG;
  if (!build_set_dfa(rs) || !rs->cores.ok) return RURE_AMD_ERR_DFA;
  const CoreSet &cs = rs->cores;
  if (info) *info = rure_amd_core_info{cs.K, cs.ncores, cs.hot, cs.dead, cs.quit, (uint32_t)cs.lds.size()};
  if (lds) memcpy(lds, cs.lds.data(), cs.lds.size());
  if (gcore) memcpy(gcore, cs.gcore.data(), cs.gcore.size() * 2);
  if (gout) memcpy(gout, cs.gout.data(), cs.gout.size() * 8);
  if (eof) memcpy(eof, cs.eof.data(), cs.eof.size() * 8);
  if (start) memcpy(start, cs.start, 256);
  return RURE_AMD_OK;
}

int64_t rure_amd_lex_export(rure *re, uint8_t *table, size_t cap, uint32_t *s0) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  if (table) memcpy(table, re->lex.data(), std::min(cap, re->lex.size()));
  if (s0) *s0 = re->lex_s0;
  return (int64_t)re->lex.size();
}

int rure_amd_first_byte_export(rure *re, uint8_t *bytes) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  if (bytes) memcpy(bytes, re->fb_bytes, 4);
  return (int)re->fb_n;
}

int rure_amd_dfa_strip_export(rure *re, uint32_t *strip) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  if (strip) memcpy(strip, re->dfwd_iter.strip.data(), re->dfwd_iter.strip.size() * 4);
  return RURE_AMD_OK;
}

int rure_amd_dfa_export(rure *re, int which, uint32_t *trans, uint8_t *eof_match, uint32_t *start) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_regex_dfas(re)) return RURE_AMD_ERR_DFA;
  if (which == 2 && !build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  const DenseDfa &d = which == 0 ? re->dfwd : which == 1 ? re->drev : re->dfwd_iter;
  if (trans) memcpy(trans, d.trans.data(), d.trans.size() * 4);
  if (eof_match) memcpy(eof_match, d.eof_match.data(), d.eof_match.size());
  if (start) memcpy(start, d.start, sizeof(d.start));
  return RURE_AMD_OK;
}

static int export_nfa(const NfaTables &nt, rure_amd_nfa_info *info, uint32_t *leaves, uint32_t *cl_off,
                      uint32_t *entries) {
  if (info) {
    info->leaves = (uint32_t)nt.leaves.size();
    info->closures = (uint32_t)nt.cl_off.size() - 1;
    info->entries = (uint32_t)nt.entries.size();
    info->root = nt.root;
    info->nmatch = nt.nmatch;
    info->anchored = nt.anchored_start;
    info->looks = nt.looks_used;
    info->unicode_wb = nt.unicode_wb;
  }
  if (leaves)
    for (size_t i = 0; i < nt.leaves.size(); ++i) {
      const NfaLeaf &l = nt.leaves[i];
      leaves[3 * i] = (uint32_t)l.kind | ((uint32_t)l.lo << 8) | ((uint32_t)l.hi << 16);
      leaves[3 * i + 1] = l.closure;
      leaves[3 * i + 2] = l.slot;
    }
  if (cl_off) memcpy(cl_off, nt.cl_off.data(), nt.cl_off.size() * 4);
  if (entries) memcpy(entries, nt.entries.data(), nt.entries.size() * 8);
  return RURE_AMD_OK;
}

int rure_amd_nfa_export(rure *re, rure_amd_nfa_info *info, uint32_t *leaves, uint32_t *cl_off, uint32_t *entries) {
  if (!re) return RURE_AMD_ERR_ARG;
  build_regex(re);
  if (!re->nfa_ok) return RURE_AMD_ERR_DFA;
  return export_nfa(re->nt, info, leaves, cl_off, entries);
}

int rure_amd_set_nfa_export(rure_set *rs, rure_amd_nfa_info *info, uint32_t *leaves, uint32_t *cl_off,
                            uint32_t *entries) {
  if (!rs) return RURE_AMD_ERR_ARG;
  if (rs->single) return rure_amd_nfa_export(rs->single, info, leaves, cl_off, entries);
  if (rs->exprs.empty()) return RURE_AMD_ERR_ARG;
  build_set(rs);
  if (!rs->nfa_ok) return RURE_AMD_ERR_DFA;
  return export_nfa(rs->nt, info, leaves, cl_off, entries);
}

int rure_amd_nfa_saves_export(rure *re, uint32_t *save_off, uint16_t *save_slot, size_t *n_slots) {
  if (!re) return RURE_AMD_ERR_ARG;
  build_regex(re);
  if (!re->nfa_ok) return RURE_AMD_ERR_DFA;
  if (n_slots) *n_slots = re->nt.save_slot.size();
  if (save_off) memcpy(save_off, re->nt.save_off.data(), re->nt.save_off.size() * 4);
  if (save_slot) memcpy(save_slot, re->nt.save_slot.data(), re->nt.save_slot.size() * 2);
  return RURE_AMD_OK;
}

int rure_amd_uses_dfa(rure *re) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_regex(re)) return RURE_AMD_ERR_DFA;
  return re->dfa_ok ? 1 : 0;
}

int rure_amd_last_fwd_path(void) { return rure_amd::last_fwd_path(); }

namespace {
void ser_lits(const std::vector<Lit> &ls, std::string *o) {
  for (const Lit &l : ls) {
    o->push_back((char)(l.cut ? 1 : 0));
    const uint32_t n = (uint32_t)l.v.size();
    o->append((const char *)&n, 4);
    o->append(l.v);
  }
}
bool de_lits(const uint8_t *in, size_t n, std::vector<Lit> *ls) {
  size_t i = 0;
  while (i < n) {
    if (i + 5 > n) return false;
    Lit l;
    l.cut = in[i] != 0;
    uint32_t k;
    memcpy(&k, in + i + 1, 4);
    i += 5;
    if (i + k > n) return false;
    l.v.assign((const char *)in + i, k);
    i += k;
    ls->push_back(l);
  }
  return true;
}
int64_t put_out(const std::string &s, uint8_t *out, size_t cap) {
  if (out && cap >= s.size()) memcpy(out, s.data(), s.size());
  return (int64_t)s.size();
}
}  // namespace

int64_t rure_amd_literals_syntax(const uint8_t *pattern, size_t length, uint32_t flags, int which, size_t limit_size,
                                 size_t limit_class, uint8_t *out, size_t cap) {
  Expr e;
  std::string err;
  if (!parse_regex(std::string((const char *)pattern, length), syntax_flags(flags), &e, &err)) return RURE_AMD_ERR_ARG;
  Literals l;
  l.limit_size = limit_size;
  l.limit_class = limit_class;
  if (which == 0) l.union_prefixes(e);
  else l.union_suffixes(e);
  std::string o;
  ser_lits(l.lits, &o);
  return put_out(o, out, cap);
}

int64_t rure_amd_literals_op(int op, const uint8_t *in, size_t in_len, uint8_t *out, size_t cap) {
  Literals l;
  if ((in_len && !in) || !de_lits(in, in_len, &l.lits)) return RURE_AMD_ERR_ARG;
  std::string o;
  switch (op) {
    case 0: ser_lits(l.unambiguous_prefixes().lits, &o); break;
    case 1: o = l.longest_common_prefix(); break;
    case 2: o = l.longest_common_suffix(); break;
    case 3: ser_lits(l.unambiguous_suffixes().lits, &o); break;
    default: return RURE_AMD_ERR_ARG;
  }
  return put_out(o, out, cap);
}

int rure_amd_match_info_get(rure *re, rure_amd_match_info *info) {
  if (!re || !info) return RURE_AMD_ERR_ARG;
  memset(info, 0, sizeof(*info));
  const ExecLiterals &x = re->xl;
  info->match_type = x.match_type;
  info->prefix_matcher = x.prefixes.matcher;
  info->suffix_matcher = x.suffixes.matcher;
  info->prefix_len = (uint32_t)x.prefixes.len;
  info->suffix_len = (uint32_t)x.suffixes.len;
  info->prefix_complete = x.prefixes.complete ? 1 : 0;
  info->suffix_complete = x.suffixes.complete ? 1 : 0;
  info->lcp_chars = (uint32_t)x.prefixes.lcp_chars;
  info->lcs_chars = (uint32_t)x.suffixes.lcs_chars;
  info->lcs_bytes = (uint32_t)std::min<size_t>(x.suffixes.lcs.size(), sizeof(info->lcs));
  memcpy(info->lcs, x.suffixes.lcs.data(), info->lcs_bytes);
  return RURE_AMD_OK;
}

int64_t rure_amd_exec_literals_export(rure *re, int which, uint8_t *out, size_t cap) {
  if (!re) return RURE_AMD_ERR_ARG;
  std::string o;
  ser_lits(which == 0 ? re->xl.prefixes.lits.lits : re->xl.suffixes.lits.lits, &o);
  return put_out(o, out, cap);
}

int rure_amd_kernel_timer(int on) { return rure_amd::ktimer_set(on); }
double rure_amd_kernel_timer_read(uint64_t *launches) { return rure_amd::ktimer_read(launches); }

int rure_amd_set_uses_dfa(rure_set *rs) {
  if (!rs) return RURE_AMD_ERR_ARG;
  if (rs->single) return rure_amd_uses_dfa(rs->single);
  if (!rs->groups.empty()) {
    int all = 1;
    for (rure_set *g : rs->groups) {
      int u = rure_amd_set_uses_dfa(g);
      if (u < 0) return u;
      all &= u;
    }
    return all;
  }
  if (!build_set(rs)) return RURE_AMD_ERR_DFA;
  return rs->dfa_ok ? 1 : 0;
}

}  // extern "C"
