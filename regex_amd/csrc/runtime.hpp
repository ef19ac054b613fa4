// Internal interface of the rure_amd runtime (regex_amd/csrc/*.cpp): the
// objects behind the C ABI handles, the device tables of a regex or set, and
// the functions the translation units share.
//   build.cpp     host automata -> packed tables -> device upload (per regex /
//                 set and device), the find_iter engines' images
//   dispatch.cpp  the reference's engine dispatch over batches (exec.rs
//                 find_at / is_match_at / many_matches_at / find_iter), the
//                 set groups, the k-mer table cache
//   scratch.cpp   the device scratch cache (stream-ordered reuse)
//   capi.cpp      the C ABI (include/rure_amd.h): rure.h's API and the
//                 batched device entry points, diagnostics and exports
#pragma once
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

namespace rt {

[[noreturn]] inline void die(const std::string &m) {
  fprintf(stderr, "rure_amd: %s\n", m.c_str());
  fprintf(stderr, "aborting\n");
  abort();
}

inline bool hip_ok(hipError_t e, std::string *err) {
  if (e == hipSuccess) return true;
  if (err) *err = std::string("HIP error: ") + hipGetErrorString(e);
  return false;
}


// the quit marker of a single search's result (the DFA quit, not resolved)
constexpr uint64_t kQuit = ~0ull - 1;

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

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
  // the on-demand forward DFA (lazy_device / run_lazy): its device copy
  // (grown as rows are built) and the reverse DFA it finds starts with
  bool lazy_tried = false, has_lazy = false;
  void *lazy_buf = nullptr, *lazy_rblob = nullptr;
  size_t lazy_cap = 0;
  RevDfaDev lr{};
  bool quit_possible = false;  // the DFA can quit (Unicode \b): Pike VM fallback pass
  bool anchored_rev = false;   // MatchType::DfaAnchoredReverse (exec.rs:1175-1177)
  // The reference's match type where its searches differ from a forward DFA
  // search (literal_sets.hpp): Literal(AnchoredStart), Literal(Unanchored)
  // chosen from complete suffixes (its prefix searcher may be Empty or
  // partial), DfaSuffix.  Those searches run match_types.hip / the wave
  // iteration with `m`.
  MatchDev m{-1, {}, {}, nullptr, 0};
  bool mt_lane = false;
  bool lcs_free = false;    // DfaSuffix: the longest common suffix cannot overlap itself (launch_suffix_long)
  int cus = 256;
};


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


struct Blob {
  std::vector<uint8_t> bytes;
  size_t add(const void *src, size_t n) {
    size_t off = align256(bytes.size());
    bytes.resize(off + align256(n));
    if (n) memcpy(bytes.data() + off, src, n);
    return off;
  }
};


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

struct NfaOffsets { size_t leaves, cl_off, entries, perlw, save_off, save_slot, cl_info, cl_big, cl_boff, cl_sub; };
struct LitOffsets { size_t bytes, off; uint32_t n; };

}  // namespace rt
using namespace rt;

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
  bool rev_ok = false;            // drev materialised (even when dfwd did not)
  bool lazy_tried = false;        // the on-demand forward DFA (lazy_device)
  std::unique_ptr<LazyDfa> lazy;
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
  std::vector<uint8_t> lex4;  // four-byte lexer table (build_lex4), empty if none
  uint32_t lex4_s0 = 0;
  LiteralSet lits;
  std::map<int, std::pair<void *, FwdDfaDev>> iter_dev;
  // the find_iter DFA's ASCII shadow (build_iter_dfa, iter_ascii_device)
  bool iter_a_ok = false;
  DenseDfa dfwd_iter_a;
  PackedFwd pf_iter_a;
  std::vector<uint8_t> lex_a, lex4_a;  // its lexer tables (build_lex / build_lex4), empty if none
  uint32_t lex_a_s0 = 0, lex4_a_s0 = 0;
  // the run engine's byte classes (run_class: the regex is C+), for the
  // find_iter DFA over all bytes and for its ASCII shadow
  bool run_ok = false, run_a_ok = false;
  std::vector<uint32_t> run_cp;  // Unicode C+: C's code point bitmap (0x110000 bits), else empty
  // every match is one byte of a class (class_replace_set): cls_one[b] = b in it
  bool cls_one_ok = false;
  uint8_t cls_one[256] = {0};
  uint8_t run_cls[256] = {0}, run_cls_a[256] = {0};
  std::map<int, std::pair<void *, FwdDfaDev>> iter_dev_a;
  // matches per MiB of text seen by the last replace / split over a
  // fixed-stride batch (iter_to_device's first guess of the match buffer;
  // -1: none yet)
  std::atomic<int64_t> iter_per_mib{-1};
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
};


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

namespace rt {

// ------------------------------------------------------------ build.cpp
// ---------------------------------------------------------- dispatch.cpp
// ----------------------------------------------------------- scratch.cpp
uint32_t uniform_start(const DenseDfa &d);
void build_stride_image(const DenseDfa &d, PackedFwd *p);
bool pack_forward(const DenseDfa &d, PackedFwd *p, std::string *err, bool all = false);
size_t core_lds_budget();
bool build_set_cores(const DenseDfa &d, size_t lds_budget, CoreSet *cs,
                     const std::vector<uint64_t> *weights = nullptr,
                     const std::unordered_map<uint64_t, uint64_t> *mask_weights = nullptr,
                     const std::vector<uint64_t> *state_weights = nullptr);
SyntaxFlags syntax_flags(uint32_t flags);
void build_big_dfas(rure *re);
bool build_regex(rure *re);
bool build_regex_dfas(rure *re);
bool build_set(rure_set *rs);
bool build_set_dfa(rure_set *rs);
NfaOffsets add_nfa(Blob &b, const NfaTables &nt);
void fix_nfa(NfaDev *n, uint8_t *base, const NfaOffsets &o, const NfaTables &nt, bool single);
bool upload_blob(const Blob &b, DevTables *t, std::string *err);
LitOffsets add_litlist(Blob &b, const Literals &l);
bool needs_mt_lane(const ExecLiterals &x);
void set_prefix_skip(const rure *re, FwdDfaDev *f);
DevTables *regex_device(rure *re, std::string *err);
bool big_device(const DevTables &tc);
bool lazy_device(const DevTables &tc);
DevTables *set_device(rure_set *rs, std::string *err);
uint32_t first_byte_rule(const DenseDfa &d, uint32_t ustart1, bool nonempty, uint8_t bytes[4], bool *holds);
bool run_class(const DenseDfa &d, uint32_t ustart1, bool nonempty, uint8_t cls[256], bool ascii);
bool build_lex4(const std::vector<uint8_t> &img, uint32_t s0, std::vector<uint8_t> *out, uint32_t *s0_row);
bool build_lex(const DenseDfa &d, uint32_t ustart1, bool fb_holds, std::vector<uint8_t> *img,
                      uint32_t *s0_idx);
bool build_iter_dfa(rure *re);
bool build_shiftand(const LiteralSet &ls, std::vector<uint64_t> *mask, uint64_t *init, uint64_t *fin,
                           uint32_t *len, uint32_t *bits);
const FwdDfaDev *iter_ascii_device(rure *re, const DevTables &t, std::string *err);
const FwdDfaDev *iter_device(rure *re, const DevTables &t, std::string *err);
bool adapt_cores(rure_set *rs, DevTables *t, const BatchDev &b, hipStream_t st, std::string *err);
int device_cus(int dev);
int grid_for(size_t count, uint32_t lds_bytes, int cus);
int pike_grid(size_t count, bool fallback, const NfaDev &n, int cus);
hipError_t run_pike(int mode, bool fallback, const BatchDev &b, const DevTables &t, void *out, hipStream_t st);
uint64_t odd_lines(uint64_t bytes);
bool long_batch(int mode, const BatchDev &b, const DevTables &t, uint64_t *chunk);
hipError_t run_dfa_step(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st, int dfa_grid,
                        const FwdDfaDev *iter);
bool lane_search_ok(const DevTables &t);
bool suffix_long_ok(const BatchDev &b, const DevTables &t, uint64_t *chunk);
hipError_t run_suffix_long(int mode, const BatchDev &b, const DevTables &t, uint64_t chunk, void *out,
                           hipStream_t st);
hipError_t run_lane_search(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st);
bool big_batch(const BatchDev &b, const DevTables &t);
hipError_t run_regex(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st, int dfa_grid,
                     const FwdDfaDev *iter = nullptr);
hipError_t run_set(const BatchDev &b, const DevTables &t, uint64_t *out, hipStream_t st, int dfa_grid);
hipError_t run_captures(const BatchDev &b, const DevTables &t, uint64_t *slots, uint32_t ns, hipStream_t st,
                        int dfa_grid);
bool to_batch(const rure_amd_batch *b, BatchDev *o);
bool single_call(rure *re, int mode, const uint8_t *hay, size_t len, size_t start, uint64_t *r0, uint64_t *r1);
uint64_t set_single_call(rure_set *rs, const uint8_t *hay, size_t len, size_t start);
const FwdDfaDev *literal_engine(int mode, rure *re, DevTables &t, const BatchDev &b);
int set_batch_word(rure_set *rs, const BatchDev &b, uint64_t *mask, hipStream_t stream);
int device_cus_cached();
int set_batch_group(rure_set *g, const rure_amd_batch *batch, const BatchDev &b, uint64_t *mask, size_t words,
                    size_t w, hipStream_t st);
hipError_t run_find_iter(rure *re, DevTables *t, const BatchDev &b, const IterOut &o, hipStream_t st,
                         std::string *err, const IterSpan *sp = nullptr);
hipError_t iter_to_device(rure *re, DevTables *t, const BatchDev &b, hipStream_t st, IterBufs *ib, std::string *err);
bool class_one_set(const Expr &e, uint8_t cls[256]);
bool build_kmer(rure *const *res, size_t n, std::vector<uint32_t> *bitmap, std::vector<uint16_t> *mask,
                std::vector<uint16_t> *hmask, KmerDev *km);
bool kmer_device(rure *const *res, size_t n, KmerDev *out);
void kmer_forget(const rure *re);
void scratch_release();
void handle_created();
void handle_freed();

}  // namespace rt
