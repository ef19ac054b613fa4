// The reference's engine dispatch over batches (src/exec.rs:382-420, 473-514,
// 998-1038, re_trait.rs:197-221): which kernel answers which search, the DFA
// -> quit -> Pike VM fallback, sets in 64-pattern groups, the find_iter
// passes and the k-mer table cache.
#include "runtime.hpp"

namespace rt {

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


int pike_grid(size_t count, bool fallback, const NfaDev &n, int cus) {
  size_t units = fallback ? (count + 63) / 64 : count;
  size_t wb = nfa_wave_bytes(n.nleaves);
  size_t per_cu = wb <= kNfaLdsMax ? std::max<size_t>(1, std::min<size_t>(32, (160u * 1024u) / wb)) : 4;
  size_t g = std::min(units, (size_t)cus * per_cu);
  return (int)std::max<size_t>(g, 1);
}

// Pike VM pass: all haystacks (no DFA) or only those the DFA quit on.
hipError_t run_pike(int mode, bool fallback, const BatchDev &b, const DevTables &t, void *out, hipStream_t st) {
  if (!fallback) note_fwd_path(-16);
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
    if (knob(Knob::Split) == 0 || mode != MODE_ISMATCH || t.anchored_rev || span < 512 || b.count < 64 ||
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
  if (knob(Knob::LongLanes) > 0) per_cu = std::max<uint64_t>(64, knob(Knob::LongLanes));
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

// DfaSuffix over few long fixed-stride haystacks: the reverse suffix scans
// cut into units (launch_suffix_long) instead of one lane per haystack; the
// haystacks where the reference falls back to the forward DFA (None) then
// take the chunked forward scan.  RURE_AMD_SUFFIX_LONG=0 keeps the lanes.
bool suffix_long_ok(const BatchDev &b, const DevTables &t, uint64_t *chunk) {
  if (t.m.mt != MT_DFA_SUFFIX || !t.lcs_free || !t.has_dfa || t.quit_possible || b.offs || b.count == 0 || !t.owner)
    return false;
  if (knob(Knob::SuffixLong) == 0) return false;
  const uint64_t span = b.length > b.start ? b.length - b.start : 0;
  if (b.count >= (uint64_t)t.cus * 16 || (span < (256u << 10) && knob(Knob::SuffixLong) != 2)) return false;
  const uint64_t target = (uint64_t)t.cus * 1024;
  const uint64_t per_h = (target + b.count - 1) / b.count;
  *chunk = odd_lines(std::max<uint64_t>(knob(Knob::SuffixLong) == 2 ? 128 : 16u << 10, (span + per_h - 1) / per_h));
  return true;
}

hipError_t run_suffix_long(int mode, const BatchDev &b, const DevTables &t, uint64_t chunk, void *out,
                           hipStream_t st) {
  uint8_t *status = nullptr;
  hipError_t e = scratch_malloc((void **)&status, b.count, st);
  if (e == hipSuccess) e = launch_suffix_long(mode, b, t.m, t.f, t.r, chunk, out, status, st, t.cus);
  std::vector<uint8_t> hs(b.count);
  if (e == hipSuccess) e = hipMemcpyAsync(hs.data(), status, b.count, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (status) { hipError_t e2 = scratch_free(status, st); if (e == hipSuccess) e = e2; }
  if (e != hipSuccess) return e;
  size_t nf = 0;
  for (uint8_t x : hs) nf += x == 3;
  if (!nf) return hipSuccess;
  // exec.rs:764-769 / 700-709: None -> the forward DFA from the search start
  std::string err;
  const FwdDfaDev *iter = iter_device(t.owner, t, &err);
  if (!iter) return hipErrorInvalidValue;
  uint64_t fchunk = 0;
  if (!long_batch(mode, b, t, &fchunk)) fchunk = chunk;
  const size_t rec = mode == MODE_FIND ? 16 : mode == MODE_SHORTEST ? 8 : 1;
  if (nf == b.count) return launch_long_scan(mode, b, *iter, t.r, fchunk, out, st, t.cus);
  void *tmp = nullptr;
  e = scratch_malloc(&tmp, b.count * rec, st);
  if (e == hipSuccess) e = launch_long_scan(mode, b, *iter, t.r, fchunk, tmp, st, t.cus);
  for (size_t h = 0; e == hipSuccess && h < b.count; ++h)
    if (hs[h] == 3)
      e = hipMemcpyAsync((uint8_t *)out + h * rec, (uint8_t *)tmp + h * rec, rec, hipMemcpyDeviceToDevice, st);
  if (tmp) { hipError_t e2 = scratch_free(tmp, st); if (e == hipSuccess) e = e2; }
  return e;
}

hipError_t run_lane_search(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st) {
  uint64_t chunk = 0;
  if (suffix_long_ok(b, t, &chunk)) return run_suffix_long(mode, b, t, chunk, out, st);
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
  if (knob(Knob::Big) == 2) return true;
  if (knob(Knob::Big) == 0) return false;
  return b.count >= (uint64_t)t.cus * 64;
}

// find / is_match / shortest on the on-demand forward DFA (lazy_device):
// rounds of lazy_dfa_kernel; between rounds the host builds the rows the
// parked lanes need (and, ahead of them, more rows in discovery order) and
// uploads the grown table.  Synchronous, as the reference's construction
// happens inside its search.  The reference gives up on its lazy DFA when
// the cache thrashes (dfa.rs:1282-1293) and runs the Pike VM; here a spent
// memory budget or kLazyRounds rounds do the same for the batch.
constexpr int kLazyRounds = 256;
hipError_t run_lazy(int mode, const BatchDev &b, const DevTables &tc, void *out, hipStream_t st) {
  DevTables &t = const_cast<DevTables &>(tc);
  rure *re = t.owner;
  std::lock_guard<std::mutex> g(re->mu);
  LazyDfa &L = *re->lazy;
  size_t ahead = 4096;  // rows built ahead per round (knob lazy_rows: tests)
  if (knob(Knob::LazyRows) > 0) ahead = (size_t)knob(Knob::LazyRows);
  bool ok = L.nbuilt() > 0 || L.expand(ahead);
  hipError_t e = hipSuccess;
  LazyPark *pk[2] = {nullptr, nullptr};
  unsigned long long *cnt = nullptr;
  const size_t pbytes = std::max<uint64_t>(b.count, 1) * sizeof(LazyPark);
  if ((e = scratch_malloc((void **)&pk[0], pbytes, st)) != hipSuccess) return e;
  if ((e = scratch_malloc((void **)&pk[1], pbytes, st)) != hipSuccess) return e;
  if ((e = scratch_malloc((void **)&cnt, 16, st)) != hipSuccess) return e;
  const LazyPark *in = nullptr;
  uint64_t nin = 0;
  std::vector<LazyPark> host;
  for (int round = 0; ok && e == hipSuccess; ++round) {
    // the table: [colmap 256][start 512][eof cap][trans cap * ncol * 4]
    const size_t ns = L.nstates(), need = 768 + ns + ns * (size_t)L.ncol * 4 + 16;
    if (need > t.lazy_cap) {
      if ((e = hipStreamSynchronize(st)) != hipSuccess) break;
      if (t.lazy_buf) (void)hipFree(t.lazy_buf);
      t.lazy_buf = nullptr;
      t.lazy_cap = std::max(need * 3 / 2, (size_t)1 << 20);
      if ((e = hipMalloc(&t.lazy_buf, t.lazy_cap)) != hipSuccess) { t.lazy_cap = 0; break; }
    }
    uint8_t *base = (uint8_t *)t.lazy_buf;
    const size_t o_eof = 768, o_trans = (768 + ns + 15) & ~(size_t)15;
    if ((e = hipMemcpyAsync(base, L.colmap, 256, hipMemcpyHostToDevice, st)) != hipSuccess) break;
    if ((e = hipMemcpyAsync(base + 256, L.start, 512, hipMemcpyHostToDevice, st)) != hipSuccess) break;
    if ((e = hipMemcpyAsync(base + o_eof, L.eof.data(), ns, hipMemcpyHostToDevice, st)) != hipSuccess) break;
    if ((e = hipMemcpyAsync(base + o_trans, L.trans.data(), L.trans.size() * 4, hipMemcpyHostToDevice, st)) !=
        hipSuccess)
      break;
    LazyDfaDev f{};
    f.colmap = base;
    f.start = (const uint32_t *)(base + 256);
    f.eof = base + o_eof;
    f.trans = (const uint32_t *)(base + o_trans);
    f.ncol = L.ncol;
    f.hot = std::min<uint32_t>((uint32_t)ns, lazy_dfa_hot_rows(L.ncol));
    LazyPark *po = pk[round & 1];
    if ((e = hipMemsetAsync(cnt, 0, 8, st)) != hipSuccess) break;
    if ((e = launch_lazy_dfa(mode, b, f, t.lr, in, nin, po, cnt, out, st, t.cus)) != hipSuccess) break;
    unsigned long long n = 0;
    if ((e = hipMemcpyAsync(&n, cnt, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) break;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) break;
    if (n == 0) break;
    if (round + 1 >= kLazyRounds) { ok = false; break; }
    host.resize(n);
    if ((e = hipMemcpyAsync(host.data(), po, n * sizeof(LazyPark), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
      break;
    size_t built0 = L.nbuilt();
    for (const LazyPark &x : host)
      if (!(ok = L.build_row(x.s))) break;
    // (a fixed number ahead: doubling the rows built ahead each round built
    // states in discovery order the text never visits, seconds of host work
    // for (?:a|b)*a(?:a|b){20})
    (void)built0;
    if (ok) ok = L.expand(ahead);
    in = po;
    nin = n;
  }
  for (int k = 0; k < 2; ++k) { hipError_t e2 = scratch_free(pk[k], st); if (e == hipSuccess) e = e2; }
  { hipError_t e2 = scratch_free(cnt, st); if (e == hipSuccess) e = e2; }
  if (e == hipSuccess && !ok) e = run_pike(mode, false, b, t, out, st);  // the whole batch again
  return e;
}

// The on-demand DFA where the eager automata did not materialise (or
// RURE_AMD_LAZY=1: tests, any regex), for batches that fill the device.
static bool lazy_batch(const BatchDev &b, const DevTables &t) {
  if (knob(Knob::Lazy) == 0) return false;
  const bool force = knob(Knob::Lazy) == 1;
  if (!force && (t.has_dfa || !big_batch(b, t))) return false;
  return lazy_device(t);
}

hipError_t run_regex(int mode, const BatchDev &b, const DevTables &t, void *out, hipStream_t st, int dfa_grid,
                     const FwdDfaDev *iter) {
  if (lane_search_ok(t)) return run_lane_search(mode, b, t, out, st);
  if (knob(Knob::Lazy) == 1 && lazy_batch(b, t))
    return run_lazy(mode, b, t, out, st);
  if (!t.has_dfa && big_batch(b, t) && big_device(t)) return launch_big_dfa(mode, b, t.bf, t.br, out, st, t.cus);
  if (!t.has_dfa && lazy_batch(b, t)) return run_lazy(mode, b, t, out, st);
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
const FwdDfaDev *literal_engine(int mode, rure *re, DevTables &t, const BatchDev &b) {
  uint64_t chunk;
  const long long env = knob(Knob::Lit);
  if (env >= 0 && env != 1) return nullptr;
  if (t.mt_lane) return nullptr;  // the reference's literal searcher differs from the regex's strings
  if (env < 0 && long_batch(mode, b, t, &chunk)) return nullptr;  // lit=1 forces the literal engine
  {
    // the literal set alone (cheap) before any find_iter DFA is built
    std::lock_guard<std::mutex> g(re->mu);
    if (!re->iter_built && !re->lits_done) re->lit_ok = extract_literals(re->nfa, kLitMax, kLitLen, &re->lits);
    re->lits_done = true;
    if (!re->lit_ok || (env < 0 && re->lits.lits.size() > kLitFindMax)) return nullptr;
  }
  std::string err;
  const FwdDfaDev *fi = iter_device(re, t, &err);
  return fi && fi->lit_n ? fi : nullptr;
}


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



// The batched find_iter (re_trait.rs:197-221) on one stream.
hipError_t run_find_iter(rure *re, DevTables *t, const BatchDev &b, const IterOut &o, hipStream_t st,
                         std::string *err, const IterSpan *sp) {
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
  // DfaSuffix over few long haystacks: the iteration over suffix occurrences
  // in parallel (launch_suffix_iter); RURE_AMD_SUFFIX_ITER=0 keeps the wave
  // path, =2 takes it at any length with 128-byte units (tests).
  // (a DFA that can quit: the path gives up on the first quit, the wave path
  // then runs with its Pike VM fallback)
  if (lane_search_ok(*t) && !sp && t->m.mt == MT_DFA_SUFFIX && t->lcs_free && !b.offs &&
      b.count && b.count < (uint64_t)t->cus * 16 && b.length > b.start) {
    const uint64_t span = b.length - b.start;
    if (knob(Knob::SuffixIter) != 0 && (span >= (256u << 10) || knob(Knob::SuffixIter) == 2)) {
      const uint64_t per_h = ((uint64_t)t->cus * 1024 + b.count - 1) / b.count;
      const uint64_t chunk =
          odd_lines(std::max<uint64_t>(knob(Knob::SuffixIter) == 2 ? 128 : 16u << 10, (span + per_h - 1) / per_h));
      const hipError_t e = launch_suffix_iter(b, t->m, t->f, t->r, chunk, o, st, t->cus);
      if (e != hipErrorNotSupported) return e;
    }
  }
  // The reference's Literal / DfaSuffix searches (DevTables::mt_lane): every
  // search of the iteration is one of those, on a wave per haystack (lane 0
  // searches, the wave runs the Pike VM where a DfaSuffix scan quits).
  if (lane_search_ok(*t) && re->nfa_ok)
    return launch_find_iter(b, t->has_dfa ? &t->f : nullptr, t->r, &t->n, false, 0, o, st, t->cus, sp, &t->m);
  // Chunked speculative iteration (iter_scan.hip); otherwise one wave per
  // haystack.  With look-around (or a DFA that can quit) it needs the
  // stripped states (not an anchored regex) and a whole haystack (no span:
  // a span's "fresh" exit is not enough to enter the next); a quit sends the
  // batch to the wave path.  RURE_AMD_ITER_LOOKS=0 keeps those on the wave
  // path (A/B).
  const FwdDfaDev *fi = nullptr;
  const bool looks = re->nt.looks_used != 0 || t->quit_possible;
  if (t->has_dfa && re->nfa_ok && (!looks || (!sp && knob(Knob::IterLooks) != 0))) fi = iter_device(re, *t, err);
  if (fi && looks && re->dfwd_iter.strip.empty()) fi = nullptr;
  if (fi) {
    uint64_t chunk = ~0ull >> 2;
    const uint64_t lim = sp ? std::min<uint64_t>(b.length, sp->hi) : b.length;
    if (!b.offs && lim > b.start && b.count) {
      const uint64_t span = lim - b.start;
      // lanes in flight: 16 waves per CU (tools/iter_sweep.py);
      // RURE_AMD_ITER_LANES (per CU) overrides (tuning)
      uint64_t per_cu = 1024;
      if (knob(Knob::IterLanes) > 0) per_cu = std::max<uint64_t>(64, knob(Knob::IterLanes));
      const uint64_t target = (uint64_t)t->cus * per_cu;
      const uint64_t per_h = (target + b.count - 1) / b.count;
      chunk = odd_lines(std::max<uint64_t>(4096, (span + per_h - 1) / per_h));
      // knob iter_chunk: the unit size in bytes (tests: many boundaries)
      if (knob(Knob::IterChunk) > 0) chunk = std::max<uint64_t>(16, knob(Knob::IterChunk));
    }
    // A regex that is one class repeated (C+: [a-z]+, (?-u)\w+, and Unicode
    // classes \w+, \S+, \pL+ over UTF-8): its matches are the maximal runs
    // (run_iter.hip), no DFA walk; the ASCII shadow's class (an ASCII-only
    // class in Unicode mode) answers ASCII text and quits on any other
    // byte.  Knob runs=0 keeps the DFA paths (A/B).
    const bool runs = !sp && knob(Knob::Runs) != 0;
    bool run_quit = false;
    if (runs && fi->run_cls) {
      bool q = false;
      const hipError_t e = launch_find_iter_runs(b, fi->run_cls, fi->run_cp, o, st, t->cus, fi->run_quit != 0, &q);
      if (e != hipErrorNotSupported && (e != hipSuccess || !q)) {
        if (e == hipSuccess) note_fwd_path(-19);
        return e;
      }
      run_quit = q;
    }
    // the ASCII shadow first (all-rows LDS tables; a non-ASCII byte quits
    // and the full automaton re-runs the batch, still chunked); not for
    // spans (the quit is read back), and not after the run engine quit (it
    // quits on a byte >= 0x80, where the shadow would quit too)
    bool shadow_quit = false;
    if (!sp && !run_quit) {
      if (const FwdDfaDev *fa = iter_ascii_device(re, *t, err)) {
        if (runs && fa->run_cls) {
          bool q = false;
          const hipError_t e = launch_find_iter_runs(b, fa->run_cls, nullptr, o, st, t->cus, true, &q);
          if (e != hipErrorNotSupported && (e != hipSuccess || !q)) {
            if (e == hipSuccess) note_fwd_path(-20);
            return e;
          }
        }
        // The full automaton cannot quit: both passes are enqueued, the
        // shadow's quit staying a device word -- its passes after the quit
        // check run while the word is 0, the full automaton's while it is set
        // (-25; nothing read back, the call only enqueues).  Knob
        // shadow_sync=1 reads the quit back (-14 / -15).
        if (!fi->can_quit && knob(Knob::ShadowSync) != 1) {
          uint32_t *qf = nullptr;
          hipError_t e = scratch_malloc((void **)&qf, 8, st);
          if (e == hipSuccess) e = hipMemsetAsync(qf, 0, 4, st);
          if (e == hipSuccess)
            e = launch_find_iter(b, fa, t->r, &t->n, true, chunk, o, st, t->cus, nullptr, nullptr, nullptr, qf);
          if (e == hipSuccess) {
            BatchDev bf = b;
            bf.gate = qf;
            bf.gate_set = 1;
            e = launch_find_iter(bf, fi, t->r, &t->n, true, chunk, o, st, t->cus, nullptr);
          }
          if (qf) {
            const hipError_t e2 = scratch_free(qf, st);
            if (e == hipSuccess) e = e2;
          }
          if (e == hipSuccess) note_fwd_path(-25);
          return e;
        }
        bool q = false;
        const hipError_t e = launch_find_iter(b, fa, t->r, &t->n, true, chunk, o, st, t->cus, sp, nullptr, &q);
        if (e != hipSuccess || !q) {
          if (e == hipSuccess) note_fwd_path(-14);
          return e;
        }
        shadow_quit = true;  // a quit: the full automaton below answers (-15)
      }
    }
    // A DFA that can quit (Unicode \b over non-ASCII bytes): the units whose
    // searches quit are served by the wave's Pike VM inside the chunked
    // iteration (iter_scan.hip iter_wspec_kernel .. iter_wemit_kernel; -27,
    // nothing read back).  Spans, and knob iter_wave=0, keep the read-back of
    // the quit and the one-wave-per-haystack fallback (-13).
    if (fi->can_quit && !sp && re->nfa_ok && knob(Knob::IterWave) != 0) {
      const hipError_t e = launch_find_iter(b, fi, t->r, &t->n, true, chunk, o, st, t->cus, nullptr);
      if (e == hipSuccess) note_fwd_path(-27);
      return e;
    }
    bool quit = false;
    const hipError_t e = launch_find_iter(b, fi, t->r, &t->n, true, chunk, o, st, t->cus, sp, nullptr, &quit);
    // last_fwd_path: -12 = the chunked iteration of a look-around regex
    // answered, -13 = it quit (the wave path answers)
    // (-21: the chunked iteration of the full automaton answered; -15: so,
    // after the ASCII shadow quit)
    if (e == hipSuccess) note_fwd_path(looks ? (quit ? -13 : -12) : shadow_quit ? -15 : -21);
    if (e != hipSuccess || !quit) return e;
  }
  if (!re->nfa_ok) return hipErrorInvalidValue;
  const hipError_t e = launch_find_iter(b, t->has_dfa ? &t->f : nullptr, t->r, &t->n, false, 0, o, st, t->cus, sp);
  if (e == hipSuccess && last_fwd_path() != -13) note_fwd_path(-22);  // one haystack per wavefront
  return e;
}


hipError_t iter_to_device(rure *re, DevTables *t, const BatchDev &b, hipStream_t st, IterBufs *ib, std::string *err) {
  ib->st = st;
  hipError_t e;
  const size_t n = b.count;
  if ((e = scratch_malloc((void **)&ib->counts, (n + 1) * 8, st)) != hipSuccess) return e;
  if ((e = scratch_malloc((void **)&ib->moff, (n + 1) * 8, st)) != hipSuccess) return e;
  if ((e = scratch_malloc((void **)&ib->total, 8, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(ib->counts, 0, (n + 1) * 8, st)) != hipSuccess) return e;
  const uint64_t bytes = b.offs ? 0 : (uint64_t)b.count * b.length;
  // first guess: the regex's density on its previous call plus an eighth,
  // else a match per 64 bytes (an overflow re-runs the search once with the
  // exact size: the regex-dna strip, a match per 61 bytes, paid that once)
  const int64_t per_mib = re->iter_per_mib.load(std::memory_order_relaxed);
  uint64_t cap = per_mib >= 0 ? (uint64_t)((double)bytes / (1 << 20) * (double)per_mib * 1.125) + 2 * n
                              : bytes / 64 + 2 * n;
  cap = std::max<uint64_t>(1024, cap);
  for (int pass = 0; pass < 2; ++pass) {
    if ((e = scratch_malloc((void **)&ib->m, cap * 16, st)) != hipSuccess) return e;
    IterOut o{ib->counts, ib->m, cap, ib->total};
    if ((e = run_find_iter(re, t, b, o, st, err)) != hipSuccess) return e;
    uint64_t tot = 0;
    if ((e = hipMemcpyAsync(&tot, ib->total, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    ib->nm = tot;
    if (bytes >= (1u << 20)) re->iter_per_mib.store((int64_t)((double)tot / ((double)bytes / (1 << 20)) + 1),
                                                    std::memory_order_relaxed);
    if (tot <= cap) break;
    (void)scratch_free(ib->m, st);
    ib->m = nullptr;
    cap = tot;
  }
  return exclusive_scan_u64(ib->counts, ib->moff, n + 1, st);
}


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

bool build_kmer(rure *const *res, size_t n, std::vector<uint32_t> *bitmap, std::vector<uint16_t> *mask,
                std::vector<uint16_t> *hmask, KmerDev *km) {
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
  km->vlut = 0;
  for (uint32_t c = 0; c < 4; ++c) {
    const uint32_t v = (km->present >> c) & 1u ? (km->lut >> (8 * c)) & 0xFFu : ((c ^ 1u) << shift);
    km->vlut |= v << (8 * c);
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
  // the masks' perfect hash for the tile kernel's LDS (kmer_hit_lds): an odd
  // multiplier whose top 10 product bits are distinct over the string codes.
  // Random multipliers find one with probability ~exp(-c^2 / 2048) per try
  // for c codes, so past 160 codes (< 4e-6 per try) none is searched for;
  // without one the hits read mask[code] from global memory (hglobal).
  std::vector<uint32_t> codes;
  for (uint32_t c = 0; c < (uint32_t)mask->size(); ++c)
    if ((*mask)[c]) codes.push_back(c);
  if (codes.size() > 512) return false;
  km->hmul = 0;
  km->hglobal = 1;
  hmask->assign(1024, 0);
  if (codes.size() > 160) return true;
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  std::vector<uint16_t> slot(1024);
  std::vector<uint8_t> used(1024);
  for (int t = 0; t < 100000; ++t) {
    rng ^= rng << 13, rng ^= rng >> 7, rng ^= rng << 17;
    const uint32_t K = (uint32_t)rng | 1u;
    std::fill(slot.begin(), slot.end(), 0);
    std::fill(used.begin(), used.end(), 0);
    bool ok = true;
    for (uint32_t c : codes) {
      const uint32_t h = (c * K) >> 22;
      if (used[h]) { ok = false; break; }
      used[h] = 1;
      slot[h] = (*mask)[c];
    }
    if (ok) {
      km->hmul = K;
      km->hglobal = 0;
      *hmask = slot;
      return true;
    }
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
  std::vector<uint16_t> hm;
  if (build_kmer(res, n, &bm, &mk, &hm, &ent.km)) {
    Blob b;
    const size_t ob = b.add(bm.data(), bm.size() * 4), om = b.add(mk.data(), mk.size() * 2);
    const size_t oh = b.add(hm.data(), hm.size() * 2);
    DevTables tmp;
    std::string err;
    if (upload_blob(b, &tmp, &err)) {
      ent.blob = tmp.blob;
      ent.km.bitmap = (const uint32_t *)((uint8_t *)tmp.blob + ob);
      ent.km.mask = (const uint16_t *)((uint8_t *)tmp.blob + om);
      ent.km.hmask = (const uint16_t *)((uint8_t *)tmp.blob + oh);
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

}  // namespace rt
