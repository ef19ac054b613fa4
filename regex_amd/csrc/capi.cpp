// rure_amd: C ABI (include/rure_amd.h) over the host compiler + HIP kernels.
//
// Mirrors the reference C API regex-capi/src/rure.rs (compile 95-150,
// is_match 158-168, find 170-187, shortest_match 207-224, iter 308-360,
// options 13-19/67-74, set 470-572, errors regex-capi/src/error.rs) and the
// engine construction of src/exec.rs:273-327 (three programs per regex: NFA,
// forward DFA with `.*?`, reverse DFA).  All matching runs on the GPU.
#include "runtime.hpp"

namespace {


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
  re->cls_one_ok = class_one_set(re->expr, re->cls_one);
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
  for (auto &kv : re->iter_dev_a) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(kv.first);
    (void)hipFree(kv.second.first);
    (void)hipSetDevice(cur);
  }
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
    if (kv.second.lazy_buf) (void)hipFree(kv.second.lazy_buf);
    if (kv.second.lazy_rblob) (void)hipFree(kv.second.lazy_rblob);
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



int rure_amd_set_matches_batch_words(rure_set *rs, const rure_amd_batch *batch, uint64_t *mask, size_t words,
                                     void *stream) {
  BatchDev b;
  if (!rs || !to_batch(batch, &b) || (!mask && b.count)) return RURE_AMD_ERR_ARG;
  const size_t n = rs->exprs.size();
  if (words < std::max<size_t>(1, (n + 63) / 64)) return RURE_AMD_ERR_ARG;
  if (b.count == 0) return RURE_AMD_OK;
  hipStream_t st = (hipStream_t)stream;
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

int rure_amd_set_matches_batch(rure_set *rs, const rure_amd_batch *batch, uint64_t *mask, void *stream) {
  if (rs && rs->exprs.size() > 64) return RURE_AMD_ERR_ARG;  // use rure_amd_set_matches_batch_words
  return rure_amd_set_matches_batch_words(rs, batch, mask, 1, stream);
}



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
    if (knob(Knob::IterLanes) > 0) per_cu = std::max<uint64_t>(64, knob(Knob::IterLanes));
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

int rure_amd_replace_all_chain(rure *const *res, const uint8_t *const *reps, const size_t *rep_lens, size_t n,
                               const uint8_t *haystack, size_t length, uint8_t *out0, uint8_t *out1,
                               size_t capacity, uint64_t *lengths, void *stream) {
  if (!res || (n && (!reps || !rep_lens)) || !lengths || !haystack || !out0 || (n > 1 && !out1) ||
      ((uintptr_t)haystack & 15) || ((uintptr_t)out0 & 15) || (out1 && ((uintptr_t)out1 & 15)))
    return RURE_AMD_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return hipMemcpyAsync(lengths, &length, 8, hipMemcpyHostToDevice, st) == hipSuccess ? RURE_AMD_OK
                                                                                              : RURE_AMD_ERR_HIP;
  std::vector<uint32_t> rl(n);
  std::vector<std::array<uint32_t, 2>> sw(n);
  std::vector<uint8_t> host(n * 320, 0);  // per step: the class (256), the replacement (64)
  int cus = 0;
  for (size_t i = 0; i < n; ++i) {
    rure *re = res[i];
    if (!re || rep_lens[i] < 1 || rep_lens[i] > 64 || !reps[i]) return RURE_AMD_ERR_ARG;
    std::string err;
    DevTables *t = regex_device(re, &err);
    if (!t) return err.rfind("HIP", 0) == 0 ? RURE_AMD_ERR_HIP : RURE_AMD_ERR_DFA;
    if (!re->cls_one_ok) return RURE_AMD_ERR_ARG;
    cus = t->cus;
    rl[i] = (uint32_t)rep_lens[i];
    memcpy(&host[i * 320], re->cls_one, 256);
    memcpy(&host[i * 320 + 256], reps[i], rep_lens[i]);
    // a class of one or two bytes as SWAR compares (as rure_amd_replace_batch)
    uint32_t w[2] = {0, 0}, nb = 0;
    for (int c = 1; c < 256 && nb <= 2; ++c)
      if (re->cls_one[c]) { if (nb < 2) w[nb] = (uint32_t)c * 0x01010101u; ++nb; }
    if (re->cls_one[0] || nb > 2) w[0] = w[1] = 0;
    else if (nb == 1) w[1] = w[0];
    sw[i] = {w[0], w[1]};
  }
  // The chain is a string homomorphism: compose each byte's image F(x) and
  // its length after every step, and run it as one map (launch_replace_hmap)
  // when the images are at most 64 bytes and fit the 4 KiB pool.
  if (knob(Knob::ChainSeq) != 1) {
    std::vector<std::string> img(256);
    std::vector<uint32_t> dl(n * 256, 0);
    bool ok = true;
    for (int x = 0; x < 256 && ok; ++x) {
      std::string cur(1, (char)x);
      for (size_t i = 0; i < n && ok; ++i) {
        std::string nx;
        for (unsigned char c : cur) {
          if (res[i]->cls_one[c]) nx.append((const char *)reps[i], rep_lens[i]);
          else nx.push_back((char)c);
        }
        cur.swap(nx);
        if (cur.size() > 64) ok = false;
        dl[i * 256 + x] = (uint32_t)cur.size() - 1;
      }
      img[x] = cur;
    }
    size_t pool = 0;
    for (int x = 0; x < 256; ++x) pool += img[x].size();
    if (ok && pool <= kHMapPoolMax) {
      std::vector<uint8_t> blob(1024 + kHMapPoolMax + n * 256 * 4, 0);
      uint16_t *so = (uint16_t *)(blob.data() + 256);
      size_t at = 0;
      uint32_t nact = 0;
      for (int x = 0; x < 256; ++x) {
        blob[x] = (uint8_t)img[x].size();
        so[x] = (uint16_t)at;
        const bool same = img[x].size() == 1 && (uint8_t)img[x][0] == x;
        blob[768 + x] = same ? 0xFF : (uint8_t)nact;
        nact += same ? 0 : 1;
        memcpy(blob.data() + 1024 + at, img[x].data(), img[x].size());
        at += img[x].size();
      }
      memcpy(blob.data() + 1024 + kHMapPoolMax, dl.data(), dl.size() * 4);
      uint8_t *db = nullptr;
      hipError_t e = scratch_malloc((void **)&db, blob.size(), st);
      if (e == hipSuccess) e = hipMemcpyAsync(db, blob.data(), blob.size(), hipMemcpyHostToDevice, st);
      uint8_t *out = (n & 1) ? out0 : out1;
      if (e == hipSuccess)
        e = launch_replace_hmap(haystack, length, (int)n, db, (uint32_t)pool, nact, out, capacity, lengths, st,
                                cus);
      if (db) { const hipError_t e2 = scratch_free(db, st); if (e == hipSuccess) e = e2; }
      if (e == hipSuccess) note_fwd_path(-24);
      if (e != hipErrorNotSupported) return e == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
    }
  }
  uint8_t *dt = nullptr;
  hipError_t e = scratch_malloc((void **)&dt, host.size(), st);
  if (e == hipSuccess) e = hipMemcpyAsync(dt, host.data(), host.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    std::vector<const uint8_t *> cls(n), rep(n);
    for (size_t i = 0; i < n; ++i) {
      cls[i] = dt + i * 320;
      rep[i] = dt + i * 320 + 256;
    }
    // the bytes of each replacement in the next step's class
    std::vector<uint32_t> nrep(n, 0);
    for (size_t i = 0; i + 1 < n; ++i)
      for (size_t t = 0; t < rep_lens[i]; ++t) nrep[i] += res[i + 1]->cls_one[reps[i][t]] ? 1u : 0u;
    e = launch_replace_class_chain(haystack, length, (int)n, cls.data(), rep.data(), rl.data(),
                                   (const uint32_t(*)[2])sw.data(), nrep.data(), out0, out1, capacity, lengths, st,
                                   cus);
  }
  if (dt) { const hipError_t e2 = scratch_free(dt, st); if (e == hipSuccess) e = e2; }
  if (e == hipErrorNotSupported) return RURE_AMD_ERR_ARG;
  if (e == hipSuccess) note_fwd_path(-23);
  return e == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
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
  const uint64_t lim = limit == 0 ? ~0ull : (uint64_t)limit;  // replacen: 0 = all
  // a regex whose matches are single bytes of one class, replace_all over
  // one haystack: no match list (launch_replace_class); no synchronisation
  if (re->cls_one_ok && b.count == 1 && !b.offs && b.start == 0 && lim == ~0ull && rep_len >= 1 && rep_len <= 64 &&
      knob(Knob::ReplaceGeneric) != 1) {
    uint8_t *dt = nullptr;
    hipError_t e = scratch_malloc((void **)&dt, 256 + 64, st);
    if (e == hipSuccess) e = hipMemcpyAsync(dt, re->cls_one, 256, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(dt + 256, rep, rep_len, hipMemcpyHostToDevice, st);
    // (a class of one or two bytes: SWAR compares instead of the table; byte
    // 0 can not be a repeated compare value, it would read as "no class")
    uint32_t sw[2] = {0, 0}, nb = 0;
    for (int c = 1; c < 256 && nb <= 2; ++c)
      if (re->cls_one[c]) { if (nb < 2) sw[nb] = (uint32_t)c * 0x01010101u; ++nb; }
    if (re->cls_one[0] || nb > 2) sw[0] = sw[1] = 0;
    else if (nb == 1) sw[1] = sw[0];
    if (e == hipSuccess)
      e = launch_replace_class(b.hay, b.length, dt, dt + 256, (uint32_t)rep_len, out, out_capacity, out_offsets, total,
                               st, t->cus, sw[0], sw[1]);
    if (dt) { const hipError_t e2 = scratch_free(dt, st); if (e == hipSuccess) e = e2; }
    if (e != hipErrorNotSupported) {
      if (e == hipSuccess) note_fwd_path(-23);
      return e == hipSuccess ? RURE_AMD_OK : RURE_AMD_ERR_HIP;
    }
  }
  IterBufs ib;
  int64_t *shift = nullptr;
  uint64_t *olen = nullptr;
  uint8_t *drep = nullptr;
  hipError_t e = iter_to_device(re, t, b, st, &ib, &err);
  if (e == hipSuccess) e = scratch_malloc((void **)&shift, (ib.nm + 1) * 8, st);
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
                            hint, st, t->cus, ib.nm);
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
  if (which == 5) {  // the find_iter automaton's ASCII shadow (build_iter_dfa)
    if (!build_iter_dfa(re) || !re->iter_a_ok) { info->ok = 0; return RURE_AMD_ERR_DFA; }
    fill_info(re->dfwd_iter_a, re->fwd, re->pf_iter_a.hot, info, &re->pf_iter_a);
    return RURE_AMD_OK;
  }
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

int64_t rure_amd_lex4_export(rure *re, uint8_t *table, size_t cap, uint32_t *s0) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  if (table) memcpy(table, re->lex4.data(), std::min(cap, re->lex4.size()));
  if (s0) *s0 = re->lex4_s0;
  return (int64_t)re->lex4.size();
}

int64_t rure_amd_lex_ascii_export(rure *re, int four, uint8_t *table, size_t cap, uint32_t *s0) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  const std::vector<uint8_t> &t = four ? re->lex4_a : re->lex_a;
  if (table) memcpy(table, t.data(), std::min(cap, t.size()));
  if (s0) *s0 = four ? re->lex4_a_s0 : re->lex_a_s0;
  return (int64_t)t.size();
}

int rure_amd_run_class_export(rure *re, int ascii, uint8_t *cls) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  const bool ok = ascii ? re->run_a_ok : re->run_ok;
  if (ok && cls) memcpy(cls, ascii ? re->run_cls_a : re->run_cls, 256);
  return ok ? 1 : 0;
}

int rure_amd_class_one_export(rure *re, uint8_t *cls) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (re->cls_one_ok && cls) memcpy(cls, re->cls_one, 256);
  return re->cls_one_ok ? 1 : 0;
}

int rure_amd_run_cp_export(rure *re, uint32_t *bits, size_t n) {
  if (!re) return RURE_AMD_ERR_ARG;
  if (!build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  if (!re->run_ok || re->run_cp.empty()) return 0;
  if (bits) memcpy(bits, re->run_cp.data(), std::min(n, re->run_cp.size()) * 4);
  return (int)re->run_cp.size();
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
  if ((which == 2 || which == 5) && !build_iter_dfa(re)) return RURE_AMD_ERR_DFA;
  if (which == 5 && !re->iter_a_ok) return RURE_AMD_ERR_DFA;
  const DenseDfa &d = which == 0 ? re->dfwd : which == 1 ? re->drev : which == 5 ? re->dfwd_iter_a : re->dfwd_iter;
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
int rure_amd_debug_set(const char *spec) { return rure_amd::knob_set(spec) ? RURE_AMD_OK : RURE_AMD_ERR_ARG; }



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
