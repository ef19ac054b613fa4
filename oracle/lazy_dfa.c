/*
 * TEST INFRASTRUCTURE ONLY.  Restatement of the reference lazy DFA,
 * src/dfa.rs (regex 0.2.5), over a byte Program.  Function-by-function:
 *   Cache/CacheInner          dfa.rs:92-158, 423-455
 *   forward/reverse/many      dfa.rs:459-570
 *   exec_at                   dfa.rs:576-764
 *   exec_at_reverse           dfa.rs:768-866
 *   next_si                   dfa.rs:873-900
 *   exec_byte                 dfa.rs:910-1048
 *   follow_epsilons           dfa.rs:1073-1134
 *   cached_state(_key)        dfa.rs:1154-1244
 *   clear_cache(_and_save)    dfa.rs:1254-1331
 *   next_state                dfa.rs:1345-1361
 *   start_state/start_flags   dfa.rs:1370-1464
 *   add_state                 dfa.rs:1479-1512
 *   StateFlags/Byte/varints   dfa.rs:1648-1697, 1791-1831
 *   prefix_at / has_prefix    dfa.rs:700-711, 1520-1522, 1562-1579
 * The prefix skip runs when the caller passes the program's prefix literals
 * (orc_dfa_forward_pfx); it is result-neutral (the reference documents it
 * so) and makes the timed CPU baseline the reference's engine path.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle_int.h"

#define STATE_UNKNOWN (1u << 31)
#define STATE_DEAD (STATE_UNKNOWN + 1)
#define STATE_QUIT (STATE_DEAD + 1)
#define STATE_START (1u << 30)
#define STATE_MATCH (1u << 29)
#define STATE_MAX (STATE_MATCH - 1)
#define BYTE_EOF 256

/* StateFlags (dfa.rs:1648-1672) */
#define SF_MATCH 1u
#define SF_WORD 2u
#define SF_EMPTY 4u

/* ------------------------------------------------------------ sparse set */
void orc_sset_init(orc_sset *s, size_t cap) {
  s->dense = (uint32_t *)calloc(cap ? cap : 1, 4);
  s->sparse = (uint32_t *)calloc(cap ? cap : 1, 4);
  s->n = 0;
  s->cap = cap;
}
void orc_sset_free(orc_sset *s) { free(s->dense); free(s->sparse); }
int orc_sset_contains(const orc_sset *s, uint32_t v) {
  uint32_t i = s->sparse[v];
  return i < s->n && s->dense[i] == v;
}
void orc_sset_insert(orc_sset *s, uint32_t v) { s->dense[s->n] = v; s->sparse[v] = (uint32_t)s->n; s->n++; }

/* -------------------------------------------------------- state storage */
static uint64_t key_hash(const uint8_t *d, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t i = 0; i < n; ++i) { h ^= d[i]; h *= 1099511628211ull; }
  return h;
}

static void map_clear(orc_dfa_cache *c) {
  for (size_t i = 0; i < c->map_cap; ++i) c->map[i] = UINT32_MAX;
  c->map_n = 0;
}

static void map_grow(orc_dfa_cache *c);

static void map_insert(orc_dfa_cache *c, uint32_t state_index) {
  if ((c->map_n + 1) * 2 > c->map_cap) map_grow(c);
  const orc_state *st = &c->states[state_index];
  size_t m = c->map_cap - 1, i = key_hash(st->data, st->len) & m;
  while (c->map[i] != UINT32_MAX) i = (i + 1) & m;
  c->map[i] = state_index;
  c->map_n++;
}

static void map_grow(orc_dfa_cache *c) {
  size_t ncap = c->map_cap ? c->map_cap * 2 : 1024;
  free(c->map);
  c->map = (uint32_t *)malloc(ncap * 4);
  c->map_cap = ncap;
  map_clear(c);
  for (size_t k = 0; k < c->nstates; ++k) {
    const orc_state *st = &c->states[k];
    size_t m = c->map_cap - 1, i = key_hash(st->data, st->len) & m;
    while (c->map[i] != UINT32_MAX) i = (i + 1) & m;
    c->map[i] = (uint32_t)k;
    c->map_n++;
  }
}

/* returns the state index or UINT32_MAX */
static uint32_t map_find(const orc_dfa_cache *c, const uint8_t *d, uint32_t n) {
  if (!c->map_cap) return UINT32_MAX;
  size_t m = c->map_cap - 1, i = key_hash(d, n) & m;
  while (c->map[i] != UINT32_MAX) {
    const orc_state *st = &c->states[c->map[i]];
    if (st->len == n && memcmp(st->data, d, n) == 0) return c->map[i];
    i = (i + 1) & m;
  }
  return UINT32_MAX;
}

static uint32_t nclasses_of(const orc_prog *p) { return (uint32_t)p->byte_classes[255] + 1 + 1; }

/* CacheInner::reset_size (dfa.rs:450-454) */
static void reset_size(orc_dfa_cache *c) { c->size = 256 * 4 + c->stack_len * 4; }

orc_dfa_cache *orc_dfa_cache_new(const orc_prog *p) {  /* dfa.rs:425-444 */
  orc_dfa_cache *c = (orc_dfa_cache *)calloc(1, sizeof(orc_dfa_cache));
  c->nclasses = nclasses_of(p);
  for (int i = 0; i < 256; ++i) c->start_states[i] = STATE_UNKNOWN;
  c->stack = (uint32_t *)malloc((p->n + 1) * 4);
  c->stack_cap = p->n + 1;
  orc_sset_init(&c->qcur, p->n);
  orc_sset_init(&c->qnext, p->n);
  reset_size(c);
  return c;
}

static void free_states(orc_dfa_cache *c) {
  for (size_t i = 0; i < c->nstates; ++i) free(c->states[i].data);
  c->nstates = 0;
}

void orc_dfa_cache_free(orc_dfa_cache *c) {
  if (!c) return;
  free_states(c);
  free(c->states);
  free(c->trans);
  free(c->map);
  free(c->stack);
  orc_sset_free(&c->qcur);
  orc_sset_free(&c->qnext);
  free(c);
}

/* --------------------------------------------------------------- varints */
static void buf_push(uint8_t **d, uint32_t *n, uint32_t *cap, uint8_t b) {
  if (*n == *cap) { *cap = *cap ? *cap * 2 : 32; *d = (uint8_t *)realloc(*d, *cap); }
  (*d)[(*n)++] = b;
}
static void write_varu32(uint8_t **d, uint32_t *n, uint32_t *cap, uint32_t v) {  /* dfa.rs:1811-1817 */
  while (v >= 0x80) { buf_push(d, n, cap, (uint8_t)(v | 0x80)); v >>= 7; }
  buf_push(d, n, cap, (uint8_t)v);
}
static void write_vari32(uint8_t **d, uint32_t *n, uint32_t *cap, int32_t v) {  /* dfa.rs:1792-1798 */
  uint32_t un = ((uint32_t)v) << 1;
  if (v < 0) un = ~un;
  write_varu32(d, n, cap, un);
}
static uint32_t read_varu32(const uint8_t *d, uint32_t n, uint32_t *used) {  /* dfa.rs:1820-1831 */
  uint32_t v = 0, shift = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (d[i] < 0x80) { *used = i + 1; return v | ((uint32_t)d[i] << shift); }
    v |= ((uint32_t)(d[i] & 0x7F)) << shift;
    shift += 7;
  }
  *used = 0;
  return 0;
}
static int32_t read_vari32(const uint8_t *d, uint32_t n, uint32_t *used) {  /* dfa.rs:1801-1808 */
  uint32_t un = read_varu32(d, n, used);
  int32_t v = (int32_t)(un >> 1);
  if (un & 1) v = ~v;
  return v;
}

/* Decodes the instruction pointers of a state (State::inst_ptrs, dfa.rs:290-323). */
static size_t state_ips(const orc_state *st, uint32_t *out) {
  size_t k = 0;
  uint32_t i = 1;
  int64_t base = 0;
  while (i < st->len) {
    uint32_t used;
    int32_t delta = read_vari32(st->data + i, st->len - i, &used);
    base += delta;
    out[k++] = (uint32_t)base;
    i += used;
  }
  return k;
}

/* ------------------------------------------------------------------ Fsm */
typedef struct {
  const orc_prog *prog;
  uint32_t start;
  size_t at;
  int quit_after_match;
  uint32_t last_match_si;
  size_t last_cache_flush;
  orc_dfa_cache *cache;
  const orc_lits *pre;  /* prefix searcher when has_prefix (dfa.rs:1562-1566), else NULL */
} Fsm;

typedef struct { int kind; size_t v; } DResult;  /* kind: 0 Match, 1 NoMatch, 2 Quit */
#define R_MATCH 0
#define R_NOMATCH 1
#define R_QUIT 2

static inline const orc_state *fsm_state(const Fsm *f, uint32_t si) {
  return &f->cache->states[si / f->cache->nclasses];
}

static inline uint32_t byte_class(const Fsm *f, int b) {  /* dfa.rs:1536-1547 */
  if (b == BYTE_EOF) return f->cache->nclasses - 1;
  return f->prog->byte_classes[b];
}

static inline int is_ascii_word_b(int b) {
  if (b == BYTE_EOF) return 0;
  return b == '_' || (b >= '0' && b <= '9') || (b >= 'a' && b <= 'z') || (b >= 'A' && b <= 'Z');
}

static int continue_past_first_match(const Fsm *f) {  /* dfa.rs:1557-1559 */
  return f->prog->is_reverse || f->prog->nmatches > 1;
}

typedef struct { int start, end, start_line, end_line, wb, nwb; } EmptyFlags;

static void follow_epsilons(Fsm *f, uint32_t ip0, orc_sset *q, EmptyFlags fl) {  /* dfa.rs:1073-1134 */
  orc_dfa_cache *c = f->cache;
  c->stack[c->stack_len++] = ip0;
  while (c->stack_len) {
    uint32_t ip = c->stack[--c->stack_len];
    if (orc_sset_contains(q, ip)) continue;
    orc_sset_insert(q, ip);
    const orc_inst *in = &f->prog->insts[ip];
    switch (in->op) {
      case OP_MATCH: case OP_BYTES: break;
      case OP_EMPTY: {
        int ok = 0;
        switch (in->look) {
          case LOOK_START_LINE: ok = fl.start_line; break;
          case LOOK_END_LINE: ok = fl.end_line; break;
          case LOOK_START_TEXT: ok = fl.start; break;
          case LOOK_END_TEXT: ok = fl.end; break;
          case LOOK_WB_ASCII: ok = fl.wb; break;
          case LOOK_NWB_ASCII: ok = fl.nwb; break;
          case LOOK_WB: ok = fl.wb; break;
          case LOOK_NWB: ok = fl.nwb; break;
        }
        if (ok) c->stack[c->stack_len++] = in->x;
        break;
      }
      case OP_SAVE: c->stack[c->stack_len++] = in->x; break;
      case OP_SPLIT:
        c->stack[c->stack_len++] = in->y;
        c->stack[c->stack_len++] = in->x;
        break;
    }
  }
}

static size_t approximate_size(const Fsm *f) {  /* dfa.rs:1586-1588, prog.rs:147-158 */
  const orc_prog *p = f->prog;
  size_t prog_size = (size_t)p->n * 40 + (size_t)p->nmatches * 8 + (size_t)p->ncaps * 24 + 256;
  return f->cache->size + prog_size;
}

/* Transitions::add + add_state (dfa.rs:1479-1512, 1611-1618).  Takes ownership of data. */
static uint32_t add_state(Fsm *f, uint8_t *data, uint32_t len) {
  orc_dfa_cache *c = f->cache;
  size_t si = c->trans_len;
  if (si > STATE_MAX) { free(data); return STATE_UNKNOWN; /* None */ }
  if (c->trans_len + c->nclasses > c->trans_cap) {
    size_t nc = c->trans_cap ? c->trans_cap * 2 : 4096;
    while (nc < c->trans_len + c->nclasses) nc *= 2;
    c->trans = (uint32_t *)realloc(c->trans, nc * 4);
    c->trans_cap = nc;
  }
  for (uint32_t k = 0; k < c->nclasses; ++k) c->trans[si + k] = STATE_UNKNOWN;
  c->trans_len += c->nclasses;
  if (f->prog->has_uwb) {
    for (int b = 128; b < 256; ++b) c->trans[si + f->prog->byte_classes[b]] = STATE_QUIT;
  }
  c->size += c->nclasses * 4 + 2 * (size_t)len + 2 * 16 + 4;
  if (c->nstates == c->states_cap) {
    c->states_cap = c->states_cap ? c->states_cap * 2 : 64;
    c->states = (orc_state *)realloc(c->states, c->states_cap * sizeof(orc_state));
  }
  c->states[c->nstates].data = data;
  c->states[c->nstates].len = len;
  c->nstates++;
  map_insert(c, (uint32_t)(c->nstates - 1));
  return (uint32_t)si;
}

static uint32_t restore_state(Fsm *f, uint8_t *data, uint32_t len) {  /* dfa.rs:1324-1331 */
  uint32_t idx = map_find(f->cache, data, len);
  if (idx != UINT32_MAX) { free(data); return idx * f->cache->nclasses; }
  return add_state(f, data, len);
}

static uint32_t start_ptr(const Fsm *f, uint32_t si) { return f->pre ? si | STATE_START : si; }  /* dfa.rs:1573-1579 */

static uint8_t *dup_state(const orc_state *st) {
  uint8_t *d = (uint8_t *)malloc(st->len ? st->len : 1);
  memcpy(d, st->data, st->len);
  return d;
}

static int clear_cache(Fsm *f) {  /* dfa.rs:1282-1320 */
  orc_dfa_cache *c = f->cache;
  size_t nstates = c->nstates;
  if (c->flush_count >= 3 && f->at >= f->last_cache_flush && (f->at - f->last_cache_flush) <= 10 * nstates)
    return 0;
  f->last_cache_flush = f->at;
  c->flush_count++;
  c->stat_flushes++;
  const orc_state *sst = fsm_state(f, f->start & ~STATE_START);
  uint32_t slen = sst->len;
  uint8_t *sdata = dup_state(sst);
  uint8_t *mdata = NULL;
  uint32_t mlen = 0;
  if (f->last_match_si <= STATE_MAX) {
    const orc_state *m = fsm_state(f, f->last_match_si);
    mlen = m->len;
    mdata = dup_state(m);
  }
  reset_size(c);
  c->trans_len = 0;
  free_states(c);
  map_clear(c);
  for (int i = 0; i < 256; ++i) c->start_states[i] = STATE_UNKNOWN;
  uint32_t sp = restore_state(f, sdata, slen);
  f->start = start_ptr(f, sp);
  if (mdata) f->last_match_si = restore_state(f, mdata, mlen);
  return 1;
}

static int clear_cache_and_save(Fsm *f, uint32_t *current) {  /* dfa.rs:1254-1276 */
  if (f->cache->nstates == 0) return 1;
  if (!current) return clear_cache(f);
  const orc_state *cur = fsm_state(f, *current);
  uint32_t len = cur->len;
  uint8_t *d = dup_state(cur);
  if (!clear_cache(f)) { free(d); return 0; }
  *current = restore_state(f, d, len);
  return 1;
}

/* cached_state_key (dfa.rs:1196-1244): returns malloc'd key or NULL (dead). */
static uint8_t *cached_state_key(Fsm *f, const orc_sset *q, uint8_t *sflags, uint32_t *out_len) {
  uint8_t *d = NULL;
  uint32_t n = 0, cap = 0;
  buf_push(&d, &n, &cap, 0);
  uint32_t prev = 0;
  int cont = continue_past_first_match(f);
  for (size_t k = 0; k < q->n; ++k) {
    uint32_t ip = q->dense[k];
    const orc_inst *in = &f->prog->insts[ip];
    int push = 0, stop = 0;
    switch (in->op) {
      case OP_SAVE: case OP_SPLIT: break;
      case OP_BYTES: push = 1; break;
      case OP_EMPTY: *sflags |= SF_EMPTY; push = 1; break;
      case OP_MATCH: push = 1; stop = !cont; break;
    }
    if (push) { write_vari32(&d, &n, &cap, (int32_t)ip - (int32_t)prev); prev = ip; }
    if (stop) break;
  }
  if (n == 1 && !(*sflags & SF_MATCH)) { free(d); return NULL; }
  d[0] = *sflags;
  *out_len = n;
  return d;
}

/* cached_state (dfa.rs:1154-1184); returns STATE_UNKNOWN for None. */
static uint32_t cached_state(Fsm *f, const orc_sset *q, uint8_t sflags, uint32_t *current) {
  uint32_t len;
  uint8_t *key = cached_state_key(f, q, &sflags, &len);
  if (!key) return STATE_DEAD;
  uint32_t idx = map_find(f->cache, key, len);
  if (idx != UINT32_MAX) { free(key); return idx * f->cache->nclasses; }
  if (approximate_size(f) > f->prog->dfa_size_limit && !clear_cache_and_save(f, current)) {
    free(key);
    return STATE_UNKNOWN;
  }
  return add_state(f, key, len);
}

/* exec_byte (dfa.rs:910-1048); returns STATE_UNKNOWN for None (quit). */
static uint32_t exec_byte(Fsm *f, uint32_t si, int b) {
  orc_dfa_cache *c = f->cache;
  orc_sset *qcur = &c->qcur, *qnext = &c->qnext;
  uint32_t ips_buf_static[64];
  const orc_state *st = fsm_state(f, si);
  uint32_t *ips = st->len <= 64 ? ips_buf_static : (uint32_t *)malloc((size_t)st->len * 4);
  size_t nips = state_ips(st, ips);
  qcur->n = 0;
  for (size_t k = 0; k < nips; ++k) orc_sset_insert(qcur, ips[k]);
  if (ips != ips_buf_static) free(ips);
  uint8_t flags = st->data[0];
  int is_word_last = (flags & SF_WORD) != 0;
  int is_word = is_ascii_word_b(b);
  if (flags & SF_EMPTY) {
    EmptyFlags fl = {0, 0, 0, 0, 0, 0};
    if (b == BYTE_EOF) { fl.end = 1; fl.end_line = 1; }
    else if (b == '\n') fl.end_line = 1;
    if (is_word_last == is_word) fl.nwb = 1; else fl.wb = 1;
    qnext->n = 0;
    for (size_t k = 0; k < qcur->n; ++k) follow_epsilons(f, qcur->dense[k], qnext, fl);
    orc_sset tmp = *qcur; *qcur = *qnext; *qnext = tmp;
  }
  EmptyFlags ef = {0, 0, 0, 0, 0, 0};
  uint8_t sflags = 0;
  ef.start_line = (b == '\n');
  if (is_ascii_word_b(b)) sflags |= SF_WORD;
  qnext->n = 0;
  int cont = continue_past_first_match(f);
  for (size_t k = 0; k < qcur->n; ++k) {
    uint32_t ip = qcur->dense[k];
    const orc_inst *in = &f->prog->insts[ip];
    if (in->op == OP_MATCH) {
      sflags |= SF_MATCH;
      if (!cont) break;
      else if (f->prog->nmatches > 1 && !orc_sset_contains(qnext, ip)) orc_sset_insert(qnext, ip);
    } else if (in->op == OP_BYTES) {
      if (b != BYTE_EOF && in->lo <= b && b <= in->hi) follow_epsilons(f, in->x, qnext, ef);
    }
  }
  int cache = 1;
  if (b == BYTE_EOF && f->prog->nmatches > 1) {
    orc_sset tmp = *qcur; *qcur = *qnext; *qnext = tmp;
    cache = 0;
  }
  uint32_t next = cached_state(f, qnext, sflags, &si);
  if (next == STATE_UNKNOWN) return STATE_UNKNOWN;
  if ((f->start & ~STATE_START) == next) next = start_ptr(f, next);
  if (next <= STATE_MAX && (fsm_state(f, next)->data[0] & SF_MATCH)) next |= STATE_MATCH;
  if (cache) c->trans[si + byte_class(f, b)] = next;
  return next;
}

/* next_state (dfa.rs:1345-1361); STATE_UNKNOWN means None (quit). */
static uint32_t next_state(Fsm *f, uint32_t si, int b) {
  if (si == STATE_DEAD) return STATE_DEAD;
  uint32_t t = f->cache->trans[si + byte_class(f, b)];
  if (t == STATE_UNKNOWN) return exec_byte(f, si, b);
  if (t == STATE_QUIT) return STATE_UNKNOWN;
  return t;
}

static inline uint32_t next_si(const Fsm *f, uint32_t si, const uint8_t *text, size_t i) {  /* dfa.rs:873-900 */
  return f->cache->trans[si + f->prog->byte_classes[text[i]]];
}

/* start_state (dfa.rs:1370-1409); STATE_UNKNOWN means None. */
static uint32_t start_state(Fsm *f, EmptyFlags ef, uint8_t sflags) {
  int flagi = (ef.start ? 1 : 0) | (ef.end ? 2 : 0) | (ef.start_line ? 4 : 0) | (ef.end_line ? 8 : 0) |
              (ef.wb ? 16 : 0) | (ef.nwb ? 32 : 0) | ((sflags & SF_WORD) ? 64 : 0);
  uint32_t s = f->cache->start_states[flagi];
  if (s != STATE_UNKNOWN) return s;
  orc_sset *q = &f->cache->qcur;
  q->n = 0;
  follow_epsilons(f, f->prog->start, q, ef);
  uint32_t sp = cached_state(f, q, sflags, NULL);
  if (sp == STATE_UNKNOWN) return STATE_UNKNOWN;
  sp = start_ptr(f, sp);
  f->cache->start_states[flagi] = sp;
  return sp;
}

static void start_flags(const uint8_t *text, size_t len, size_t at, EmptyFlags *ef, uint8_t *sf) {  /* dfa.rs:1415-1434 */
  memset(ef, 0, sizeof(*ef));
  *sf = 0;
  ef->start = at == 0;
  ef->end = len == 0;
  ef->start_line = at == 0 || text[at - 1] == '\n';
  ef->end_line = len == 0;
  int wl = at > 0 && is_ascii_word_b(text[at - 1]);
  int w = at < len && is_ascii_word_b(text[at]);
  if (wl) *sf |= SF_WORD;
  if (w == wl) ef->nwb = 1; else ef->wb = 1;
}

static void start_flags_reverse(const uint8_t *text, size_t len, size_t at, EmptyFlags *ef, uint8_t *sf) {  /* dfa.rs:1440-1464 */
  memset(ef, 0, sizeof(*ef));
  *sf = 0;
  ef->start = at == len;
  ef->end = len == 0;
  ef->start_line = at == len || text[at] == '\n';
  ef->end_line = len == 0;
  int wl = at < len && is_ascii_word_b(text[at]);
  int w = at > 0 && is_ascii_word_b(text[at - 1]);
  if (wl) *sf |= SF_WORD;
  if (w == wl) ef->nwb = 1; else ef->wb = 1;
}

static DResult set_non_match(DResult r, size_t at) { if (r.kind == R_NOMATCH) r.v = at; return r; }

static int just_matches(const Fsm *f, uint32_t si) {
  const orc_state *st = fsm_state(f, si);
  uint32_t buf[256];
  uint32_t *ips = st->len <= 256 ? buf : (uint32_t *)malloc((size_t)st->len * 4);
  size_t n = state_ips(st, ips);
  int all = 1;
  for (size_t k = 0; k < n; ++k) if (f->prog->insts[ips[k]].op != OP_MATCH) { all = 0; break; }
  if (ips != buf) free(ips);
  return all;
}

/* exec_at (dfa.rs:576-764).  *stop receives the input position where the scan ended. */
static DResult exec_at(Fsm *f, const uint8_t *text, size_t len, size_t *stop) {
  DResult result = {R_NOMATCH, f->at};
  uint32_t prev_si = f->start, nsi = f->start;
  size_t at = f->at;
  /* the table and class map in locals (next_si, dfa.rs:873-900); the table
   * moves only when the slow path adds a state, so it is reloaded per round */
  const uint8_t *cls = f->prog->byte_classes;
  const uint32_t *T;
  while (at < len) {
    T = f->cache->trans;
    while (nsi <= STATE_MAX && at < len) {
      prev_si = T[(nsi) + cls[text[at]]];
      at += 1;
      if (prev_si > STATE_MAX || at + 2 >= len) { uint32_t t = prev_si; prev_si = nsi; nsi = t; break; }
      nsi = T[(prev_si) + cls[text[at]]];
      at += 1;
      if (nsi > STATE_MAX) break;
      prev_si = T[(nsi) + cls[text[at]]];
      at += 1;
      if (prev_si > STATE_MAX) { uint32_t t = prev_si; prev_si = nsi; nsi = t; break; }
      nsi = T[(prev_si) + cls[text[at]]];
      at += 1;
    }
    if (nsi & STATE_MATCH) {
      nsi &= ~STATE_MATCH;
      result.kind = R_MATCH; result.v = at - 1;
      if (f->quit_after_match) { *stop = at; return result; }
      f->last_match_si = nsi;
      prev_si = nsi;
      if (f->prog->nmatches > 1 && just_matches(f, nsi)) { *stop = at; return result; }
      size_t cur = at;
      while ((nsi & ~STATE_MATCH) == prev_si && at + 2 < len) {
        nsi = T[(nsi & ~STATE_MATCH) + cls[text[at]]];
        at += 1;
      }
      if (at > cur) { result.kind = R_MATCH; result.v = at - 2; }
    } else if (nsi & STATE_START) {
      /* dfa.rs:700-711: in the start state, skip to the next prefix occurrence */
      nsi &= ~STATE_START;
      prev_si = nsi;
      if (f->pre) {
        size_t s, e;
        if (!orc_lits_find(f->pre, text + at, len - at, &s, &e)) {
          *stop = len;
          result.kind = R_NOMATCH;
          result.v = len;
          return result;
        }
        at += s;
      }
    } else if (nsi >= STATE_UNKNOWN) {
      if (nsi == STATE_QUIT) { *stop = at; result.kind = R_QUIT; return result; }
      int byte = text[at - 1];
      prev_si &= STATE_MAX;
      f->at = at;
      uint32_t n2 = next_state(f, prev_si, byte);
      if (n2 == STATE_UNKNOWN) { *stop = at; result.kind = R_QUIT; return result; }
      if (n2 == STATE_DEAD) { *stop = at; return set_non_match(result, at); }
      nsi = n2;
      if (nsi & STATE_MATCH) {
        nsi &= ~STATE_MATCH;
        result.kind = R_MATCH; result.v = at - 1;
        if (f->quit_after_match) { *stop = at; return result; }
        f->last_match_si = nsi;
      }
      prev_si = nsi;
    } else {
      prev_si = nsi;
    }
  }
  *stop = len;
  prev_si &= STATE_MAX;
  uint32_t n3 = next_state(f, prev_si, BYTE_EOF);
  if (n3 == STATE_UNKNOWN) { result.kind = R_QUIT; return result; }
  if (n3 == STATE_DEAD) return set_non_match(result, len);
  prev_si = n3 & ~STATE_START;
  if (prev_si & STATE_MATCH) {
    prev_si &= ~STATE_MATCH;
    f->last_match_si = prev_si;
    result.kind = R_MATCH; result.v = len;
  }
  return result;
}

/* exec_at_reverse (dfa.rs:768-866) */
static DResult exec_at_reverse(Fsm *f, const uint8_t *text, size_t len, size_t *consumed) {
  (void)len;
  DResult result = {R_NOMATCH, f->at};
  uint32_t prev_si = f->start, nsi = f->start;
  size_t at = f->at;
  const size_t at0 = f->at;
  const uint8_t *cls = f->prog->byte_classes;
  const uint32_t *T;
  while (at > 0) {
    T = f->cache->trans;
    while (nsi <= STATE_MAX && at > 0) {
      at -= 1;
      prev_si = T[(nsi) + cls[text[at]]];
      if (prev_si > STATE_MAX || at <= 4) { uint32_t t = prev_si; prev_si = nsi; nsi = t; break; }
      at -= 1;
      nsi = T[(prev_si) + cls[text[at]]];
      if (nsi > STATE_MAX) break;
      at -= 1;
      prev_si = T[(nsi) + cls[text[at]]];
      if (prev_si > STATE_MAX) { uint32_t t = prev_si; prev_si = nsi; nsi = t; break; }
      at -= 1;
      nsi = T[(prev_si) + cls[text[at]]];
    }
    if (nsi & STATE_MATCH) {
      nsi &= ~STATE_MATCH;
      result.kind = R_MATCH; result.v = at + 1;
      if (f->quit_after_match) { *consumed = at0 - at; return result; }
      f->last_match_si = nsi;
      prev_si = nsi;
      size_t cur = at;
      while ((nsi & ~STATE_MATCH) == prev_si && at >= 2) {
        at -= 1;
        nsi = T[(nsi & ~STATE_MATCH) + cls[text[at]]];
      }
      if (at < cur) { result.kind = R_MATCH; result.v = at + 2; }
    } else if (nsi >= STATE_UNKNOWN) {
      if (nsi == STATE_QUIT) { *consumed = at0 - at; result.kind = R_QUIT; return result; }
      int byte = text[at];
      prev_si &= STATE_MAX;
      f->at = at;
      uint32_t n2 = next_state(f, prev_si, byte);
      if (n2 == STATE_UNKNOWN) { *consumed = at0 - at; result.kind = R_QUIT; return result; }
      if (n2 == STATE_DEAD) { *consumed = at0 - at; return set_non_match(result, at); }
      nsi = n2;
      if (nsi & STATE_MATCH) {
        nsi &= ~STATE_MATCH;
        result.kind = R_MATCH; result.v = at + 1;
        if (f->quit_after_match) { *consumed = at0 - at; return result; }
        f->last_match_si = nsi;
      }
      prev_si = nsi;
    } else {
      prev_si = nsi;
    }
  }
  *consumed = at0;
  uint32_t n3 = next_state(f, prev_si, BYTE_EOF);
  if (n3 == STATE_UNKNOWN) { result.kind = R_QUIT; return result; }
  if (n3 == STATE_DEAD) return set_non_match(result, 0);
  prev_si = n3;
  if (prev_si & STATE_MATCH) {
    prev_si &= ~STATE_MATCH;
    f->last_match_si = prev_si;
    result.kind = R_MATCH; result.v = 0;
  }
  return result;
}

static void fsm_init(Fsm *f, const orc_prog *p, orc_dfa_cache *c, int qam, size_t at) {
  f->prog = p;
  f->start = 0;
  f->at = at;
  f->quit_after_match = qam;
  f->last_match_si = STATE_UNKNOWN;
  f->last_cache_flush = at;
  f->cache = c;
  f->pre = NULL;
}

/* Fsm::forward (dfa.rs:459-489).  Returns kind, *pos = value, *stop = scan end. */
int orc_dfa_forward(const orc_prog *p, orc_dfa_cache *c, int quit_after_match, const uint8_t *text, size_t len,
                    size_t at, size_t *pos, size_t *stop) {
  return orc_dfa_forward_pfx(p, c, quit_after_match, NULL, text, len, at, pos, stop);
}

int orc_dfa_forward_pfx(const orc_prog *p, orc_dfa_cache *c, int quit_after_match, const orc_lits *pre,
                        const uint8_t *text, size_t len, size_t at, size_t *pos, size_t *stop) {
  Fsm f;
  fsm_init(&f, p, c, quit_after_match, at);
  /* has_prefix (dfa.rs:1562-1566) */
  if (pre && pre->matcher != 0 && pre->n > 0 && !p->is_reverse && !p->anchored_start) f.pre = pre;
  EmptyFlags ef;
  uint8_t sf;
  start_flags(text, len, at, &ef, &sf);
  uint32_t s = start_state(&f, ef, sf);
  *stop = at;
  if (s == STATE_UNKNOWN) return R_QUIT;
  if (s == STATE_DEAD) { *pos = at; return R_NOMATCH; }
  f.start = s;
  DResult r = exec_at(&f, text, len, stop);
  *pos = r.v;
  return r.kind;
}

/* Fsm::reverse (dfa.rs:492-522); text is the slice, at the reverse start. */
int orc_dfa_reverse(const orc_prog *p, orc_dfa_cache *c, int quit_after_match, const uint8_t *text, size_t len,
                    size_t at, size_t *pos, size_t *consumed) {
  Fsm f;
  fsm_init(&f, p, c, quit_after_match, at);
  EmptyFlags ef;
  uint8_t sf;
  start_flags_reverse(text, len, at, &ef, &sf);
  uint32_t s = start_state(&f, ef, sf);
  *consumed = 0;
  if (s == STATE_UNKNOWN) return R_QUIT;
  if (s == STATE_DEAD) { *pos = at; return R_NOMATCH; }
  f.start = s;
  DResult r = exec_at_reverse(&f, text, len, consumed);
  *pos = r.v;
  return r.kind;
}

/* Fsm::forward_many (dfa.rs:525-570) */
int orc_dfa_forward_many(const orc_prog *p, orc_dfa_cache *c, uint8_t *matches, const uint8_t *text, size_t len,
                         size_t at, size_t *pos, size_t *stop) {
  Fsm f;
  fsm_init(&f, p, c, 0, at);
  EmptyFlags ef;
  uint8_t sf;
  start_flags(text, len, at, &ef, &sf);
  uint32_t s = start_state(&f, ef, sf);
  *stop = at;
  if (s == STATE_UNKNOWN) return R_QUIT;
  if (s == STATE_DEAD) { *pos = at; return R_NOMATCH; }
  f.start = s;
  DResult r = exec_at(&f, text, len, stop);
  *pos = r.v;
  if (r.kind == R_MATCH) {
    if (p->nmatches == 1) {
      matches[0] = 1;
    } else {
      const orc_state *st = fsm_state(&f, f.last_match_si);
      uint32_t *ips = (uint32_t *)malloc(((size_t)st->len + 1) * 4);
      size_t n = state_ips(st, ips);
      for (size_t k = 0; k < n; ++k) {
        const orc_inst *in = &p->insts[ips[k]];
        if (in->op == OP_MATCH) matches[in->x] = 1;
      }
      free(ips);
    }
  }
  return r.kind;
}

size_t orc_dfa_cache_nstates(const orc_dfa_cache *c) { return c->nstates; }
