/*
 * TEST INFRASTRUCTURE ONLY.  Restatement of the reference Pike VM,
 * src/pikevm.rs (exec 102-128, exec_ 130-223, step 237-280, add/add_step
 * 284-352, Threads 355-377) over a byte Program with the reference's
 * ByteInput (src/input.rs:227-318, only_utf8 = false for bytes::Regex) and
 * its UTF-8 helpers (src/utf8.rs:83-175) for the Unicode word boundary.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle_int.h"
#include "unicode_word.h"

#define NONE_POS SIZE_MAX
#define NO_CHAR UINT32_MAX

typedef struct { int is_ip; uint32_t ip; size_t slot; size_t pos; } Frame;

struct orc_pike_cache {
  orc_sset set[2];
  size_t *caps[2];
  size_t slots_per_thread;
  Frame *stack;
  size_t stack_len, stack_cap;
};

orc_pike_cache *orc_pike_cache_new(const orc_prog *p) {
  orc_pike_cache *c = (orc_pike_cache *)calloc(1, sizeof(*c));
  c->slots_per_thread = (size_t)p->ncaps * 2;
  for (int k = 0; k < 2; ++k) {
    orc_sset_init(&c->set[k], p->n);
    c->caps[k] = (size_t *)malloc((c->slots_per_thread * p->n + 1) * sizeof(size_t));
    for (size_t i = 0; i < c->slots_per_thread * p->n; ++i) c->caps[k][i] = NONE_POS;
  }
  c->stack_cap = 64;
  c->stack = (Frame *)malloc(c->stack_cap * sizeof(Frame));
  return c;
}

void orc_pike_cache_free(orc_pike_cache *c) {
  if (!c) return;
  for (int k = 0; k < 2; ++k) { orc_sset_free(&c->set[k]); free(c->caps[k]); }
  free(c->stack);
  free(c);
}

static void push(orc_pike_cache *c, Frame f) {
  if (c->stack_len == c->stack_cap) {
    c->stack_cap *= 2;
    c->stack = (Frame *)realloc(c->stack, c->stack_cap * sizeof(Frame));
  }
  c->stack[c->stack_len++] = f;
}

/* ------------------------------------------------------------ utf8.rs */
static uint32_t decode_utf8(const uint8_t *s, size_t n, size_t *len) {  /* utf8.rs:83-150 */
  if (n == 0) return NO_CHAR;
  uint8_t b0 = s[0];
  if (b0 <= 0x7F) { *len = 1; return b0; }
  if (b0 >= 0xC0 && b0 <= 0xDF) {
    if (n < 2 || (s[1] & 0xC0) != 0x80) return NO_CHAR;
    uint32_t cp = ((uint32_t)(b0 & 0x1F) << 6) | (s[1] & 0x3F);
    if (cp < 0x80 || cp > 0x7FF) return NO_CHAR;
    *len = 2; return cp;
  }
  if (b0 >= 0xE0 && b0 <= 0xEF) {
    if (n < 3 || (s[1] & 0xC0) != 0x80 || (s[2] & 0xC0) != 0x80) return NO_CHAR;
    uint32_t cp = ((uint32_t)(b0 & 0x0F) << 12) | ((uint32_t)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
    if (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF)) return NO_CHAR;
    *len = 3; return cp;
  }
  if (b0 >= 0xF0 && b0 <= 0xF7) {
    if (n < 4 || (s[1] & 0xC0) != 0x80 || (s[2] & 0xC0) != 0x80 || (s[3] & 0xC0) != 0x80) return NO_CHAR;
    uint32_t cp = ((uint32_t)(b0 & 0x07) << 18) | ((uint32_t)(s[1] & 0x3F) << 12) |
                  ((uint32_t)(s[2] & 0x3F) << 6) | (s[3] & 0x3F);
    if (cp < 0x10000 || cp > 0x10FFFF) return NO_CHAR;
    *len = 4; return cp;
  }
  return NO_CHAR;
}

static int is_start_byte(uint8_t b) { return (b & 0xC0) != 0x80; }

static uint32_t decode_last_utf8(const uint8_t *s, size_t n) {  /* utf8.rs:154-175 */
  if (n == 0) return NO_CHAR;
  size_t start = n - 1;
  if (s[start] <= 0x7F) return s[start];
  size_t lim = n >= 4 ? n - 4 : 0;
  while (start > lim) {
    start -= 1;
    if (is_start_byte(s[start])) break;
  }
  size_t len;
  uint32_t cp = decode_utf8(s + start, n - start, &len);
  if (cp == NO_CHAR) return NO_CHAR;
  if (len < n - start) return NO_CHAR;
  return cp;
}

static int is_word_char(uint32_t c) {  /* regex-syntax lib.rs:1729-1744 */
  if (c == NO_CHAR) return 0;
  if (c == '_' || (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) return 1;
  size_t lo = 0, hi = ORC_PERLW_N;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (c < ORC_PERLW[2 * mid]) hi = mid;
    else if (c > ORC_PERLW[2 * mid + 1]) lo = mid + 1;
    else return 1;
  }
  return 0;
}

static int is_word_byte_char(uint32_t c) {  /* input.rs Char::is_word_byte */
  if (c == NO_CHAR || c > 0x7F) return 0;
  return c == '_' || (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}

typedef struct { const uint8_t *text; size_t len; } In;

static uint32_t next_char(const In *in, size_t pos) {
  size_t l;
  if (pos > in->len) return NO_CHAR;
  return decode_utf8(in->text + pos, in->len - pos, &l);
}
static uint32_t prev_char(const In *in, size_t pos) { return decode_last_utf8(in->text, pos); }

static int is_empty_match(const In *in, size_t pos, uint8_t look) {  /* input.rs:268-318 */
  switch (look) {
    case LOOK_START_LINE: return pos == 0 || prev_char(in, pos) == '\n';
    case LOOK_END_LINE: return pos == in->len || next_char(in, pos) == '\n';
    case LOOK_START_TEXT: return pos == 0;
    case LOOK_END_TEXT: return pos == in->len;
    case LOOK_WB: return is_word_char(prev_char(in, pos)) != is_word_char(next_char(in, pos));
    case LOOK_NWB: return is_word_char(prev_char(in, pos)) == is_word_char(next_char(in, pos));
    case LOOK_WB_ASCII: return is_word_byte_char(prev_char(in, pos)) != is_word_byte_char(next_char(in, pos));
    case LOOK_NWB_ASCII: return is_word_byte_char(prev_char(in, pos)) == is_word_byte_char(next_char(in, pos));
  }
  return 0;
}

/* add + add_step (pikevm.rs:284-352).  thread_caps has tc_len entries. */
static void add(const orc_prog *p, orc_pike_cache *c, const In *in, int nl, size_t *thread_caps, size_t tc_len,
                uint32_t ip0, size_t at) {
  orc_sset *set = &c->set[nl];
  size_t spt = c->slots_per_thread;
  Frame f0 = {1, ip0, 0, 0};
  push(c, f0);
  while (c->stack_len) {
    Frame fr = c->stack[--c->stack_len];
    if (!fr.is_ip) { thread_caps[fr.slot] = fr.pos; continue; }
    uint32_t ip = fr.ip;
    for (;;) {
      if (orc_sset_contains(set, ip)) break;
      orc_sset_insert(set, ip);
      const orc_inst *i = &p->insts[ip];
      if (i->op == OP_EMPTY) {
        if (is_empty_match(in, at, i->look)) { ip = i->x; continue; }
        break;
      } else if (i->op == OP_SAVE) {
        if (i->y < tc_len) {
          Frame cf = {0, 0, i->y, thread_caps[i->y]};
          push(c, cf);
          thread_caps[i->y] = at;
        }
        ip = i->x;
        continue;
      } else if (i->op == OP_SPLIT) {
        Frame sf = {1, i->y, 0, 0};
        push(c, sf);
        ip = i->x;
        continue;
      } else {  /* Match / Bytes: record the thread's captures */
        size_t *t = c->caps[nl] + (size_t)ip * spt;
        size_t m = spt < tc_len ? spt : tc_len;
        for (size_t k = 0; k < m; ++k) t[k] = thread_caps[k];
        break;
      }
    }
  }
}

int orc_pike_exec(const orc_prog *p, orc_pike_cache *c, uint8_t *matches, size_t nmatches, size_t *slots,
                  size_t nslots, int quit_after_match, const uint8_t *text, size_t len, size_t start) {
  In in = {text, len};
  int cl = 0, nl = 1;
  int matched = 0, all_matched = 0;
  size_t spt = c->slots_per_thread;
  c->set[0].n = 0;
  c->set[1].n = 0;
  size_t at = start;
  for (;;) {
    if (c->set[cl].n == 0) {
      if ((matched && nmatches <= 1) || all_matched || (at != 0 && p->anchored_start)) break;
    }
    if (c->set[cl].n == 0 || (!p->anchored_start && !all_matched))
      add(p, c, &in, cl, slots, nslots, p->start, at);
    size_t at_next = at + 1;
    int brk = 0;
    for (size_t i = 0; i < c->set[cl].n; ++i) {
      uint32_t ip = c->set[cl].dense[i];
      const orc_inst *inst = &p->insts[ip];
      size_t *tcaps = c->caps[cl] + (size_t)ip * spt;
      int step_matched = 0;
      if (inst->op == OP_MATCH) {  /* step (pikevm.rs:237-280) */
        if (inst->x < nmatches) matches[inst->x] = 1;
        size_t m = nslots < spt ? nslots : spt;
        for (size_t k = 0; k < m; ++k) slots[k] = tcaps[k];
        step_matched = 1;
      } else if (inst->op == OP_BYTES) {
        if (at < len && inst->lo <= text[at] && text[at] <= inst->hi)
          add(p, c, &in, nl, tcaps, spt, inst->x, at_next);
      }
      if (step_matched) {
        matched = 1;
        if (!all_matched) {
          int all = 1;
          for (size_t k = 0; k < nmatches; ++k) if (!matches[k]) { all = 0; break; }
          all_matched = all;
        }
        if (quit_after_match) { brk = 2; break; }
        if (p->nmatches == 1) break;
      }
    }
    if (brk == 2) break;
    if (at >= len) break;
    at = at_next;
    int t = cl; cl = nl; nl = t;
    c->set[nl].n = 0;
  }
  return matched;
}
