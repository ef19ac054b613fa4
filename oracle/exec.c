/*
 * TEST INFRASTRUCTURE ONLY.  Restatement of the reference dispatcher for
 * the DFA match types, src/exec.rs:
 *   shortest_match_at  382-420   (Dfa arm; Quit -> shortest_nfa)
 *   is_match_at        427-468   (Dfa arm; Quit -> match_nfa)
 *   find_at            473-514   (Dfa arm; Quit -> find_nfa)
 *   find_dfa_forward   632-662
 *   find_dfa_anchored_reverse 671-688 and the DfaAnchoredReverse arms of
 *                      the above (chosen at exec.rs:1175-1177 for regexes
 *                      anchored at the end but not at the start)
 *   many_matches_at    998-1038  (DfaMany arm; Quit -> exec_nfa)
 * and the iteration rule of src/re_trait.rs:197-221 (Matches::next).
 * Engine choice is result-neutral in the reference (HACKING.md:60-61) except
 * for DfaAnchoredReverse, which runs the reverse DFA over text[start..] from
 * the end: the byte before `start` is not visible to it (a match at `start`
 * of e.g. `\bx$` or `(?m)^x$` is found where the forward DFA's look-behind
 * rejects it), so that arm is restated as well; the literal arms answer as
 * the DFA arms.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_int.h"

#define R_MATCH 0
#define R_NOMATCH 1
#define R_QUIT 2

orc_prog *orc_prog_new(const orc_inst *insts, uint32_t n, uint32_t start, const uint8_t *byte_classes,
                       int is_reverse, int anchored_start, int anchored_end, int has_uwb, uint32_t ncaps,
                       size_t dfa_size_limit) {
  orc_prog *p = (orc_prog *)calloc(1, sizeof(orc_prog));
  p->insts = (orc_inst *)malloc((n ? n : 1) * sizeof(orc_inst));
  memcpy(p->insts, insts, n * sizeof(orc_inst));
  p->n = n;
  p->start = start;
  memcpy(p->byte_classes, byte_classes, 256);
  p->is_reverse = is_reverse;
  p->anchored_start = anchored_start;
  p->anchored_end = anchored_end;
  p->has_uwb = has_uwb;
  p->ncaps = ncaps;
  p->dfa_size_limit = dfa_size_limit;
  for (uint32_t i = 0; i < n; ++i) if (insts[i].op == OP_MATCH) p->nmatches++;
  return p;
}

void orc_prog_free(orc_prog *p) {
  if (!p) return;
  free(p->insts);
  free(p);
}

orc_regex *orc_regex_new(orc_prog *nfa, orc_prog *fwd, orc_prog *rev) {
  orc_regex *r = (orc_regex *)calloc(1, sizeof(orc_regex));
  r->nfa = nfa;
  r->fwd = fwd;
  r->rev = rev;
  r->mt = -1;
  return r;
}

static void lits_free(orc_lits *l) {
  for (size_t i = 0; i < l->n; ++i) free(l->lit[i]);
  free(l->lit);
  free(l->len);
  free(l->pair);
  free(l->quad);
  memset(l, 0, sizeof(*l));
}

void orc_regex_free(orc_regex *r) {
  if (!r) return;
  orc_prog_free(r->nfa);
  orc_prog_free(r->fwd);
  orc_prog_free(r->rev);
  lits_free(&r->pre);
  lits_free(&r->suf);
  free(r->lcs);
  free(r);
}

static inline uint32_t quad_hash(uint32_t w) { return (w * 0x9E3779B1u) >> 16; }

static void lits_parse(orc_lits *l, const uint8_t *b, size_t n, int matcher) {
  lits_free(l);
  l->matcher = matcher;
  for (size_t i = 0; i + 5 <= n;) {
    uint32_t k;
    memcpy(&k, b + i + 1, 4);
    l->lit = (uint8_t **)realloc(l->lit, (l->n + 1) * sizeof(uint8_t *));
    l->len = (size_t *)realloc(l->len, (l->n + 1) * sizeof(size_t));
    l->lit[l->n] = (uint8_t *)malloc(k ? k : 1);
    memcpy(l->lit[l->n], b + i + 5, k);
    l->len[l->n] = k;
    l->n++;
    i += 5 + k;
  }
  l->pair = (uint8_t *)calloc(65536 / 8, 1);
  l->quad = (uint8_t *)calloc(65536 / 8, 1);
  for (size_t j = 0; j < l->n; ++j) {
    if (l->len[j] == 0) { l->any_empty = 1; continue; }
    if (l->len[j] >= 4) {
      uint32_t w;
      memcpy(&w, l->lit[j], 4);
      const uint32_t h = quad_hash(w);
      l->quad[h >> 3] |= (uint8_t)(1u << (h & 7));
      l->any_long = 1;
      continue;
    }
    l->any_short = 1;
    const uint8_t b0 = l->lit[j][0];
    l->first[b0] = 1;
    if (l->len[j] == 1) { l->single[b0] = 1; continue; }
    const unsigned k = ((unsigned)b0 << 8) | l->lit[j][1];
    l->pair[k >> 3] |= (uint8_t)(1u << (k & 7));
  }
}

void orc_regex_set_exec(orc_regex *r, int match_type, const uint8_t *pre, size_t pre_len, int pre_matcher,
                        const uint8_t *suf, size_t suf_len, int suf_matcher, const uint8_t *lcs, size_t lcs_len) {
  r->mt = match_type;
  lits_parse(&r->pre, pre, pre_len, pre_matcher);
  lits_parse(&r->suf, suf, suf_len, suf_matcher);
  free(r->lcs);
  r->lcs = (uint8_t *)malloc(lcs_len ? lcs_len : 1);
  memcpy(r->lcs, lcs, lcs_len);
  r->lcs_len = lcs_len;
}

orc_cache *orc_cache_new(const orc_regex *r) {
  orc_cache *c = (orc_cache *)calloc(1, sizeof(orc_cache));
  if (r->fwd) c->fwd = orc_dfa_cache_new(r->fwd);
  if (r->rev) c->rev = orc_dfa_cache_new(r->rev);
  if (r->nfa) c->pike = orc_pike_cache_new(r->nfa);
  return c;
}

void orc_cache_free(orc_cache *c) {
  if (!c) return;
  orc_dfa_cache_free(c->fwd);
  orc_dfa_cache_free(c->rev);
  orc_pike_cache_free(c->pike);
  free(c);
}

void orc_cache_stats(const orc_cache *c, orc_stats *out) {
  *out = c->st;
  out->flushes = (c->fwd ? c->fwd->stat_flushes : 0) + (c->rev ? c->rev->stat_flushes : 0);
  out->states = c->fwd ? orc_dfa_cache_nstates(c->fwd) : 0;
}

void orc_cache_reset_stats(orc_cache *c) { memset(&c->st, 0, sizeof(c->st)); }

/* exec.rs:840-855 find_nfa (Pike VM, slots [None, None]) */
int orc_find_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start, size_t *ms,
                 size_t *me) {
  uint8_t m[1] = {0};
  size_t slots[2] = {SIZE_MAX, SIZE_MAX};
  if (!orc_pike_exec(r->nfa, c->pike, m, 1, slots, 2, 0, text, len, start)) return 0;
  if (slots[0] == SIZE_MAX || slots[1] == SIZE_MAX) return 0;
  *ms = slots[0];
  *me = slots[1];
  return 1;
}

int orc_captures_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start, size_t *slots,
                     size_t nslots) {
  uint8_t m[1] = {0};
  for (size_t i = 0; i < nslots; ++i) slots[i] = SIZE_MAX;
  return orc_pike_exec(r->nfa, c->pike, m, 1, slots, nslots, 0, text, len, start);
}

/* exec.rs:1175-1177: a single regex anchored at the end and not at the start
 * runs the reverse DFA from the end of the text (MatchType::DfaAnchoredReverse;
 * Literal(AnchoredEnd), chosen before it for complete suffixes, answers the
 * same: such regexes have no assertions). */
static int anchored_rev(const orc_regex *r) {
  return r->rev && r->nfa && r->nfa->nmatches == 1 && !r->nfa->anchored_start && r->nfa->anchored_end;
}

/* exec.rs:671-688 find_dfa_anchored_reverse (quit_after_match: the
 * is_match / shortest_match arms, exec.rs:395-406, 442-453) */
static int find_dfa_anchored_reverse(const orc_regex *r, orc_cache *c, int quit_after_match, const uint8_t *text,
                                     size_t len, size_t start, size_t *ms, size_t *me) {
  size_t s, consumed;
  int k = orc_dfa_reverse(r->rev, c->rev, quit_after_match, text + start, len - start, len - start, &s, &consumed);
  c->st.rev_bytes += consumed;
  if (k != R_MATCH) return k;
  *ms = start + s;
  *me = len;
  return R_MATCH;
}

/* The forward DFA's prefix literals (dfa.prefixes = nfa.prefixes,
 * exec.rs:308-311), when the product exported them (orc_regex_set_exec). */
static const orc_lits *dfa_prefixes(const orc_regex *r) { return r->mt >= 0 ? &r->pre : NULL; }

/* exec.rs:632-662 find_dfa_forward */
static int find_dfa_forward(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                            size_t *ms, size_t *me) {
  size_t end, stop;
  int k = orc_dfa_forward_pfx(r->fwd, c->fwd, 0, dfa_prefixes(r), text, len, start, &end, &stop);
  c->st.fwd_bytes += stop - start;
  if (k != R_MATCH) return k;
  if (end == start) { *ms = start; *me = start; return R_MATCH; }
  size_t s, consumed;
  int k2 = orc_dfa_reverse(r->rev, c->rev, 0, text + start, len - start, end - start, &s, &consumed);
  c->st.rev_bytes += consumed;
  if (k2 != R_MATCH) return k2;
  *ms = start + s;
  *me = end;
  return R_MATCH;
}

/* Leftmost occurrence of `needle` in hay[0..n) (memmem), -1 if none. */
static long find_sub(const uint8_t *hay, size_t n, const uint8_t *needle, size_t k) {
  if (k == 0) return 0;
  for (size_t i = 0; i + k <= n;) {
    const uint8_t *p = (const uint8_t *)memchr(hay + i, needle[0], n - k + 1 - i);
    if (!p) return -1;
    i = (size_t)(p - hay);
    if (memcmp(p, needle, k) == 0) return (long)i;
    ++i;
  }
  return -1;
}

/* LiteralSearcher::find (src/literals.rs:92-103) over hay[0..n): Empty
 * matches the empty string at 0; Bytes the first byte of the set; one
 * literal its first occurrence; several (Teddy / Aho-Corasick) the leftmost
 * occurrence of any (the set is unambiguous: no member is a substring of
 * another, so one literal at most occurs at a position; at a tie the first
 * literal in order is taken).  One forward pass: a position is tested only
 * when its first four bytes hash like a literal's (or its first bytes begin
 * a literal of 1-3 bytes: lits_parse's tables), so a find_iter over a long
 * text stays linear. */
static int lit_at(const orc_lits *l, const uint8_t *hay, size_t n, size_t i, size_t *s, size_t *e) {
  for (size_t j = 0; j < l->n; ++j) {
    const size_t k = l->len[j];
    if (k <= n - i && memcmp(hay + i, l->lit[j], k) == 0) {
      *s = i;
      *e = i + k;
      return 1;
    }
  }
  return 0;
}

/* memchr / memchr2 / memchr3 (SingleByteSet::find, literals.rs:353-361):
 * the first byte of hay[0..n) in {a, b, c} (k of them), SWAR 8 bytes a step */
static inline uint64_t zero_bytes(uint64_t x) { return (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull; }
static long memchr_k(const uint8_t *hay, size_t n, int k, uint8_t a, uint8_t b, uint8_t c) {
  const uint64_t ra = 0x0101010101010101ull * a, rb = 0x0101010101010101ull * b, rc = 0x0101010101010101ull * c;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, hay + i, 8);
    uint64_t z = zero_bytes(w ^ ra);
    if (k > 1) z |= zero_bytes(w ^ rb);
    if (k > 2) z |= zero_bytes(w ^ rc);
    if (z) break;  /* (the SWAR test can flag a byte after a true hit only: rescan bytewise) */
  }
  for (; i < n; ++i)
    if (hay[i] == a || (k > 1 && hay[i] == b) || (k > 2 && hay[i] == c)) return (long)i;
  return -1;
}

int orc_lits_find(const orc_lits *l, const uint8_t *hay, size_t n, size_t *s, size_t *e) {
  if (l->matcher == 0) { *s = *e = 0; return 1; }
  if (l->matcher == 1 && l->n <= 3 && !l->any_empty) {  /* Bytes: every literal is one byte */
    const uint8_t a = l->lit[0][0], b = l->n > 1 ? l->lit[1][0] : a, c = l->n > 2 ? l->lit[2][0] : a;
    const long i = memchr_k(hay, n, (int)l->n, a, b, c);
    if (i < 0) return 0;
    *s = (size_t)i;
    *e = (size_t)i + 1;
    return 1;
  }
  if (l->any_empty) return lit_at(l, hay, n, 0, s, e);
  for (size_t i = 0; i < n; ++i) {
    int cand = 0;
    if (l->any_long && i + 4 <= n) {
      uint32_t w;
      memcpy(&w, hay + i, 4);
      const uint32_t h = quad_hash(w);
      cand = (l->quad[h >> 3] >> (h & 7)) & 1;
    }
    if (!cand && l->any_short) {
      const uint8_t b = hay[i];
      if (l->single[b]) cand = 1;
      else if (l->first[b] && i + 1 < n) {
        const unsigned k = ((unsigned)b << 8) | hay[i + 1];
        cand = (l->pair[k >> 3] >> (k & 7)) & 1;
      }
    }
    if (cand && lit_at(l, hay, n, i, s, e)) return 1;
  }
  return 0;
}

/* find_start / find_end (literals.rs:105-128): the first literal of iter()
 * (Empty yields none) that the text starts / ends with. */
static int lits_find_start(const orc_lits *l, const uint8_t *hay, size_t n, size_t *s, size_t *e) {
  if (l->matcher == 0) return 0;
  for (size_t j = 0; j < l->n; ++j)
    if (l->len[j] <= n && memcmp(hay, l->lit[j], l->len[j]) == 0) { *s = 0; *e = l->len[j]; return 1; }
  return 0;
}
static int lits_find_end(const orc_lits *l, const uint8_t *hay, size_t n, size_t *s, size_t *e) {
  if (l->matcher == 0) return 0;
  for (size_t j = 0; j < l->n; ++j)
    if (l->len[j] <= n && memcmp(hay + n - l->len[j], l->lit[j], l->len[j]) == 0) {
      *s = n - l->len[j];
      *e = n;
      return 1;
    }
  return 0;
}

/* exec.rs:601-625 find_literals */
static int find_literals(const orc_regex *r, const uint8_t *text, size_t len, size_t start, size_t *ms, size_t *me) {
  size_t s, e;
  int ok;
  if (r->mt == 0) ok = orc_lits_find(&r->pre, text + start, len - start, &s, &e);
  else if (r->mt == 1) ok = lits_find_start(&r->pre, text + start, len - start, &s, &e);
  else ok = lits_find_end(&r->suf, text + start, len - start, &s, &e);
  if (!ok) return 0;
  *ms = start + s;
  *me = start + e;
  return 1;
}

/* exec.rs:725-756 exec_dfa_reverse_suffix.  Returns R_MATCH / R_NOMATCH /
 * R_QUIT, or -1 for None (the reverse scan reached its slice start: give up
 * to the forward DFA).  Each reverse scan sees only text[start..end], the
 * previous suffix occurrence's end to this one's (its look-around at both
 * slice edges is that of a text edge). */
static int exec_dfa_reverse_suffix(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len,
                                   size_t original_start, size_t *ms, size_t *me) {
  size_t start = original_start, end = start;
  while (end <= len) {
    start = end;
    long i = find_sub(text + end, len - end, r->lcs, r->lcs_len);
    if (i < 0) return R_NOMATCH;
    end += (size_t)i + r->lcs_len;
    size_t pos, consumed;
    int k = orc_dfa_reverse(r->rev, c->rev, 0, text + start, end - start, end - start, &pos, &consumed);
    c->st.rev_bytes += consumed;
    if ((k == R_MATCH || k == R_NOMATCH) && pos == 0) return -1;
    if (k == R_MATCH) { *ms = pos + start; *me = end; return R_MATCH; }
    if (k == R_NOMATCH) continue;
    return R_QUIT;
  }
  return R_NOMATCH;
}

/* exec.rs:764-794 find_dfa_reverse_suffix */
static int find_dfa_reverse_suffix(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                                   size_t *ms, size_t *me) {
  size_t s0, e0;
  int k = exec_dfa_reverse_suffix(r, c, text, len, start, &s0, &e0);
  if (k < 0) return find_dfa_forward(r, c, text, len, start, ms, me);
  if (k != R_MATCH) return k;
  /* the suffix occurrence is the earliest possible end: run the forward DFA
   * from the match start for the leftmost-first end */
  size_t end, stop;
  int k2 = orc_dfa_forward_pfx(r->fwd, c->fwd, 0, dfa_prefixes(r), text, len, s0, &end, &stop);
  c->st.fwd_bytes += stop - s0;
  if (k2 == R_QUIT) return R_QUIT;
  if (k2 != R_MATCH) return R_NOMATCH;  /* the reference panics here ("BUG: reverse match implies ...") */
  *ms = s0;
  *me = end;
  return R_MATCH;
}

/* exec.rs:700-710 shortest_dfa_reverse_suffix (end of the shortest match) */
static int shortest_dfa_reverse_suffix(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len,
                                       size_t start, size_t *end) {
  size_t s0, e0, stop;
  int k = exec_dfa_reverse_suffix(r, c, text, len, start, &s0, &e0);
  if (k < 0) {
    k = orc_dfa_forward_pfx(r->fwd, c->fwd, 1, dfa_prefixes(r), text, len, start, end, &stop);
    c->st.fwd_bytes += stop - start;
    return k;
  }
  if (k == R_MATCH) *end = e0;
  return k;
}

static int is_literal(const orc_regex *r) { return r->mt >= 0 && r->mt <= 2; }
static int use_anchored_rev(const orc_regex *r) { return r->mt < 0 ? anchored_rev(r) : r->mt == 4; }

int orc_find_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start, size_t *ms,
                size_t *me) {
  if (start > len) return 0;
  if (is_literal(r)) return find_literals(r, text, len, start, ms, me);
  if (r->mt == 6) return orc_find_nfa(r, c, text, len, start, ms, me);
  int k = r->mt == 5 ? find_dfa_reverse_suffix(r, c, text, len, start, ms, me)
          : use_anchored_rev(r) ? find_dfa_anchored_reverse(r, c, 0, text, len, start, ms, me)
                                : find_dfa_forward(r, c, text, len, start, ms, me);
  if (k == R_MATCH) return 1;
  if (k == R_NOMATCH) return 0;
  c->st.quits++;
  return orc_find_nfa(r, c, text, len, start, ms, me);
}

/* utf8.rs:24-39 */
static size_t next_utf8(const uint8_t *text, size_t len, size_t i) {
  if (i >= len) return i + 1;
  uint8_t b = text[i];
  return i + (b <= 0x7F ? 1 : b <= 0xDF ? 2 : b <= 0xEF ? 3 : 4);
}

/* exec.rs:524-596 read_captures_at, MatchType::Dfa arm (the literal and
 * reverse match types produce the same bounds and also continue with
 * captures_nfa_with_match, exec.rs:861-875). */
int orc_captures_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start, size_t *slots,
                    size_t nslots) {
  for (size_t i = 0; i < nslots; ++i) slots[i] = SIZE_MAX;
  if (start > len) return 0;
  if (nslots <= 2) {
    size_t ms, me;
    if (!orc_find_at(r, c, text, len, start, &ms, &me)) return 0;
    if (nslots == 2) { slots[0] = ms; slots[1] = me; }
    return 1;
  }
  size_t ms, me;
  int k;
  if (is_literal(r)) {
    k = find_literals(r, text, len, start, &ms, &me) ? R_MATCH : R_NOMATCH;
  } else if (r->mt == 6 || ((r->mt < 0 || r->mt == 3) && r->nfa->anchored_start)) {
    return orc_captures_nfa(r, c, text, len, start, slots, nslots) && slots[0] != SIZE_MAX &&
           slots[1] != SIZE_MAX;
  } else {
    k = r->mt == 5 ? find_dfa_reverse_suffix(r, c, text, len, start, &ms, &me)
        : use_anchored_rev(r) ? find_dfa_anchored_reverse(r, c, 0, text, len, start, &ms, &me)
                              : find_dfa_forward(r, c, text, len, start, &ms, &me);
  }
  if (k == R_NOMATCH) return 0;
  size_t n = len;
  if (k == R_MATCH) {
    size_t e = next_utf8(text, len, next_utf8(text, len, me));
    n = e < len ? e : len;
    start = ms;
  } else {
    c->st.quits++;
  }
  if (!orc_captures_nfa(r, c, text, n, start, slots, nslots)) return 0;
  return slots[0] != SIZE_MAX && slots[1] != SIZE_MAX;
}

/* exec.rs:825-837 shortest_nfa: quit_after_match Pike VM, slots[1] */
int orc_shortest_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start, size_t *end) {
  uint8_t m[1] = {0};
  size_t slots[2] = {SIZE_MAX, SIZE_MAX};
  if (start > len) return 0;
  if (!orc_pike_exec(r->nfa, c->pike, m, 1, slots, 2, 1, text, len, start)) return 0;
  if (slots[1] == SIZE_MAX) return 0;
  *end = slots[1];
  return 1;
}

int orc_shortest_match_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                          size_t *end) {
  if (start > len) return 0;
  size_t e, stop;
  int k;
  if (is_literal(r)) {
    size_t s;
    if (!find_literals(r, text, len, start, &s, &e)) return 0;
    *end = e;
    return 1;
  }
  if (r->mt == 6) return orc_shortest_nfa(r, c, text, len, start, end);
  if (r->mt == 5) {
    k = shortest_dfa_reverse_suffix(r, c, text, len, start, &e);
  } else if (use_anchored_rev(r)) {
    size_t s;
    k = find_dfa_anchored_reverse(r, c, 1, text, len, start, &s, &e);
  } else {
    k = orc_dfa_forward_pfx(r->fwd, c->fwd, 1, dfa_prefixes(r), text, len, start, &e, &stop);
    c->st.fwd_bytes += stop - start;
  }
  if (k == R_MATCH) { *end = e; return 1; }
  if (k == R_NOMATCH) return 0;
  c->st.quits++;
  return orc_shortest_nfa(r, c, text, len, start, end);
}

int orc_is_match_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start) {
  if (start > len) return 0;
  size_t e, stop;
  int k;
  if (is_literal(r)) {
    size_t s;
    return find_literals(r, text, len, start, &s, &e);
  }
  if (r->mt == 6) {
    uint8_t m[1] = {0};
    return orc_pike_exec(r->nfa, c->pike, m, 1, NULL, 0, 1, text, len, start);
  }
  if (r->mt == 5) {
    k = shortest_dfa_reverse_suffix(r, c, text, len, start, &e);
  } else if (use_anchored_rev(r)) {
    size_t s;
    k = find_dfa_anchored_reverse(r, c, 1, text, len, start, &s, &e);
  } else {
    k = orc_dfa_forward_pfx(r->fwd, c->fwd, 1, dfa_prefixes(r), text, len, start, &e, &stop);
    c->st.fwd_bytes += stop - start;
  }
  if (k == R_MATCH) return 1;
  if (k == R_NOMATCH) return 0;
  c->st.quits++;
  uint8_t m[1] = {0};
  return orc_pike_exec(r->nfa, c->pike, m, 1, NULL, 0, 1, text, len, start);
}

int orc_many_matches_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                         uint8_t *matches) {
  return orc_pike_exec(r->nfa, c->pike, matches, r->nfa->nmatches, NULL, 0, 0, text, len, start);
}

int orc_many_matches_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                        uint8_t *matches) {
  if (start > len) return 0;
  size_t pos, stop;
  int k = orc_dfa_forward_many(r->fwd, c->fwd, matches, text, len, start, &pos, &stop);
  c->st.fwd_bytes += stop - start;
  if (k == R_MATCH) return 1;
  if (k == R_NOMATCH) return 0;
  c->st.quits++;
  return orc_many_matches_nfa(r, c, text, len, start, matches);
}

int64_t orc_find_iter_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                         size_t *pairs, size_t cap) {  /* re_trait.rs:197-221, the first search at `start` */
  size_t last_end = start;
  int has_last = 0;
  size_t last_match = 0;
  int64_t count = 0;
  for (;;) {
    if (last_end > len) break;
    size_t s, e;
    if (!orc_find_at(r, c, text, len, last_end, &s, &e)) break;
    if (s == e) {
      last_end = e + 1;  /* next_after_empty for bytes (exec.rs:375-377) */
      if (has_last && last_match == e) continue;
    } else {
      last_end = e;
    }
    has_last = 1;
    last_match = e;
    if ((size_t)count < cap) { pairs[2 * count] = s; pairs[2 * count + 1] = e; }
    count++;
  }
  return count;
}

int64_t orc_find_iter(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t *pairs,
                      size_t cap) {
  return orc_find_iter_at(r, c, text, len, 0, pairs, cap);
}

/* ---------------------------------------------------------- batch baseline */
typedef struct {
  const orc_regex *r;
  const uint8_t *buf;
  const uint64_t *offs;
  size_t stride, length, lo, hi;
  int mode;  /* 0 find, 1 is_match, 2 set, 3 shortest_match */
  uint64_t *out;
  uint8_t *out8;
  orc_stats st;
} Job;

static void *worker(void *arg) {
  Job *j = (Job *)arg;
  orc_cache *c = orc_cache_new(j->r);
  uint8_t matches[64];
  for (size_t i = j->lo; i < j->hi; ++i) {
    const uint8_t *t;
    size_t len;
    if (j->offs) { t = j->buf + j->offs[i]; len = (size_t)(j->offs[i + 1] - j->offs[i]); }
    else { t = j->buf + i * j->stride; len = j->length; }
    if (j->mode == 0) {
      size_t s, e;
      if (orc_find_at(j->r, c, t, len, 0, &s, &e)) { j->out[2 * i] = s; j->out[2 * i + 1] = e; }
      else { j->out[2 * i] = UINT64_MAX; j->out[2 * i + 1] = UINT64_MAX; }
    } else if (j->mode == 1) {
      j->out8[i] = (uint8_t)orc_is_match_at(j->r, c, t, len, 0);
    } else if (j->mode == 3) {  /* shortest_match: the end, UINT64_MAX for none */
      size_t e;
      j->out[i] = orc_shortest_match_at(j->r, c, t, len, 0, &e) ? (uint64_t)e : UINT64_MAX;
    } else {
      uint32_t nm = j->r->fwd->nmatches;
      memset(matches, 0, sizeof(matches));
      orc_many_matches_at(j->r, c, t, len, 0, matches);
      uint64_t m = 0;
      for (uint32_t k = 0; k < nm && k < 64; ++k) if (matches[k]) m |= 1ull << k;
      j->out[i] = m;
    }
  }
  orc_cache_stats(c, &j->st);  /* counters, plus this thread's cache flushes and final state count */
  orc_cache_free(c);
  return NULL;
}

static int run_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                     size_t n, int nthreads, int mode, uint64_t *out, uint8_t *out8, orc_stats *stats) {
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n && n > 0) nthreads = (int)n;
  Job *jobs = (Job *)calloc((size_t)nthreads, sizeof(Job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  size_t per = (n + nthreads - 1) / (nthreads ? nthreads : 1);
  for (int k = 0; k < nthreads; ++k) {
    Job *j = &jobs[k];
    j->r = r; j->buf = buf; j->offs = offs; j->stride = stride; j->length = length;
    j->lo = (size_t)k * per; j->hi = j->lo + per; if (j->hi > n) j->hi = n; if (j->lo > n) j->lo = n;
    j->mode = mode; j->out = out; j->out8 = out8;
    if (nthreads == 1) worker(j); else pthread_create(&th[k], NULL, worker, j);
  }
  if (stats) memset(stats, 0, sizeof(*stats));
  for (int k = 0; k < nthreads; ++k) {
    if (nthreads > 1) pthread_join(th[k], NULL);
    if (stats) {
      stats->fwd_bytes += jobs[k].st.fwd_bytes;
      stats->rev_bytes += jobs[k].st.rev_bytes;
      stats->quits += jobs[k].st.quits;
      stats->flushes += jobs[k].st.flushes;
      stats->states += jobs[k].st.states;
    }
  }
  free(jobs);
  free(th);
  return 0;
}

int orc_find_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                   size_t n, int nthreads, uint64_t *out_pairs, orc_stats *stats) {
  return run_batch(r, buf, offs, stride, length, n, nthreads, 0, out_pairs, NULL, stats);
}
int orc_is_match_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                       size_t n, int nthreads, uint8_t *out) {
  return run_batch(r, buf, offs, stride, length, n, nthreads, 1, NULL, out, NULL);
}
int orc_shortest_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                       size_t n, int nthreads, uint64_t *out) {
  return run_batch(r, buf, offs, stride, length, n, nthreads, 3, out, NULL, NULL);
}
int orc_set_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                  size_t n, int nthreads, uint64_t *masks) {
  return run_batch(r, buf, offs, stride, length, n, nthreads, 2, masks, NULL, NULL);
}
int orc_set_batch_stats(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                        size_t n, int nthreads, uint64_t *masks, orc_stats *stats) {
  return run_batch(r, buf, offs, stride, length, n, nthreads, 2, masks, NULL, stats);
}
