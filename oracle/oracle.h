/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle for the batched byte-regex scan path.
 *
 * A plain-C restatement of the reference engines (Nemo157/regex = rust-lang
 * regex 0.2.5) that run over a compiled byte Program:
 *   lazy DFA            src/dfa.rs        (forward/reverse/forward_many, cache + flush + quit)
 *   Pike VM             src/pikevm.rs     (+ src/input.rs ByteInput empty-width assertions)
 *   dispatch            src/exec.rs       (find_dfa_forward, shortest_dfa, many_matches_at,
 *                                          NFA fallback on DFA Quit)
 *   iteration           src/re_trait.rs:197-221
 * The engine choice (exec.rs:1130-1210) is restated where it is observable:
 * MatchType::Literal searches the literal sets (exec.rs:601-625) and
 * DfaSuffix scans for the suffix literal first (exec.rs:725-794).
 *
 * The Program (src/prog.rs contract) is supplied by the caller as flat
 * 12-byte instruction records (the product's host compiler exports them via
 * rure_amd_program_export).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * or the timed CPU baseline — never as a product path.
 *
 * Parity pinning: tests/test_oracle_golden.py checks this oracle against the
 * reference's own golden vectors (the mat!/matiter!/matset! vectors of its tests, Fowler
 * .dat files, sherlock / regexdna known answers) extracted into tests/golden/.
 */
#ifndef RURE_ORACLE_H
#define RURE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

typedef struct orc_inst {
  uint8_t op, look, lo, hi; /* op: 0 Match(x=slot) 1 Save(x=goto,y=slot) 2 Split(x,y) 3 EmptyLook(x=goto) 4 Bytes(x=goto) */
  uint32_t x, y;
} orc_inst;

typedef struct orc_prog orc_prog;
typedef struct orc_regex orc_regex;
typedef struct orc_cache orc_cache;

orc_prog *orc_prog_new(const orc_inst *insts, uint32_t n, uint32_t start, const uint8_t *byte_classes,
                       int is_reverse, int anchored_start, int anchored_end, int has_uwb, uint32_t ncaps,
                       size_t dfa_size_limit);
void orc_prog_free(orc_prog *p);

/* rev may be NULL for sets.  Takes ownership of the programs. */
orc_regex *orc_regex_new(orc_prog *nfa, orc_prog *fwd, orc_prog *rev);
void orc_regex_free(orc_regex *r);

/* The reference's engine choice for a single regex (src/exec.rs:1130-1210;
 * the product computes it, rure_amd_match_info_get) and the literal sets it
 * rests on, serialized as records {u8 cut, u32 len, bytes}: the unambiguous
 * prefixes (nfa.prefixes) and suffixes with their searchers' matcher kinds
 * (0 Empty, 1 Bytes, 2 one literal, 3 several), and suffixes.lcs().
 * match_type: 0 Literal(Unanchored), 1 Literal(AnchoredStart),
 * 2 Literal(AnchoredEnd), 3 Dfa, 4 DfaAnchoredReverse, 5 DfaSuffix, 6 Nfa.
 * Without this call the oracle dispatches as for Dfa / DfaAnchoredReverse. */
void orc_regex_set_exec(orc_regex *r, int match_type, const uint8_t *pre, size_t pre_len, int pre_matcher,
                        const uint8_t *suf, size_t suf_len, int suf_matcher, const uint8_t *lcs, size_t lcs_len);

orc_cache *orc_cache_new(const orc_regex *r);
void orc_cache_free(orc_cache *c);

/* exec.rs:473-514 find_at.  Returns 1 on match. */
int orc_find_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                size_t *ms, size_t *me);
/* exec.rs:382-420 shortest_match_at. */
int orc_shortest_match_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                          size_t *end);
/* exec.rs:427-468 is_match_at. */
int orc_is_match_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start);
/* Forced Pike VM (the reference's `nfa` test targets). */
int orc_find_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                 size_t *ms, size_t *me);
int orc_shortest_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                     size_t *end);
/* Pike VM captures: slots[2*ncaps] (SIZE_MAX = unset). */
int orc_captures_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                     size_t *slots, size_t nslots);
/* exec.rs:524-596 read_captures_at (DFA bounds, then the Pike VM on
 * text[..min(next_utf8(next_utf8(end)), len)] from the match start). */
int orc_captures_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                    size_t *slots, size_t nslots);
/* re_trait.rs:197-221 find_iter.  Writes up to cap (s,e) pairs; returns the total count. */
int64_t orc_find_iter(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t *pairs,
                      size_t cap);
int64_t orc_find_iter_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                         size_t *pairs, size_t cap);
/* exec.rs:998-1038 many_matches_at; matches[nmatches]. */
int orc_many_matches_at(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                        uint8_t *matches);
int orc_many_matches_nfa(const orc_regex *r, orc_cache *c, const uint8_t *text, size_t len, size_t start,
                         uint8_t *matches);

/* Statistics of the last forward-DFA scan on this cache. */
typedef struct orc_stats {
  uint64_t fwd_bytes;      /* bytes consumed by forward DFA scans (incl. the byte that killed it) */
  uint64_t rev_bytes;      /* bytes consumed by reverse DFA scans */
  uint64_t quits;          /* DFA gave up (NFA fallback used) */
  uint64_t flushes;        /* cache flushes */
  uint64_t states;         /* states currently cached (fwd) */
} orc_stats;
void orc_cache_stats(const orc_cache *c, orc_stats *out);
void orc_cache_reset_stats(orc_cache *c);

/* Multi-threaded batch baselines (one private cache per thread, static
 * contiguous split), haystack i = [offs[i], offs[i+1]) or fixed stride. */
int orc_find_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                   size_t n, int nthreads, uint64_t *out_pairs, orc_stats *stats);
/* orc_set_batch with the engine statistics summed over the threads: DFA
 * quits (lines answered by the Pike VM after the cache thrashed, dfa.rs:
 * 1282-1293), cache flushes, and the threads' final cached-state counts. */
int orc_set_batch_stats(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                        size_t n, int nthreads, uint64_t *masks, orc_stats *stats);
int orc_is_match_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride,
                       size_t length, size_t n, int nthreads, uint8_t *out);
/* shortest_match (exec.rs:382-420) per haystack: the end, UINT64_MAX for none. */
int orc_shortest_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                       size_t n, int nthreads, uint64_t *out);
int orc_set_batch(const orc_regex *r, const uint8_t *buf, const uint64_t *offs, size_t stride, size_t length,
                  size_t n, int nthreads, uint64_t *masks);

#endif
