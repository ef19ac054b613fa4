/* TEST INFRASTRUCTURE ONLY: internal structures of the CPU oracle. */
#ifndef RURE_ORACLE_INT_H
#define RURE_ORACLE_INT_H
#include <stddef.h>
#include <stdint.h>

#include "oracle.h"

enum { OP_MATCH = 0, OP_SAVE = 1, OP_SPLIT = 2, OP_EMPTY = 3, OP_BYTES = 4 };
/* prog.rs:334-351 */
enum {
  LOOK_START_LINE = 0, LOOK_END_LINE = 1, LOOK_START_TEXT = 2, LOOK_END_TEXT = 3,
  LOOK_WB = 4, LOOK_NWB = 5, LOOK_WB_ASCII = 6, LOOK_NWB_ASCII = 7
};

struct orc_prog {
  orc_inst *insts;
  uint32_t n;
  uint32_t start;
  uint8_t byte_classes[256];
  int is_reverse, anchored_start, anchored_end, has_uwb;
  uint32_t nmatches;
  uint32_t ncaps;
  size_t dfa_size_limit;
};

typedef struct { uint32_t *dense, *sparse; size_t n, cap; } orc_sset;
void orc_sset_init(orc_sset *s, size_t cap);
void orc_sset_free(orc_sset *s);
int orc_sset_contains(const orc_sset *s, uint32_t v);
void orc_sset_insert(orc_sset *s, uint32_t v);

typedef struct { uint8_t *data; uint32_t len; } orc_state;

typedef struct orc_dfa_cache {
  uint32_t nclasses;
  uint32_t *trans;
  size_t trans_len, trans_cap;
  orc_state *states;
  size_t nstates, states_cap;
  uint32_t *map;
  size_t map_cap, map_n;
  uint32_t start_states[256];
  uint32_t *stack;
  size_t stack_len, stack_cap;
  uint64_t flush_count;
  uint64_t stat_flushes;
  size_t size;
  orc_sset qcur, qnext;
} orc_dfa_cache;

orc_dfa_cache *orc_dfa_cache_new(const orc_prog *p);
void orc_dfa_cache_free(orc_dfa_cache *c);
size_t orc_dfa_cache_nstates(const orc_dfa_cache *c);
int orc_dfa_forward(const orc_prog *p, orc_dfa_cache *c, int quit_after_match, const uint8_t *text, size_t len,
                    size_t at, size_t *pos, size_t *stop);
int orc_dfa_reverse(const orc_prog *p, orc_dfa_cache *c, int quit_after_match, const uint8_t *text, size_t len,
                    size_t at, size_t *pos, size_t *consumed);
int orc_dfa_forward_many(const orc_prog *p, orc_dfa_cache *c, uint8_t *matches, const uint8_t *text, size_t len,
                         size_t at, size_t *pos, size_t *stop);

typedef struct orc_pike_cache orc_pike_cache;
orc_pike_cache *orc_pike_cache_new(const orc_prog *p);
void orc_pike_cache_free(orc_pike_cache *c);
int orc_pike_exec(const orc_prog *p, orc_pike_cache *c, uint8_t *matches, size_t nmatches, size_t *slots,
                  size_t nslots, int quit_after_match, const uint8_t *text, size_t len, size_t start);

/* A literal set (src/literals.rs LiteralSearcher): literals in order. */
typedef struct {
  int matcher;          /* 0 Empty, 1 Bytes, 2 one literal, 3 several (Teddy / AC) */
  size_t n;
  uint8_t **lit;
  size_t *len;
  /* lits_find's prefilter (lits_parse): for literals of 1-3 bytes their
   * first bytes, the one-byte literals and a bitmap of first byte pairs; for
   * the longer ones a bitmap of a hash of their first four bytes; any_empty:
   * some literal is empty (it occurs at every position) */
  uint8_t first[256], single[256];
  uint8_t *pair, *quad;
  int any_empty, any_short, any_long;
} orc_lits;

/* LiteralSearcher::find (src/literals.rs:92-103) over hay[0..n) (exec.c). */
int orc_lits_find(const orc_lits *l, const uint8_t *hay, size_t n, size_t *s, size_t *e);
/* Fsm::forward with the program's prefix literals (dfa.prefixes, exec.rs:
 * 308-311): in a start state the scan jumps to the next prefix occurrence
 * (dfa.rs:700-711 prefix_at, has_prefix dfa.rs:1562-1566).  pre NULL: none
 * (orc_dfa_forward). */
int orc_dfa_forward_pfx(const orc_prog *p, orc_dfa_cache *c, int quit_after_match, const orc_lits *pre,
                        const uint8_t *text, size_t len, size_t at, size_t *pos, size_t *stop);

struct orc_regex {
  orc_prog *nfa, *fwd, *rev;
  int mt;               /* MatchType code (orc_regex_set_exec), -1: not set (Dfa dispatch) */
  orc_lits pre, suf;    /* nfa.prefixes, suffixes (exec.rs:308-321) */
  uint8_t *lcs;         /* suffixes.lcs() (DfaSuffix) */
  size_t lcs_len;
};

struct orc_cache {
  orc_dfa_cache *fwd, *rev;
  orc_pike_cache *pike;
  orc_stats st;
};

#endif
