/*
 * rure_amd.h — MI355X drop-in for the batched byte-regex scan path of the
 * reference `rure` C API (regex 0.2.5, regex-capi/include/rure.h).
 *
 * Part 1 re-declares the `rure` entry points a C caller of the reference
 * binds, with the same names, argument meaning, flag values and ownership
 * rules; each cites the reference declaration it replaces.  Every search
 * entry point runs on the GPU (HIP kernels for gfx950); there is no CPU
 * matching path inside this library.
 *
 * Part 2 adds the batched device-pointer entry points the hot path needs
 * (one call scans many haystacks resident in HBM).  Plain pointers and sizes
 * only; `stream` is a `hipStream_t` passed as `void *` (NULL = the null
 * stream).
 */
#ifndef RURE_AMD_H
#define RURE_AMD_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- Part 1 */

typedef struct rure rure;                  /* rure.h:29 */
typedef struct rure_set rure_set;          /* rure.h:36 */
typedef struct rure_options rure_options;  /* rure.h:47 */
typedef struct rure_iter rure_iter;        /* rure.h:106 */
typedef struct rure_error rure_error;      /* rure.h:130 */
typedef struct rure_captures rure_captures;                      /* rure.h:95 */
typedef struct rure_iter_capture_names rure_iter_capture_names;  /* rure.h:117 */

/* rure.h:56-68 */
#define RURE_FLAG_CASEI (1 << 0)
#define RURE_FLAG_MULTI (1 << 1)
#define RURE_FLAG_DOTNL (1 << 2)
#define RURE_FLAG_SWAP_GREED (1 << 3)
#define RURE_FLAG_SPACE (1 << 4)
#define RURE_FLAG_UNICODE (1 << 5)
#define RURE_DEFAULT_FLAGS RURE_FLAG_UNICODE

/* rure.h:73-78 */
typedef struct rure_match {
  size_t start;
  size_t end;
} rure_match;

/* rure.h:147 — aborts (after printing the error) if the pattern is invalid. */
rure *rure_compile_must(const char *pattern);
/* rure.h:168-169 — NULL on error (error filled if non-NULL). */
rure *rure_compile(const uint8_t *pattern, size_t length, uint32_t flags,
                   rure_options *options, rure_error *error);
/* rure.h:177 */
void rure_free(rure *re);
/* rure.h:197-198 */
bool rure_is_match(rure *re, const uint8_t *haystack, size_t length, size_t start);
/* rure.h:220-221 — `match` may be NULL. */
bool rure_find(rure *re, const uint8_t *haystack, size_t length, size_t start,
               rure_match *match);
/* rure.h:273-274 */
bool rure_shortest_match(rure *re, const uint8_t *haystack, size_t length,
                         size_t start, size_t *end);
/* rure.h:317-345 — iterator over successive non-overlapping matches. */
rure_iter *rure_iter_new(rure *re);
void rure_iter_free(rure_iter *it);
bool rure_iter_next(rure_iter *it, const uint8_t *haystack, size_t length,
                    rure_match *match);
/* rure.h:248-249 — leftmost-first match with every capture group's location
 * (exec.rs:524-596 dispatch: DFA bounds, then the Pike VM for the groups). */
bool rure_find_captures(rure *re, const uint8_t *haystack, size_t length,
                        size_t start, rure_captures *captures);
/* rure.h:285 — index of the named group, -1 if none. */
int32_t rure_capture_name_index(rure *re, const char *name);
/* rure.h:292-307 — group names in index order ("" for unnamed groups). */
rure_iter_capture_names *rure_iter_capture_names_new(rure *re);
void rure_iter_capture_names_free(rure_iter_capture_names *it);
bool rure_iter_capture_names_next(rure_iter_capture_names *it, char **name);
/* rure.h:369-371 */
bool rure_iter_next_captures(rure_iter *it, const uint8_t *haystack, size_t length,
                             rure_captures *captures);
/* rure.h:385-411 */
rure_captures *rure_captures_new(rure *re);
void rure_captures_free(rure_captures *captures);
bool rure_captures_at(rure_captures *captures, size_t i, rure_match *match);
size_t rure_captures_len(rure_captures *captures);
/* rure.h:423-454 */
rure_options *rure_options_new(void);
void rure_options_free(rure_options *options);
void rure_options_size_limit(rure_options *options, size_t limit);
void rure_options_dfa_size_limit(rure_options *options, size_t limit);
/* rure.h:476-538 */
rure_set *rure_compile_set(const uint8_t **patterns, const size_t *patterns_lengths,
                           size_t patterns_count, uint32_t flags,
                           rure_options *options, rure_error *error);
void rure_set_free(rure_set *re);
bool rure_set_is_match(rure_set *re, const uint8_t *haystack, size_t length, size_t start);
bool rure_set_matches(rure_set *re, const uint8_t *haystack, size_t length, size_t start,
                      bool *matches);
size_t rure_set_len(rure_set *re);
/* rure.h:551-568 */
rure_error *rure_error_new(void);
void rure_error_free(rure_error *err);
const char *rure_error_message(rure_error *err);

/* ---------------------------------------------------------------- Part 2 */

/* Status codes of the batched calls. */
#define RURE_AMD_OK 0
#define RURE_AMD_ERR_ARG (-1)        /* bad argument */
#define RURE_AMD_ERR_HIP (-2)        /* HIP runtime error (no device, launch failure) */
#define RURE_AMD_ERR_DFA (-3)        /* automaton could not be materialized */

/* A batch of haystacks resident in device memory.  Haystack i is
 *   bytes [offsets[i], offsets[i+1])            when offsets != NULL, else
 *   bytes [i*stride, i*stride + length)         (fixed stride).
 * The search in every haystack starts at `start` (with look-behind context,
 * like rure_find's `start`, rure.h:186-192).  Offsets in results are relative
 * to the haystack's first byte.
 * The kernels load whole aligned 16-byte blocks: the buffer must be readable
 * up to the 16-byte-rounded end of its last haystack (device allocations of
 * the HIP runtime and torch are); bytes outside a haystack never influence
 * its results. */
typedef struct rure_amd_batch {
  const uint8_t *haystack;
  const uint64_t *offsets;
  size_t stride;
  size_t length;
  size_t count;
  size_t start;
} rure_amd_batch;

/* Batched rure_find: out[i] = leftmost-first match, or {SIZE_MAX, SIZE_MAX}. */
int rure_amd_find_batch(rure *re, const rure_amd_batch *batch, rure_match *out, void *stream);
/* Batched rure_is_match: out[i] in {0, 1}. */
int rure_amd_is_match_batch(rure *re, const rure_amd_batch *batch, uint8_t *out, void *stream);
/* Batched rure_shortest_match: end[i] or SIZE_MAX. */
int rure_amd_shortest_match_batch(rure *re, const rure_amd_batch *batch, size_t *end, void *stream);
/* Batched rure_set_matches (rure.h:532-533): bit j of mask[i] set iff
 * pattern j matches; sets of at most 64 patterns (RURE_AMD_ERR_ARG above). */
int rure_amd_set_matches_batch(rure_set *re, const rure_amd_batch *batch, uint64_t *mask,
                               void *stream);
/* The same for any number of patterns: `words` >= ceil(rure_set_len / 64)
 * u64 per haystack; bit (j % 64) of mask[i * words + j / 64] set iff pattern j
 * matches haystack i (unused bits and words are zero). */
int rure_amd_set_matches_batch_words(rure_set *re, const rure_amd_batch *batch, uint64_t *mask,
                                     size_t words, void *stream);

/* Batched find_iter (bytes::Regex::find_iter, re_trait.rs:197-221): every
 * successive non-overlapping leftmost-first match of every haystack.
 * counts[i] (device) = number of matches in haystack i; `matches` (device)
 * receives them concatenated in haystack order, at most `capacity` records;
 * *total (device) = the number of matches (rerun with a larger buffer if it
 * exceeds `capacity`).  Long fixed-stride haystacks are scanned in parallel
 * chunks with exact boundary repair. */
int rure_amd_find_iter_batch(rure *re, const rure_amd_batch *batch, uint64_t *counts, rure_match *matches,
                             size_t capacity, uint64_t *total, void *stream);

/* find_iter over one span [lo, hi) of a long haystack (sharded or streamed
 * iteration): the iteration of re_trait.rs:197-221 restricted to
 * the matches that START in [lo, hi) (a match may end past hi; the haystack
 * bytes after hi and before lo are read as context).  entry (device, may be
 * NULL) = the state the previous span's call left in its `exit`; NULL or
 * entry->fresh != 0 starts afresh at lo (no previous match).  *count
 * (device) = matches owned, the first `capacity` written to `matches`
 * (device).  *exit (device) = the state at hi: fresh != 0 when it is
 * equivalent to a fresh start at hi (the next span's speculative result
 * stands), else the next span must be recomputed with it as entry.  A span
 * with hi == length also owns an empty match at the very end.  Concatenating
 * the spans' matches in order equals rure_amd_find_iter_batch over the whole
 * haystack from lo of the first span. */
typedef struct rure_amd_iter_state {
  uint64_t next;        /* where the next search starts */
  uint64_t last_match;  /* end of the previous match, SIZE_MAX if none */
  uint64_t fresh;       /* 1: same as a fresh iteration from the span end */
} rure_amd_iter_state;
int rure_amd_find_iter_span(rure *re, const uint8_t *haystack, size_t length, size_t lo, size_t hi,
                            const rure_amd_iter_state *entry, uint64_t *count, rure_match *matches,
                            size_t capacity, rure_amd_iter_state *exit, void *stream);
/* rure_amd_find_iter_span for n regexes over the same span [lo, hi) of one
 * haystack: regex i's results go to count[i], matches[i] (capacity[i]
 * records) and exit[i], entered with entry[i] (NULL entry array or element:
 * a fresh start) — host arrays of device pointers; each regex's output is
 * exactly its own rure_amd_find_iter_span's.  Regexes that are finite sets of
 * strings of one common length (the regex-dna variants) are scanned together
 * in one pass over the text; otherwise each runs its own pass. */
int rure_amd_find_iter_span_multi(rure *const *res, size_t n, const uint8_t *haystack, size_t length, size_t lo,
                                  size_t hi, const rure_amd_iter_state *const *entry, uint64_t *const *count,
                                  rure_match *const *matches, const size_t *capacity,
                                  rure_amd_iter_state *const *exit, void *stream);

/* Batched replacen with a literal replacement (bytes::Regex::replacen's
 * no-expansion path, re_bytes.rs:489-512): in every haystack the first
 * `limit` matches (0 = all) of the batched find_iter are replaced by
 * rep[0..rep_len) (host memory; `$` is not expanded, as with NoExpand).
 * out_offsets (device, n + 1) = the output layout (exclusive sums of the
 * output lengths); out (device) receives the concatenated outputs, at most
 * out_capacity bytes; *total (device) = the bytes needed (call again with a
 * larger buffer if it exceeds out_capacity).  Synchronises the stream once
 * to size the match buffer (twice if the first guess was short), except for
 * replace_all (limit 0) of a regex whose matches are single bytes of one
 * class over one fixed-stride haystack, which only enqueues. */
int rure_amd_replace_batch(rure *re, const rure_amd_batch *batch, const uint8_t *rep, size_t rep_len,
                           size_t limit, uint8_t *out, uint64_t *out_offsets, size_t out_capacity,
                           uint64_t *total, void *stream);
/* A chain of replace_all calls over one haystack, step i on step i - 1's
 * output: the regex-dna shootout's IUB substitutions
 * (examples/shootout-regex-dna-bytes.rs:44-60, each a bytes::Regex::
 * replace_all with NoExpand, re_bytes.rs:489-512).  Step i replaces every
 * match of res[i] by reps[i][0..rep_lens[i]) (host memory, no `$`
 * expansion).  Every res[i] must be a regex whose matches are single bytes of
 * one class (a literal byte, a byte class: rure_amd_class_one_export) and
 * 1 <= rep_lens[i] <= 64, else RURE_AMD_ERR_ARG.  haystack (device, 16-byte
 * aligned) holds `length` bytes; step i writes out0 if i is even, else out1
 * (device, 16-byte aligned, `capacity` bytes each; readable 16 bytes past
 * capacity); the result is in out0 if n is odd, else out1.  lengths (device,
 * n + 1 uint64) = length, then each step's output length.  An output longer
 * than capacity is cut; that step's length is exact, the steps after it read
 * their input cut and their lengths are lower bounds (a step never shortens
 * its text, so lengths[n] > capacity): retry with capacity = lengths[n]
 * until lengths[n] <= capacity.  Only enqueues:
 * each step's match count per 4 KiB is counted by the previous step's kernel
 * as it writes the text, and nothing is read back. */
int rure_amd_replace_all_chain(rure *const *res, const uint8_t *const *reps, const size_t *rep_lens, size_t n,
                               const uint8_t *haystack, size_t length, uint8_t *out0, uint8_t *out1,
                               size_t capacity, uint64_t *lengths, void *stream);
/* Batched split / splitn (re_bytes.rs:699-749): the fields between matches
 * as (start, end) records relative to each haystack, concatenated;
 * counts[i] (device) = fields of haystack i; at most `limit` fields per
 * haystack with SplitN's rule (the last is the rest of the haystack);
 * limit = SIZE_MAX for split.  *total (device) = number of fields.
 * Synchronises the stream once (twice if the first guess of the match
 * buffer was short) to size the match buffer. */
int rure_amd_split_batch(rure *re, const rure_amd_batch *batch, size_t limit, uint64_t *counts,
                         rure_match *pieces, size_t capacity, uint64_t *total, void *stream);

/* Match records of a batched find for the multi-GPU gather (the
 * path's only exchange): records[3*j .. 3*j+2] (device) = (base + i, start,
 * end) of the j-th haystack i, in haystack order, whose found[i] (device,
 * the output of rure_amd_find_batch over n haystacks) holds a match; at most
 * `capacity` records are written; *count (device) = the number of matches
 * (may exceed capacity).  No host synchronisation. */
int rure_amd_compact_matches(const rure_match *found, size_t n, uint64_t base, uint64_t *records,
                             size_t capacity, uint64_t *count, void *stream);

/* Batched rure_find_captures: slots[i * 2 * ngroups + 2 * g + {0, 1}]
 * (device, size_t) = start / end of group g in haystack i, SIZE_MAX where the
 * group did not participate or the haystack has no match.  ngroups =
 * rure_amd_captures_len(re). */
int rure_amd_captures_batch(rure *re, const rure_amd_batch *batch, size_t *slots, void *stream);
/* Number of capture groups including group 0 (= rure_captures_len). */
size_t rure_amd_captures_len(rure *re);

/* Returns the device scratch this library keeps cached for reuse (blocks
 * of the stream-ordered allocator freed by earlier batched calls; at most
 * max(256 MiB, 2 x the peak of live scratch) are kept) to the allocator.
 * Also done when the last rure / rure_set is freed.  Safe at any time: each
 * block is freed after the kernels that last used it. */
void rure_amd_release_scratch(void);
// Scratch bookkeeping: bytes cached for reuse, bytes held by calls in
// flight, and the number of rure / rure_set handles alive.
void rure_amd_scratch_stats(size_t *cached, size_t *live, long *handles);

/* Diagnostics (host only, no GPU needed). */
typedef struct rure_amd_dfa_info {
  int32_t ok;            /* 1 if the automaton was materialized */
  int32_t states;        /* minimised states incl. dead/quit */
  int32_t raw_states;    /* lazy-DFA states before minimisation */
  int32_t normal;        /* [0, normal) carry no match flag */
  int32_t match_end;     /* [normal, match_end) carry the match flag */
  int32_t dead;
  int32_t quit;          /* -1 if none */
  int32_t hot;           /* states held in the LDS fast table */
  int32_t byte_classes;
  int32_t insts;
  int32_t fast_stride;   /* bytes per dependent LDS lookup in the tile kernel (1, 2, 4) */
  int32_t fast_classes;  /* local byte classes of the multi-byte table (K) */
} rure_amd_dfa_info;
/* which: 0 = forward DFA, 1 = reverse DFA, 2 = find_iter forward DFA,
 * 3 / 4 = the forward / reverse automata past the u16 tables (u32 column
 * form, built when 0 / 1 exceed 65535 states; byte_classes = columns),
 * 5 = the find_iter forward DFA's ASCII shadow (bytes >= 0x80 quit; built
 * where 2 is too big for the all-rows LDS table, else RURE_AMD_ERR_DFA). */
int rure_amd_dfa_info_get(rure *re, int which, rure_amd_dfa_info *info);
int rure_amd_set_dfa_info_get(rure_set *re, rure_amd_dfa_info *info);

/* Export of the compiled byte programs (the reference's Program/Inst
 * contract, prog.rs:18-75, 261-425) as flat 12-byte records, for the CPU
 * oracle and tests.  which: 0 = forward DFA program (with `.*?`),
 * 1 = reverse DFA program, 2 = NFA program (with capture saves).
 * Returns the number of instructions; copies at most `cap` records. */
typedef struct rure_amd_inst {
  uint8_t op, look, lo, hi;
  uint32_t x, y;
} rure_amd_inst;
typedef struct rure_amd_prog_info {
  uint32_t ninsts, start, nmatches, ncaptures;
  uint8_t anchored_start, anchored_end, has_unicode_word_boundary, is_reverse;
  uint8_t byte_classes[256];
} rure_amd_prog_info;
int64_t rure_amd_program_export(rure *re, int which, rure_amd_prog_info *info,
                                rure_amd_inst *insts, size_t cap);
int64_t rure_amd_set_program_export(rure_set *re, int which, rure_amd_prog_info *info,
                                    rure_amd_inst *insts, size_t cap);
/* Export of a materialized DFA: trans = states*256 u32, eof_match = states
 * bytes, start = 128 u32.  which: 0 forward, 1 reverse, 2 the forward DFA
 * of the chunked find_iter (with stripped states, see _strip_export), 5 its
 * ASCII shadow. */
int rure_amd_dfa_export(rure *re, int which, uint32_t *trans, uint8_t *eof_match,
                        uint32_t *start);
/* Export of a set's DFA (rure_amd_set_dfa_info_get gives the sizes): trans =
 * states*256 u32, eof_mask / now_mask = states u64 (patterns matched at the
 * end of the text / reported on entering the state), start = 128 u32. */
int rure_amd_set_dfa_export(rure_set *re, uint32_t *trans, uint64_t *eof_mask, uint64_t *now_mask,
                            uint32_t *start);
/* Core form of a large set's DFA (used by the set kernel when the set DFA has
 * more than 255 ordinary or match-reporting states): sizes in info; lds =
 * 256-byte class map + (hot + 1) x K u16 entries (next core << 6 | output
 * code), gcore / gout = ncores x K next core (u16) / reported patterns (u64),
 * eof = ncores u64, start = 128 u16.  RURE_AMD_ERR_DFA if not in core form. */
typedef struct rure_amd_core_info {
  uint32_t K, ncores, hot, dead, quit, lds_bytes;
} rure_amd_core_info;
int rure_amd_set_core_export(rure_set *re, rure_amd_core_info *info, uint8_t *lds, uint16_t *gcore,
                             uint64_t *gout, uint64_t *eof, uint16_t *start);
/* strip[s] (states u32) of the find_iter forward DFA: s without the `.*?` prefix. */
int rure_amd_dfa_strip_export(rure *re, uint32_t *strip);
/* The first-byte start rule of the find_iter DFA (host only): returns |F|
 * (1..4, bytes[0..|F|) = F) when every match starts with a byte of F and an
 * anchored run from such a byte cannot die before matching — the chunked
 * find_iter then takes a match's start from the first F byte of its search
 * instead of a reverse scan — else 0; negative on error. */
int rure_amd_first_byte_export(rure *re, uint8_t *bytes);
/* The find_iter lexer table (host only; iter_spec_lex_tile_kernel): u8
 * entries e = 4 row + code; the next entry after byte b is table[76 e + b];
 * code (e & 3): 0 = an ordinary state, 1 = the start state (*s0 = its entry),
 * 2 = its twin, 3 = another restart twin (entering a twin = a match ended at
 * that byte).  Returns the table's size in bytes (0: no lexer table), copies
 * at most `cap`. */
int64_t rure_amd_lex_export(rure *re, uint8_t *table, size_t cap, uint32_t *s0);
/* The same lexer four bytes per step (host only): kLex4Bytes = 5120 bytes,
 * next row at [256 row + c] where c packs four byte classes (2 bits each,
 * byte j at bits 2j; class 3 = no byte), the four bytes' codes (2 bits each)
 * at [2048 + 256 row + c], byte -> class << 2j at [4096 + 256 j + b];
 * *s0 = the start row.  Returns the size (0: the lexer does not fit: more
 * than 8 rows or 3 ASCII byte classes, or no lexer table). */
int64_t rure_amd_lex4_export(rure *re, uint8_t *table, size_t cap, uint32_t *s0);
/* The lexer tables of the find_iter automaton's ASCII shadow (four = 0: the
 * byte table, 1: four bytes per step), as rure_amd_lex_export; 0 if the
 * shadow has none (its first-byte rule may have any number of first bytes:
 * \w+, \S+, \pL+). */
int64_t rure_amd_lex_ascii_export(rure *re, int four, uint8_t *table, size_t cap, uint32_t *s0);
/* 1 if the regex is one byte class repeated (C+, the find_iter run engine:
 * matches = the maximal runs of C bytes) on all bytes (ascii = 0) or on
 * ASCII text (ascii = 1, the ASCII shadow: bytes >= 0x80 quit), with cls[b]
 * bit 0 = b in C, bit 1 = b quits, bit 2 = b (>= 0x80) is read as UTF-8
 * (a Unicode class: rure_amd_run_cp_export); 0 if not. */
int rure_amd_run_class_export(rure *re, int ascii, uint8_t *cls);
/* The run engine's code point bitmap of a Unicode class C+ (\w+, \pL+,
 * \S+ in Unicode mode: bit c of bits[c / 32]), at most n words copied;
 * returns its size in words (0x110000 / 32) or 0 if the engine reads no
 * UTF-8 for this regex. */
int rure_amd_run_cp_export(rure *re, uint32_t *bits, size_t n);
/* 1 if every match of the regex is exactly one byte of a class (cls[b] = 1
 * for its bytes): its replace_all over one haystack then runs without a
 * match list (rure_amd_replace_batch, last_fwd_path -23); 0 if not. */
int rure_amd_class_one_export(rure *re, uint8_t *cls);

/* Export of the Pike VM closure tables the NFA kernel runs (host only):
 * leaves = 3 u32 per leaf (kind | lo << 8 | hi << 16, closure, slot),
 * cl_off = closures + 1 u32, entries = 2 u32 per entry (leaf,
 * cond | (1 + previous same-leaf entry) << 8).  Pass NULL arrays to query
 * the sizes.  Returns RURE_AMD_OK or an error. */
typedef struct rure_amd_nfa_info {
  uint32_t leaves, closures, entries, root, nmatch, anchored, looks, unicode_wb;
} rure_amd_nfa_info;
int rure_amd_nfa_export(rure *re, rure_amd_nfa_info *info, uint32_t *leaves, uint32_t *cl_off,
                        uint32_t *entries);
int rure_amd_set_nfa_export(rure_set *re, rure_amd_nfa_info *info, uint32_t *leaves, uint32_t *cl_off,
                            uint32_t *entries);
/* Capture slots each closure entry sets (the Saves on its path): save_off =
 * entries + 1 u32 CSR offsets into save_slot (u16).  *n_slots receives the
 * length of save_slot; NULL arrays query it. */
int rure_amd_nfa_saves_export(rure *re, uint32_t *save_off, uint16_t *save_slot, size_t *n_slots);
/* The regex as a finite string set, as the literal find_iter engine uses it
 * (the GPU counterpart of the reference's complete-prefix Literal engine,
 * exec.rs:1148-1166): returns the number of literals (0 = not a string set:
 * the DFA kernels iterate), in leftmost-first priority order; lens[i] and
 * bytes[32 * i ...] receive the first `cap` of them (NULL arrays: count only).
 * Host only. */
int64_t rure_amd_literals_export(rure *re, uint32_t *lens, uint8_t *bytes, size_t cap);
/* Diagnostics (host only): the Shift-And image of the find_iter string set
 * (iter_spec_sa_kernel) — 256 u64 byte masks, the first / last bit of every
 * class sequence and the string length.  Returns the state width in bits, 0
 * when the regex is not a set of equal-length strings that fits 64 bits. */
int64_t rure_amd_shiftand_export(rure *re, uint64_t *mask, uint64_t *init, uint64_t *fin, uint32_t *len);
/* Literal sets and the reference's engine choice (host only).
 * rure_amd_literals_syntax: regex-syntax's Expr::prefixes (which 0) /
 * suffixes (which 1) of a pattern (regex-syntax/src/literals.rs:285-304)
 * with the given limits (the reference's defaults: 250 bytes, 10 class
 * members), serialized as records {u8 cut, u32 length, bytes}; returns the
 * serialized size (copied only when cap suffices).  rure_amd_literals_op on
 * such records: 0 unambiguous_prefixes, 1 longest_common_prefix (raw bytes),
 * 2 longest_common_suffix (raw bytes), 3 unambiguous_suffixes.
 * rure_amd_exec_literals_export: the unambiguous prefix (which 0) / suffix
 * (which 1) set the reference's Exec builds for this regex (exec.rs:308-321).
 * rure_amd_match_info_get: its MatchType (exec.rs:1130-1210; codes:
 * 0 Literal(Unanchored), 1 Literal(AnchoredStart), 2 Literal(AnchoredEnd),
 * 3 Dfa, 4 DfaAnchoredReverse, 5 DfaSuffix, 6 Nfa, 7 Nothing), the two
 * LiteralSearchers' matcher kind (0 Empty, 1 Bytes, 2 one literal,
 * 3 several), len(), complete(), lcp / lcs character lengths and the lcs. */
typedef struct rure_amd_match_info {
  int32_t match_type;
  int32_t prefix_matcher, suffix_matcher;
  uint32_t prefix_len, suffix_len;
  uint8_t prefix_complete, suffix_complete, pad[2];
  uint32_t lcp_chars, lcs_chars;
  uint32_t lcs_bytes;
  uint8_t lcs[256];
} rure_amd_match_info;
int64_t rure_amd_literals_syntax(const uint8_t *pattern, size_t length, uint32_t flags, int which,
                                 size_t limit_size, size_t limit_class, uint8_t *out, size_t cap);
int64_t rure_amd_literals_op(int op, const uint8_t *in, size_t in_len, uint8_t *out, size_t cap);
int64_t rure_amd_exec_literals_export(rure *re, int which, uint8_t *out, size_t cap);
int rure_amd_match_info_get(rure *re, rure_amd_match_info *info);
/* 1 if batched searches of this regex run the DFA kernels, 0 if only the
 * Pike VM kernel (automaton too large), negative on error. */
int rure_amd_uses_dfa(rure *re);
int rure_amd_set_uses_dfa(rure_set *re);
/* Diagnostics (host only): the scan engine the last batched launch of this
 * process used — 0 = the per-lane streaming kernel, 1 / 2 / 4 = the
 * coalesced-tile kernel with that many bytes per dependent table lookup,
 * -2 = the reverse DFA from the end (DfaAnchoredReverse), -3 = the literal
 * engine (MatchType::Literal), -4 = the chunked cut-bounded scan (long
 * haystacks, small batches split into units), -5 = the lane search of the
 * Literal / DfaSuffix match types, -6 = the big (u32) DFA, (-7: unused
 * since round 5), -8 = the ragged line kernel, -9 = the
 * chunked DfaSuffix scan, -10 = the on-demand DFA, -11 = the DfaSuffix
 * find_iter, -12 / -13 = the chunked find_iter of a look-around regex (no
 * quit / a quit sent it to the wave path), -14 / -15 = the ASCII-shadow
 * find_iter (answered / quit), -16 = the Pike VM alone (no DFA), -17 = the
 * core-form set kernel over an offset batch, -19 / -20 = the find_iter run
 * engine of a C+ regex (its class over all bytes / the ASCII shadow's),
 * -21 = the chunked find_iter of the full automaton (no look-around), -22 =
 * find_iter with one haystack per wavefront, -23 = replace_all of a
 * one-byte-class regex without a match list; -1 before the first launch. */
int rure_amd_last_fwd_path(void);
/* Debug-only overrides of the engine dispatch and launch geometry
 * (regex_amd/csrc/host/knobs.hpp lists them): replaces the whole override
 * table, read once per process from RURE_AMD_DEBUG, by spec
 * ("name=value,..."; NULL or "" clears it).  For tests and A/B tools; no
 * production path needs an override.  Returns RURE_AMD_ERR_ARG (table
 * unchanged) on an unknown name or a malformed value.  Tables a regex has
 * already built for a device keep the overrides they were built under. */
int rure_amd_debug_set(const char *spec);
/* Diagnostics (bench): rure_amd_kernel_timer(1) resets and starts timing the
 * speculative kernel of every find_iter pass (the dominant kernel of a pass:
 * iter_spec_*; HIP events on the launch stream), (0) stops;
 * rure_amd_kernel_timer_read waits for the timed launches and returns their
 * average duration in ms (*launches = how many; -1 on a HIP error). */
int rure_amd_kernel_timer(int on);
double rure_amd_kernel_timer_read(uint64_t *launches);

#ifdef __cplusplus
}
#endif
#endif /* RURE_AMD_H */
