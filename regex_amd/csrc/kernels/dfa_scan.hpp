// Device-side descriptors shared by the HIP kernels and the host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../host/knobs.hpp"

namespace rure_amd {

// Row pitch of the LDS hot tables (bytes).  256 columns + 48 bytes: row s
// starts 12 banks after row s-1, so lanes in the few dominant states reading
// random printable bytes (24 dwords of a row) collide least; a bank-conflict
// model over the C2 haystacks gives 4.15 LDS cycles per lookup
// wave-instruction at 304 vs 4.67 at 260 and 4.86 at 256 (2 = conflict free).
constexpr uint32_t kRow = 304;
// Column of the forward hot rows (in the padding) holding the row's own
// number: the identity step for bytes outside a masked block.
constexpr uint32_t kIdCol = 256;

enum { MODE_FIND = 0, MODE_ISMATCH = 1, MODE_SHORTEST = 2 };

struct BatchDev {
  const uint8_t *hay;
  const uint64_t *offs;   // n+1 offsets or nullptr (fixed stride)
  uint64_t stride, length, count, start;
  // set (atomic OR) by the DFA kernels when a haystack's DFA quit; the Pike VM
  // fallback pass then runs, else it returns at once (nullptr: always runs)
  uint32_t *quit_flag = nullptr;
  // a deferred fallback's gate (nullptr: always runs): the find_iter kernels
  // return at once unless (*gate != 0) == gate_set, so the ASCII shadow's
  // passes after its quit check and the full automaton's re-run are both
  // enqueued and one of them works (dispatch.cpp run_find_iter)
  const uint32_t *gate = nullptr;
  uint32_t gate_set = 0;
  // set masks (the Pike VM's MODE_SET): words between consecutive haystacks'
  // masks (a set of more than 64 patterns: group g writes word g)
  uint32_t out_stride = 1;
};

// Forward DFA on the device.  State ids: [0, hot) are in the LDS fast table
// (u8, 256 columns, row `hot` = absorbing sentinel); [0, n_normal) carry no
// match flag; [n_normal, n_match_end) carry the match flag; `dead`, `quit`.
struct FwdDfaDev {
  const uint8_t *lds_image;   // (hot + 1) * 256 bytes, padded to 16
  uint32_t lds_bytes;
  uint32_t hot;
  // Multi-byte fast table for the coalesced-tile kernel (stride 2 or 4 bytes
  // per LDS lookup over local byte classes of the ASCII-hot sub-DFA);
  // stride == 1 means "use lds_image".  Image: 4 x 256 u8 class tables
  // (class * K^(stride-1-p) for byte position p) then (hot_s + 1) * P u16
  // entries holding next_state * P; sentinel = hot_s * P.
  const uint8_t *lds_image_s;
  uint32_t lds_bytes_s;
  uint32_t stride, hot_s, P, sent;
  uint32_t cus;               // compute units of the device (launch heuristics)
  const uint16_t *full;       // nstates * 256
  const uint8_t *eof;         // nstates: EOF step yields a match flag
  const uint16_t *start;      // 128 start states by flag index
  const uint16_t *strip;      // find_iter DFA only: state minus the `.*?` prefix (or null)
  uint32_t n_normal, n_match_end, dead, quit;
  uint32_t all;               // lds_image rows are exact for every state (hot = nstates <= 255)
  uint32_t ustart1;           // 1 + the start state when it does not depend on the flags, else 0
  uint32_t nonempty;          // the regex never matches the empty string (the iteration's
                              // last-match state then never matters)
  // find_iter DFA only: the regex as a finite string set (host/literals.hpp),
  // lit_n = 0 if it is not one.  Image (kLit* offsets): 64 Kibit bitmap over
  // a hash of the first lit_k bytes, then keys (u32, first lit_k bytes), lens
  // (u8) and bytes (32 per literal), in leftmost-first priority order.
  const uint8_t *lit_image;
  uint32_t lit_bytes, lit_n, lit_k, lit_minlen, lit_maxlen;
  uint32_t lit_k8;            // every literal has >= 8 bytes: a second bitmap filters on bytes 4..7
  // find_iter DFA only: the string set as a bit-parallel Shift-And automaton
  // (sa_len = 0: none).  Every string has sa_len bytes; the set is a union of
  // class sequences (strings that differ in one position merged), sequence x
  // owning bits [x * sa_len, (x + 1) * sa_len).  sa_image: 256 u64 masks,
  // bit i of mask[b] = byte b is in the class of bit position i.
  const uint64_t *sa_image;
  uint64_t sa_init, sa_final;   // first / last bit of every sequence
  uint32_t sa_len, sa_bits;
  // find_iter DFA only: the first-byte start rule (fb_n = 0: off).  Every
  // match starts with one of fb_n <= 4 bytes (fb_rep[i] = byte * 0x01010101),
  // and an anchored run from such a byte never dies before it has matched
  // (host: first_byte_rule).  Then the leftmost match of a search from p
  // that ends in the dead state before the end of the text starts at the
  // first of those bytes at or after p, so the start needs no reverse scan.
  uint32_t fb_n;
  uint32_t fb_rep[4];
  // find_iter DFA only: the lexer table (lex_bytes = 0: none; host build_lex).
  // When the first-byte start rule holds and every match-flag state is
  // terminal (all transitions dead), the iteration itself is a DFA: entering
  // a match state at byte x ends the search there and the next one starts at
  // x, so that transition goes to a twin of the start state's successor on
  // the same byte.  u8 rows of kRow bytes; states numbered [others, S0 =
  // lex_s0, twin(S0), other twins] with the codes 0, 1, 2, 3 = the byte's
  // flags: 1 = the state after it is the start state (Z), 2 = Z and a
  // match ended at it (EMIT), 3 = EMIT only.
  const uint8_t *lex_image;
  uint32_t lex_bytes, lex_s0;
  // The same lexer four bytes per step (host build_lex4; lex4_image null:
  // none): at most kLex4Rows rows and 3 byte classes over ASCII, class 3 =
  // "no byte" (a partial word's tail).  kLex4Bytes of LDS: next row at
  // [row * 256 + c] (c = the four bytes' classes, 2 bits each), the four
  // bytes' flags (2 bits each, codes as above) at kLex4Flags + the same
  // index, and four byte -> class << 2j tables at kLex4Cls + 256 j.
  const uint8_t *lex4_image;
  uint32_t lex4_s0;
  // The start-state prefix skip (dfa.rs:700-711, 1504-1506 prefix_at): when
  // the regex has prefix literals (literal_sets.hpp, dfa.prefixes) whose
  // first bytes are at most 4 (pfx_rep[i] = byte * 0x01010101), every match
  // starts with one of them, so a scan in the start state (ustart1 - 1: the
  // start does not depend on look-behind) jumps over the 128-byte bursts
  // that hold none of those bytes (fwd_range); pfx_n = 0: off.
  uint32_t pfx_n;
  uint32_t pfx_rep[4];
  // The same skip on the prefixes' rarest bytes (literals.rs:390-510
  // FreqyPacked picks the rarest byte by a frequency table; here the table
  // is host/byte_freq.h, and on 128-byte bursts a pair is needed, a single
  // common-word letter being in nearly every burst): every prefix has byte
  // class 1 at offset i1 and class 2 at i1 + rare_d (d <= 3; d = 0: one
  // byte), each one byte or an ASCII letter's two cases (x | rare_or ==
  // rare_rep).  A burst [a, a + 128) is skipped when no q in [a, a + 144)
  // has class 1 at q and class 2 at q + d (i1 + d <= 15, so every start in
  // the burst is covered; positions past it only add candidates).  Used
  // where the prefixes have several first bytes ((?i)holmes); rare_on = 0:
  // the first-byte skip above.
  uint32_t rare_on, rare_d;
  uint32_t rare_rep[2], rare_or[2];
  // find_iter DFA only: the regex has look-around assertions (the chunked
  // iteration then repairs units whose first reverse scan reached their
  // start, and a reverse NoMatch ends the iteration; iter_scan.hip), and its
  // DFA can quit (1; 2: a Unicode word boundary's quit, whose units the wave
  // serves, iter_scan.hip).  The literal, Shift-And, lexer and first-byte
  // engines are off.
  uint32_t looks, can_quit;
  // find_iter DFA only: the regex is one byte class repeated (C+, host
  // run_class): run_cls[b] bit 0 = b is in C, bit 1 = b quits (the ASCII
  // shadow: bytes >= 0x80), bit 2 = decode (a Unicode class C+, host
  // unicode_run_set: bytes >= 0x80 are read as UTF-8 against run_cp, its
  // code point bitmap); null: not such a regex (run_iter.hip)
  const uint8_t *run_cls;
  const uint32_t *run_cp;
  uint32_t run_quit;  // some byte quits (bit 1): the run engine's flag is read back
};
constexpr uint32_t kLexMaxRows = 24;  // lexer table rows (iter_spec_lex_tile_kernel's static LDS)
constexpr uint32_t kLexUnit = kRow / 4;  // lexer entry -> row address multiplier
constexpr uint32_t kLexBytes = (kLexMaxRows * kRow + 3 * kLexUnit + 15) & ~15u;  // largest lexer image
constexpr uint32_t kLex4Rows = 8, kLex4Flags = kLex4Rows * 256, kLex4Cls = 2 * kLex4Flags;
constexpr uint32_t kLex4Bytes = kLex4Cls + 4 * 256;

// Literal engine image layout (at most kLitMax literals of kLitLen bytes).
constexpr uint32_t kLitMax = 64, kLitLen = 32;
constexpr uint32_t kLitKeys = 8192, kLitLens = kLitKeys + 4 * kLitMax, kLitBytes = kLitLens + kLitMax;
constexpr uint32_t kLitBitmap2 = kLitBytes + kLitMax * kLitLen;  // second bitmap: bytes 4..7 (lit_k8)
constexpr uint32_t kLitImage = kLitBitmap2 + 8192;
__host__ __device__ inline uint32_t lit_hash(uint32_t key) { return (key * 0x9E3779B1u) >> 16; }

// The reference's engine choice where it differs from the forward DFA
// (host/literal_sets.hpp): MatchType::Literal over the reference's literal
// sets (exec.rs:601-625) and DfaSuffix (exec.rs:725-794).  Literal lists:
// `n` literals, literal i = bytes[off[i] .. off[i + 1]), in the searcher's
// iteration order; matcher 0 = Empty (literals.rs:92-96: every search finds
// the empty string at its start).
struct LitListDev {
  const uint8_t *bytes;
  const uint32_t *off;
  uint32_t n;
  int32_t matcher;
};
// mt: host/literal_sets.hpp MatchTypeCode (0-2 the Literal types, 5 DfaSuffix)
enum { MT_LIT_UNANCHORED = 0, MT_LIT_ANCHORED_START = 1, MT_LIT_ANCHORED_END = 2 };
struct MatchDev {
  int32_t mt;             // MT_* code
  LitListDev pre, suf;    // nfa.prefixes, suffixes
  const uint8_t *lcs;     // suffixes.lcs() (DfaSuffix)
  uint32_t lcs_len;
};

struct RevDfaDev {
  const uint8_t *lds_image;   // hot table (same layout as FwdDfaDev::lds_image)
  uint32_t lds_bytes;
  uint32_t hot;
  const uint16_t *full;
  const uint8_t *eof;
  const uint16_t *start;
  uint32_t n_normal, n_match_end, dead, quit;
  uint32_t all;               // as FwdDfaDev::all
  uint32_t ustart1;           // as FwdDfaDev::ustart1
};

// Set DFA: the answer is the union of now_mask[s] over the states entered
// ([n_normal, n_match_end) have now_mask != 0) and eof_mask[final state].
struct SetDfaDev {
  const uint8_t *lds_image;
  uint32_t lds_bytes;
  uint32_t hot;
  const uint16_t *full;
  const uint64_t *eof_mask;
  const uint64_t *now_mask;
  uint64_t all;               // every pattern (early exit)
  const uint16_t *start;
  uint32_t n_normal, n_match_end, dead, quit;
};

// Set DFA in "core" form for large sets (host: build_set_cores): states that
// differ only in the matches their entry reports share a core; a transition
// (core, byte class) carries the next core and an output code.  Entries of
// the LDS table (hot cores [0, hot), sentinel row `hot`): bits 15..6 = next
// core (`hot` = leaves the LDS set), bits 5..0 = output code (0 none, 1..62 =
// pattern code-1 matched, 63 = consult gout).  Global tables cover all cores.
struct SetCoreDev {
  const uint8_t *lds_image;   // 256-byte class map, then (hot + 1) x K u16 entries
  uint32_t lds_bytes;
  uint32_t hot, K;
  const uint16_t *gcore;      // ncores x K next core
  const uint64_t *gout;       // ncores x K matches reported by the transition
  const uint64_t *eof;        // ncores: matches at the end of the text
  const uint16_t *start;      // 128 start cores
  uint64_t all;
  uint32_t dead, quit;        // quit = 0xFFFFFFFF if none
  uint32_t mt_off;            // byte offset in the LDS image of the 64 u64 code masks
  const uint16_t *mid;        // profile only: ncores x K mask id + 1 of gout (0: none)
};
hipError_t launch_set_cores(const BatchDev &b, const SetCoreDev &f, uint64_t *out, hipStream_t st, int cus);

hipError_t launch_core_profile(const BatchDev &b, const SetCoreDev &f, uint64_t count, unsigned int *visits,
                               unsigned int *mask_counts, hipStream_t st, int cus);

// Pike VM closure tables (host/nfa_build.hpp) on the device.
struct NfaDev {
  const uint32_t *leaves;     // 3 words per leaf: kind | lo << 8 | hi << 16, closure, slot
  const uint32_t *cl_off;     // closure CSR offsets
  const uint2 *entries;       // (leaf, cond | (1 + prev same-leaf entry) << 8)
  const uint32_t *perlw;      // Unicode word-character ranges (pairs), regex-syntax PERLW
  uint32_t perlw_n;
  uint32_t nleaves, root, nmatch;
  uint32_t anchored, single, looks, unicode_wb;
  uint32_t ncl_off, nentries;  // cl_off's and entries' lengths (the wave kernels stage them in LDS)
  const uint32_t *cl_info;     // per closure: its Bytes leaves' bytes (8 words), needed looks | Match << 8
  const uint32_t *cl_big;      // per closure: its bucket set (closures of > 64 entries), else ~0
  const uint32_t *cl_boff;     // per bucket set: 258 offsets into cl_sub (bytes 0-255, the text end)
  const uint2 *cl_sub;         // the buckets' entries (as `entries`, same-leaf links within the bucket)
  const uint32_t *save_off;   // per entry: CSR offsets into save_slot (Saves on its path)
  const uint16_t *save_slot;
};

// Per-wave working set of the Pike VM: stamp + two thread lists.
__host__ __device__ inline size_t nfa_wave_bytes(uint32_t nleaves) { return ((size_t)nleaves * 28 + 64 + 255) & ~(size_t)255; }
constexpr size_t kNfaLdsMax = 160 * 1024;   // a gfx950 workgroup may take the whole LDS

// mode: MODE_FIND / MODE_ISMATCH / MODE_SHORTEST, or MODE_SET.  fallback:
// only haystacks whose DFA result is the quit marker are (re)computed.
enum { MODE_SET = 3 };
hipError_t launch_pike(int mode, bool fallback, const BatchDev &b, const NfaDev &n, void *out, void *scratch,
                       hipStream_t st, int grid);

// Captures (exec.rs:524-596 read_captures_at; Pike VM with capture slots,
// pikevm.rs:237-352).  found: per haystack the forward/reverse DFA's
// (start, end), NONE or the quit marker; null when every haystack is searched
// whole from `start` (anchored-start programs).  slots: count x nslots u64,
// NONE = unset.  Per-wave working set: caps_wave_bytes (LDS when it fits).
__host__ __device__ inline size_t caps_wave_bytes(uint32_t nleaves, uint32_t nslots) {
  return ((size_t)nleaves * (16 * (size_t)nslots + 12) + 64 + 255) & ~(size_t)255;
}
hipError_t launch_captures(const BatchDev &b, const NfaDev &n, const uint64_t *found, uint64_t *slots,
                           uint32_t nslots, void *scratch, hipStream_t st, int grid);

// replacen / split over find_iter output (replace_scan.hip).  counts / moff:
// matches per haystack and their exclusive sums; m: the records.
hipError_t exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t st);
// shift: nm + 1 entries; one haystack with every match replaced holds the
// replacement starts there instead (the plan's output, the copy's input).
hipError_t launch_replace_plan(const BatchDev &b, const uint64_t *counts, const uint64_t *moff, const uint64_t *m,
                               uint64_t limit, uint64_t rep_len, int64_t *shift, uint64_t *out_len, hipStream_t st,
                               int cus,
                               uint64_t nm);
hipError_t launch_replace_copy(const BatchDev &b, const uint64_t *ooff, const uint64_t *counts, const uint64_t *moff,
                               const uint64_t *m, const int64_t *shift, uint64_t limit, const uint8_t *rep,
                               uint64_t rep_len, uint8_t *out, uint64_t cap, uint64_t total_hint, hipStream_t st,
                               int cus,
                               uint64_t nm);
// replace_all of a regex whose matches are single bytes of one class over
// one 16-byte aligned haystack (replace_scan.hip); hipErrorNotSupported if
// the replacement is empty or longer than 64 bytes.
// sw1 / sw2: a class of at most two bytes (byte * 0x01010101; sw2 = sw1 for
// one byte), else 0 (the cls table).
hipError_t launch_replace_class(const uint8_t *hay, uint64_t n, const uint8_t *cls, const uint8_t *rep,
                                uint32_t rep_len, uint8_t *out, uint64_t cap, uint64_t *ooff, uint64_t *total,
                                hipStream_t st, int cus, uint32_t sw1, uint32_t sw2);
// A chain of one-byte-class replace_all calls (replace_scan.hip): step i
// reads step i - 1's output, buffers alternate out0 / out1, lengths (device,
// steps + 1) = the input length, then each step's output length; sw[i] = step
// i's class as up to two SWAR bytes ({0, 0}: wider, counted from cls[i]).
// The same chain as one byte -> string map composed on the host (blob:
// |F(x)| 256 u8, offsets 256 u16, changed-byte indices 256 u8 (0xFF: F(x) =
// x; nact changed), the strings (<= 4096 bytes), per step |F_i(x)| - 1 as
// 256 u32); the final text to out.
constexpr uint32_t kHMapPoolMax = 4096;
hipError_t launch_replace_hmap(const uint8_t *in, uint64_t n, int steps, const uint8_t *blob, uint32_t pool_len,
                               uint32_t nact, uint8_t *out, uint64_t cap, uint64_t *lengths, hipStream_t st,
                               int cus);
// nrep[i] = the bytes of step i's replacement in step i + 1's class.
hipError_t launch_replace_class_chain(const uint8_t *hay, uint64_t n0, int steps, const uint8_t *const *cls,
                                      const uint8_t *const *rep, const uint32_t *rep_len, const uint32_t (*sw)[2],
                                      const uint32_t *nrep, uint8_t *out0, uint8_t *out1, uint64_t cap,
                                      uint64_t *lengths, hipStream_t st, int cus);
hipError_t launch_split(const BatchDev &b, const uint64_t *counts, const uint64_t *moff, const uint64_t *m,
                        uint64_t lim, uint64_t *fields, uint64_t *foff, uint64_t *pieces, uint64_t cap,
                        uint64_t nmatches, hipStream_t st, int cus);

// Batched find_iter (iter_scan.hip).  counts: per haystack; matches:
// (start, end) pairs, the first `cap` written; total: number of matches.
struct IterOut {
  uint64_t *counts;
  uint64_t *matches;
  uint64_t cap;
  uint64_t *total;
};
// A span of one haystack (sharded / streamed find_iter): the iteration owns
// the matches starting before `hi`; entry (device, 3 u64: next, last match,
// fresh) = the state the previous span left (fresh: start at b.start); exit
// (device, 3 u64) receives the state at hi (fresh = equivalent to a fresh
// iteration starting at hi).
struct IterSpan {
  uint64_t hi;
  const uint64_t *entry;
  uint64_t *exit;
  uint64_t tail;  // the text length when the span runs to the end (hi = ~0), else ~0
};
// find_iter of a C+ regex (FwdDfaDev::run_cls, run_iter.hip): fixed-stride
// batches whose searched bytes are 16-byte aligned (hipErrorNotSupported
// otherwise); *quit = a byte of the quit class was read (can_quit: the
// flag is read back) and the results are not the answer.
// cp: a Unicode class's code point bitmap (class bit 2 on bytes >= 0x80),
// else null.
hipError_t launch_find_iter_runs(const BatchDev &b, const uint8_t *cls, const uint32_t *cp, const IterOut &o,
                                 hipStream_t st, int cus, bool can_quit, bool *quit);
hipError_t launch_find_iter(const BatchDev &b, const FwdDfaDev *f, const RevDfaDev &r, const NfaDev *nf,
                            bool chunked, uint64_t chunk, const IterOut &o, hipStream_t st, int cus,
                            const IterSpan *span = nullptr, const MatchDev *mt = nullptr, bool *quit = nullptr,
                            uint32_t *quit_dev = nullptr);
// (quit: chunked with a DFA that can quit, f->can_quit; set when a search
// quit, the outputs then being void: the caller runs the wave path.  Reads
// the flag back, so the call synchronises the stream.  quit_dev instead (a
// zeroed device word, chunked, no span): a quit ORs 1 into it and the passes
// after the speculative one run gated on it staying 0 -- nothing is read
// back, and the caller enqueues its fallback gated on the word being set.)
// The k-mer probe engine of launch_find_iter_multi: the regexes' strings all
// have one length len <= 8 over an alphabet of at most 4 bytes whose codes
// (b >> shift) & 3 are distinct.  bitmap: 2048 u32, bit c set iff the L-mer
// with code c (2 bits per byte, first byte lowest) is a string of some regex;
// mask: 4^len u16, regex q's bit set iff its strings hold it; lut / present:
// the byte of each code (verification of probe hits on the text).
struct KmerDev {
  const uint32_t *bitmap;
  const uint16_t *mask;
  const uint16_t *hmask;  // 1024: mask[c] at (c * hmul) >> 22, injective on the string codes
  uint32_t hmul;
  uint32_t hglobal;       // 1: no injective hash was found; hits read mask[code] from global memory
  uint32_t vlut;  // byte k: the alphabet byte of code k (absent code: a byte of another code)
  uint32_t shift, lut, present, cmask;
  uint64_t len;
};
// Several Shift-And regexes over one span in one speculative pass, then each
// regex's own passes; hipErrorNotSupported (nothing launched) if they do not
// qualify (iter_scan.hip).  km (may be null): the k-mer probe engine for the
// pass instead of the Shift-And words.
hipError_t launch_find_iter_multi(const BatchDev &b, int nre, const FwdDfaDev *const *f, const RevDfaDev *const *r,
                                  uint64_t chunk, const IterOut *o, hipStream_t st, int cus, const IterSpan *spn,
                                  const KmerDev *km = nullptr);

// One search per haystack over few long fixed-stride haystacks, chunked
// (iter_scan.hip); f must be the find_iter DFA (with strip).
hipError_t launch_long_scan(int mode, const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, uint64_t chunk,
                            void *out, hipStream_t st, int cus);

hipError_t launch_dfa_fwd(int mode, const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out,
                          hipStream_t st, int grid);
// find / is_match / shortest_match of a batch under the reference's Literal
// or DfaSuffix match type (match_types.hip): one lane per haystack, global
// DFA tables for DfaSuffix's reverse / forward scans; same output layout and
// quit markers as launch_dfa_fwd (the Pike VM pass resolves quits);
// last_fwd_path() = -5.
hipError_t launch_lane_search(int mode, const BatchDev &b, const MatchDev &m, const FwdDfaDev &f,
                              const RevDfaDev &r, void *out, hipStream_t st, int cus);
// DfaSuffix over few long fixed-stride haystacks (match_types.hip): answers
// into out where the reverse suffix scans decide; status[h] = 3 where the
// reference falls back to the forward DFA (the caller runs it).  Needs a
// longest common suffix that cannot overlap itself.
// find_iter of a DfaSuffix regex over few long fixed-stride haystacks
// (match_types.hip): every suffix occurrence's slice scanned once, each
// search's match and successor per occurrence, the iteration's searches
// marked by pointer doubling.  hipErrorNotSupported: nothing written (a
// reverse scan quit), the caller runs the wave path.
hipError_t launch_suffix_iter(const BatchDev &b, const MatchDev &m, const FwdDfaDev &f, const RevDfaDev &r,
                              uint64_t chunk, const IterOut &o, hipStream_t st, int cus);
hipError_t launch_suffix_long(int mode, const BatchDev &b, const MatchDev &m, const FwdDfaDev &f,
                              const RevDfaDev &r, uint64_t chunk, void *out, uint8_t *status, hipStream_t st,
                              int cus);
// MatchType::Literal (exec.rs:601-625, 1148-1166) for MODE_FIND / MODE_ISMATCH
// batches of a regex that is a finite string set: f = the find_iter DFA
// (lit_n > 0); same output layout as launch_dfa_fwd; last_fwd_path() = -3.
hipError_t launch_lit_find(int mode, const BatchDev &b, const FwdDfaDev &f, void *out, hipStream_t st);
// Which forward-scan kernel the last launch_dfa_fwd call launched (tests
// assert the instantiation the bench times): 0 = dfa_fwd_kernel (per-lane
// streaming), 1 / 2 / 4 = dfa_fwd_tile_kernel with that many bytes per
// dependent LDS lookup, -2 = the anchored reverse scan, -3 = the literal
// engine, -4 = the chunked long scan (launch_long_scan).
int last_fwd_path();
void note_fwd_path(int path);
// Kernel timer (rure_amd_kernel_timer): HIP event pairs around bracketed launches.
void ktimer_begin(hipStream_t st);
void ktimer_end(hipStream_t st);
int ktimer_set(int on);
double ktimer_read(uint64_t *launches);
// Multi-GPU gather (gather_scan.hip): records (3 u64: base + haystack, start,
// end) of the haystacks whose find result holds a match, first `cap`; *count.
hipError_t launch_compact_matches(const uint64_t *found, uint64_t n, uint64_t base, uint64_t *rec, uint64_t cap,
                                  uint64_t *count, hipStream_t st);
// find_iter from the batched find result when a haystack holds at most that
// match (gather_scan.hip): counts, records, total as launch_find_iter.
hipError_t launch_find_to_iter(const uint64_t *found, uint64_t n, uint64_t *counts, uint64_t *matches, uint64_t cap,
                               uint64_t *total, hipStream_t st);
// dst[i * words + w] = src (u8 0/1 or u64 mask) of haystack i (gather_scan.hip).
hipError_t launch_mask_column(const uint8_t *s8, const uint64_t *s64, uint64_t n, uint64_t *dst, uint64_t words,
                              uint64_t w, hipStream_t st);
// MatchType::DfaAnchoredReverse (exec.rs:671-688, 395-406, 442-453): the
// reverse DFA over text[start..] from its end; same output layout and quit
// markers as launch_dfa_fwd.
hipError_t launch_dfa_anchored_rev(int mode, const BatchDev &b, const RevDfaDev &r, void *out, hipStream_t st,
                                   int grid);
hipError_t launch_dfa_set(const BatchDev &b, const SetDfaDev &f, uint64_t *out, hipStream_t st, int grid);

// An automaton past the u16 tables (more than 65535 states, host
// kBigDfaRawStates budget): u32 next states in column form, trans[s * ncol +
// colmap[b]], same state numbering as FwdDfaDev / RevDfaDev (no quit state:
// programs with a Unicode word boundary keep the Pike VM).  The first `hot`
// rows are staged in LDS (states in BFS order from the start states).
struct BigDfaDev {
  const uint32_t *trans;
  const uint8_t *colmap;      // 256 bytes
  const uint8_t *eof;         // nstates
  const uint32_t *start;      // 128 start states by flag index
  uint32_t ncol, nstates, hot, n_normal, n_match_end, dead, ustart1;
};
// find / is_match / shortest_match over a batch, one lane per haystack:
// find_dfa_forward (exec.rs:632-662) with the big forward and reverse DFAs.
hipError_t launch_big_dfa(int mode, const BatchDev &b, const BigDfaDev &f, const BigDfaDev &r, void *out,
                          hipStream_t st, int cus);
// Rows of a big forward DFA the kernel holds in LDS.
uint32_t big_dfa_hot_rows(uint32_t ncol, uint32_t nstates);

// A forward DFA built on demand (host LazyDfa): entries are next-state ids,
// | 0x80000000 when that state carries the match flag, 0x7FFFFFFF for a row
// not built yet; id 0 is the dead state.  The first `hot` rows sit in LDS.
struct LazyDfaDev {
  const uint32_t *trans;
  const uint8_t *colmap;      // 256 bytes
  const uint8_t *eof;         // per state
  const uint32_t *start;      // 128 start entries by flag index
  uint32_t ncol, hot;
};
// A lane stopped at a row not built yet: haystack, position of the byte it
// needs, the last match end so far (~0: none), the state.
struct LazyPark {
  uint64_t h, p, last;
  uint32_t s, pad;
};
// One round of a batched forward scan on a LazyDfaDev (find: the reverse
// DFA r gives the start, exec.rs:632-662): lanes are the haystacks (in =
// nullptr) or the parked lanes of the previous round; lanes that need a
// missing row are appended to park (*npark).
hipError_t launch_lazy_dfa(int mode, const BatchDev &b, const LazyDfaDev &f, const RevDfaDev &r, const LazyPark *in,
                           uint64_t nin, LazyPark *park, unsigned long long *npark, void *out, hipStream_t st,
                           int cus);
uint32_t lazy_dfa_hot_rows(uint32_t ncol);

// Scratch device memory for the scans, cached by the library (scratch.cpp):
// a freed block is kept with an event recorded on the freeing stream and
// reused, after a wait on that event, by the next allocation of at most twice
// its size on any stream of the device — freeing to the driver (hipFree,
// hipFreeAsync) waits for queued work: 1-2 ms host stalls, one per freed
// scratch, made the C3 variant phase spend more host time freeing than the
// GPU spent scanning.  The cache is bounded and released on request
// (rure_amd_release_scratch).  Same signatures as hipMallocAsync /
// hipFreeAsync (the memory is usable on any stream once the call returns).
hipError_t scratch_malloc(void **p, size_t bytes, hipStream_t st);
hipError_t scratch_free(void *p, hipStream_t st);

}  // namespace rure_amd
