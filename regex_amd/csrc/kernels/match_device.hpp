// Device side of the reference's Literal and DfaSuffix match types (see
// MatchDev in dfa_scan.hpp): one lane runs one search.  Shared by the batch
// kernel (match_types.hip) and the wave-per-haystack find_iter kernel
// (iter_scan.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfa_device.hpp"

namespace rure_amd {

// Bit mask (bit k = byte k) of the bytes of w equal to the byte repeated in
// rep; may over-report above a match (borrow), never under-report.
__device__ __forceinline__ uint32_t eq_bytes(uint32_t w, uint32_t rep) {
  const uint32_t x = w ^ rep;
  const uint32_t z = (x - 0x01010101u) & ~x & 0x80808080u;
  return (z >> 7 & 1u) | (z >> 14 & 2u) | (z >> 21 & 4u) | (z >> 28 & 8u);
}

__device__ __forceinline__ bool bytes_at(const uint8_t *base, uint64_t p, const uint8_t *lit, uint32_t n) {
  for (uint32_t j = 0; j < n; ++j)
    if (base[p + j] != lit[j]) return false;
  return true;
}

// First p in [from, len - n] with text[p..p + n) == lit (n >= 1), or NONE:
// 16-byte aligned loads, a byte-equality mask of the first byte, then a
// byte-wise verification of the candidates (FreqyPacked::find, literals.rs
// 436-470, as a memchr on the first byte).
__device__ __forceinline__ uint64_t find_lit(const uint8_t *base, uint64_t from, uint64_t len, const uint8_t *lit,
                                             uint32_t n) {
  if (n == 0) return from <= len ? from : NONE;
  if (from + n > len) return NONE;
  const int64_t last = (int64_t)(len - n);  // last possible start
  const uint32_t rep = (uint32_t)lit[0] * 0x01010101u;
  // walk the 16-byte aligned blocks of memory (the haystack need not be
  // aligned; the buffer is readable at 16-byte granularity)
  int64_t blk = (int64_t)(((uintptr_t)(base + from)) & ~(uintptr_t)15) - (int64_t)(uintptr_t)base;
  for (; blk <= last; blk += 16) {
    const uint4 v = *(const uint4 *)(base + blk);
    uint32_t m = eq_bytes(v.x, rep) | eq_bytes(v.y, rep) << 4 | eq_bytes(v.z, rep) << 8 | eq_bytes(v.w, rep) << 12;
    while (m) {
      const int64_t q = blk + __builtin_ctz(m);
      m &= m - 1;
      if (q < (int64_t)from) continue;
      if (q > last) return NONE;
      if (bytes_at(base, (uint64_t)q, lit, n)) return (uint64_t)q;
    }
  }
  return NONE;
}

__device__ __forceinline__ const uint8_t *lit_ptr(const LitListDev &l, uint32_t i, uint32_t *n) {
  *n = l.off[i + 1] - l.off[i];
  return l.bytes + l.off[i];
}

// LiteralSearcher::find (literals.rs:92-103) over text[at..len): Empty -> the
// empty string at `at`; otherwise the leftmost occurrence of any literal
// (the set is unambiguous: at most one literal occurs at a position).
__device__ __forceinline__ bool lits_find(const LitListDev &l, const uint8_t *base, uint64_t len, uint64_t at,
                                          uint64_t *ms, uint64_t *me) {
  if (l.matcher == 0) {
    *ms = *me = at;
    return true;
  }
  uint64_t best = NONE, bend = NONE;
  for (uint32_t i = 0; i < l.n; ++i) {
    uint32_t n;
    const uint8_t *lit = lit_ptr(l, i, &n);
    // only occurrences starting before the best so far
    const uint64_t lim = best == NONE ? len : min(len, best + n - 1);
    const uint64_t q = find_lit(base, at, lim, lit, n);
    if (q != NONE && (best == NONE || q < best)) {
      best = q;
      bend = q + n;
    }
  }
  if (best == NONE) return false;
  *ms = best;
  *me = bend;
  return true;
}

// find_start / find_end (literals.rs:105-128)
__device__ __forceinline__ bool lits_find_start(const LitListDev &l, const uint8_t *base, uint64_t len,
                                                uint64_t at, uint64_t *ms, uint64_t *me) {
  if (l.matcher == 0) return false;
  for (uint32_t i = 0; i < l.n; ++i) {
    uint32_t n;
    const uint8_t *lit = lit_ptr(l, i, &n);
    if (at + n <= len && bytes_at(base, at, lit, n)) {
      *ms = at;
      *me = at + n;
      return true;
    }
  }
  return false;
}
__device__ __forceinline__ bool lits_find_end(const LitListDev &l, const uint8_t *base, uint64_t len, uint64_t at,
                                              uint64_t *ms, uint64_t *me) {
  if (l.matcher == 0) return false;
  for (uint32_t i = 0; i < l.n; ++i) {
    uint32_t n;
    const uint8_t *lit = lit_ptr(l, i, &n);
    if (n <= len - at && bytes_at(base, len - n, lit, n)) {
      *ms = len - n;
      *me = len;
      return true;
    }
  }
  return false;
}

// Reverse DFA over the slice text[lo..hi) as its own text (Fsm::reverse
// on &text[lo..hi], dfa.rs:492-522, 768-866), from hi: kind 1 = Match(pos),
// 0 = NoMatch(pos) (where the DFA died, lo when it ran out of input, hi for
// a dead start state), 2 = Quit.  Positions are absolute.
__device__ __forceinline__ int rev_slice(const RevDfaDev &r, const uint8_t *base, uint64_t lo, uint64_t hi,
                                         uint64_t *pos) {
  uint32_t s = r.ustart1 ? r.ustart1 - 1 : r.start[rev_flag_index(base, lo, hi, hi)];
  if (s == r.dead) { *pos = hi; return 0; }
  uint64_t rs = NONE;
  uint64_t a = hi;
  while (a > lo) {
    --a;
    s = r.full[(size_t)s * 256 + base[a]];
    if (s >= r.n_normal) {
      if (s < r.n_match_end) {
        rs = a + 1;
      } else if (s == r.dead) {
        *pos = rs != NONE ? rs : a;
        return rs != NONE ? 1 : 0;
      } else {
        return 2;
      }
    }
  }
  if (r.eof[s]) rs = lo;
  if (rs != NONE) { *pos = rs; return 1; }
  *pos = lo;  // ran out of input: NoMatch(0) whether the EOF step died or not
  return 0;
}

// exec.rs:725-756 exec_dfa_reverse_suffix: 1 Match (*ms, *me), 0 NoMatch,
// 2 Quit, -1 None (a reverse scan reached its slice start: the caller runs
// the forward DFA instead).
__device__ __forceinline__ int suffix_scan(const MatchDev &m, const RevDfaDev &r, const uint8_t *base, uint64_t len,
                                           uint64_t start0, uint64_t *ms, uint64_t *me) {
  uint64_t start = start0, end = start0;
  while (end <= len) {
    start = end;
    const uint64_t q = find_lit(base, end, len, m.lcs, m.lcs_len);
    if (q == NONE) return 0;
    end = q + m.lcs_len;
    uint64_t pos;
    const int k = rev_slice(r, base, start, end, &pos);
    if (k == 2) return 2;
    if (pos == start) return -1;  // Match(0) | NoMatch(0)
    if (k == 1) {
      *ms = pos;
      *me = end;
      return 1;
    }
  }
  return 0;
}

// One search of the regex under its match type (exec.rs:382-514) from `at`:
// MODE_FIND -> (ms, me), MODE_SHORTEST / MODE_ISMATCH -> me = the end.
// Returns 0 no match, 1 match, 2 quit.  fg: global-table forward DFA
// (hot = 0, all = 0).
template <int MODE>
__device__ __forceinline__ int mt_search(const MatchDev &m, const FwdDfaDev &fg, const RevDfaDev &r,
                                         const uint8_t *base, uint64_t len, uint64_t at, uint64_t *ms,
                                         uint64_t *me) {
  if (at > len) return 0;
  if (m.mt == MT_LIT_UNANCHORED) return lits_find(m.pre, base, len, at, ms, me) ? 1 : 0;
  if (m.mt == MT_LIT_ANCHORED_START) return lits_find_start(m.pre, base, len, at, ms, me) ? 1 : 0;
  if (m.mt == MT_LIT_ANCHORED_END) return lits_find_end(m.suf, base, len, at, ms, me) ? 1 : 0;
  // DfaSuffix
  uint64_t s0, e0;
  const int k = suffix_scan(m, r, base, len, at, &s0, &e0);
  if (k == 2) return 2;
  if (k == 0) return 0;
  if (k == 1 && MODE != MODE_FIND) {  // shortest_dfa_reverse_suffix: the suffix end
    *me = e0;
    return 1;
  }
  LaneState L;
  const uint64_t from = k == 1 ? s0 : at;  // None: the forward DFA from the search start
  if (MODE != MODE_FIND) {                 // shortest_dfa (quit after the first match)
    lane_start(L, fg, base, len, from);
    fwd_run<MODE_SHORTEST>(L, fg, nullptr, base, len, from);
    if (L.quit) return 2;
    if (L.last == NONE) return 0;
    *me = L.last;
    return 1;
  }
  if (k < 0) return dfa_find(fg, r, nullptr, nullptr, base, len, at, ms, me);
  // exec.rs:781-793: the forward DFA from the reverse scan's match start
  lane_start(L, fg, base, len, from);
  fwd_run<MODE_FIND>(L, fg, nullptr, base, len, from);
  if (L.quit) return 2;
  if (L.last == NONE) return 0;  // the reference panics ("reverse match implies forward match")
  *ms = s0;
  *me = L.last;
  return 1;
}

}  // namespace rure_amd
