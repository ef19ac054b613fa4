// Device-side DFA stepping shared by the scan kernels (dfa_scan.hip) and the
// find_iter kernels (iter_scan.hip).  See dfa_scan.hip for the layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfa_scan.hpp"

namespace rure_amd {

__device__ __forceinline__ bool word_byte(uint32_t b) {
  return b == '_' || (b - '0') < 10u || ((b | 0x20) - 'a') < 26u;
}

// dfa.rs:1415-1434
__device__ __forceinline__ uint32_t fwd_flag_index(const uint8_t *base, uint64_t len, uint64_t at) {
  bool start = at == 0, end = len == 0;
  bool start_line = at == 0 || base[at - 1] == '\n';
  bool wl = at > 0 && word_byte(base[at - 1]);
  bool wn = at < len && word_byte(base[at]);
  return (start ? 1u : 0u) | (end ? 2u : 0u) | (start_line ? 4u : 0u) | (end ? 8u : 0u) |
         (wl != wn ? 16u : 32u) | (wl ? 64u : 0u);
}

// dfa.rs:1440-1464, on the slice text[lo..] with the search ending at `at`.
__device__ __forceinline__ uint32_t rev_flag_index(const uint8_t *base, uint64_t lo, uint64_t len,
                                                   uint64_t at) {
  bool start = at == len, end = lo == len;
  bool start_line = at == len || base[at] == '\n';
  bool wl = at < len && word_byte(base[at]);
  bool wn = at > lo && word_byte(base[at - 1]);
  return (start ? 1u : 0u) | (end ? 2u : 0u) | (start_line ? 4u : 0u) | (end ? 8u : 0u) |
         (wl != wn ? 16u : 32u) | (wl ? 64u : 0u);
}

struct LaneState {
  uint32_t s;
  uint64_t last;   // last match end (NONE if none)
  bool done;
  bool quit;
  bool fast;       // multi-byte path: t holds s * P and s may be stale
  uint32_t t;
};

static constexpr uint64_t NONE = ~0ull;
static constexpr uint64_t QUITMARK = ~0ull - 1;

// The bookkeeping of entering state s at haystack position `pos`.
template <int MODE>
__device__ __forceinline__ void enter_state(LaneState &L, const FwdDfaDev &f, uint32_t s, uint64_t pos) {
  L.s = s;
  if (s >= f.n_normal) {
    if (s < f.n_match_end) {                 // dfa.rs:658-668: Match(at - 1)
      L.last = pos;
      if (MODE != MODE_FIND) L.done = true;  // quit_after_match
    } else if (s == f.dead) {                // dfa.rs:728-731
      L.done = true;
    } else {                                 // STATE_QUIT (dfa.rs:713-715)
      L.quit = true;
      L.done = true;
    }
  }
}

// Full-table step for one byte at haystack position `pos` (careful path).
template <int MODE>
__device__ __forceinline__ void careful_step(LaneState &L, const FwdDfaDev &f, uint32_t b, uint64_t pos) {
  enter_state<MODE>(L, f, f.full[(size_t)L.s * 256 + b], pos);
}

template <int MODE>
__device__ __forceinline__ void step1(LaneState &L, const FwdDfaDev &f, const uint8_t *lds,
                                      uint32_t b, uint64_t pos) {
  if (f.all) {  // exact LDS table for every state
    enter_state<MODE>(L, f, lds[__umul24(L.s, kRow) + b], pos);
    return;
  }
  if (L.s < f.hot) {
    uint32_t t = lds[__umul24(L.s, kRow) + b];
    if (t != f.hot) { L.s = t; return; }
  }
  careful_step<MODE>(L, f, b, pos);
}

// 4 fast-path steps on the bytes of `w` (little endian): byte extraction is
// off the dependency chain; the chain is one v_mad_u32_u24 + one ds_read_u8.
__device__ __forceinline__ uint32_t fast4(uint32_t s, uint32_t w, const uint8_t *lds) {
  const uint32_t b0 = w & 0xFF, b1 = (w >> 8) & 0xFF, b2 = (w >> 16) & 0xFF, b3 = w >> 24;
  s = lds[__umul24(s, kRow) + b0];
  s = lds[__umul24(s, kRow) + b1];
  s = lds[__umul24(s, kRow) + b2];
  s = lds[__umul24(s, kRow) + b3];
  return s;
}

// 4 exact steps (every state in LDS); mx collects the largest state entered
// (off the dependency chain): mx < n_normal means no match / dead / quit.
__device__ __forceinline__ uint32_t exact4(uint32_t s, uint32_t w, const uint8_t *lds, uint32_t &mx) {
  s = lds[__umul24(s, kRow) + (w & 0xFF)];
  mx = max(mx, s);
  s = lds[__umul24(s, kRow) + ((w >> 8) & 0xFF)];
  mx = max(mx, s);
  s = lds[__umul24(s, kRow) + ((w >> 16) & 0xFF)];
  mx = max(mx, s);
  s = lds[__umul24(s, kRow) + (w >> 24)];
  mx = max(mx, s);
  return s;
}

template <int MODE>
__device__ __forceinline__ void chunk16(LaneState &L, const FwdDfaDev &f, const uint8_t *lds,
                                        uint4 v, uint64_t pos) {
  if (f.all) {
    uint32_t t = L.s, mx = 0;
    t = exact4(t, v.x, lds, mx);
    t = exact4(t, v.y, lds, mx);
    t = exact4(t, v.z, lds, mx);
    t = exact4(t, v.w, lds, mx);
    if (mx < f.n_normal) { L.s = t; return; }
  } else if (L.s < f.hot) {
    uint32_t t = L.s;
    t = fast4(t, v.x, lds);
    t = fast4(t, v.y, lds);
    t = fast4(t, v.z, lds);
    t = fast4(t, v.w, lds);
    if (t != f.hot) { L.s = t; return; }
  }
  // Re-run the chunk exactly, byte by byte.
  uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll 1
  for (int j = 0; j < 16; ++j) {
    step1<MODE>(L, f, lds, (words[j >> 2] >> ((j & 3) * 8)) & 0xFF, pos + j);
    if (L.done) return;
  }
}

// Multi-byte fast path (STRIDE = 2 or 4 bytes per dependent LDS lookup).
// The class lookups do not depend on the state, so only one LDS round trip
// per STRIDE bytes sits on the critical path.
template <int STRIDE>
__device__ __forceinline__ uint32_t fastS(uint32_t t, uint32_t w, const uint8_t *cls, const uint16_t *tab) {
  if (STRIDE == 4) {
    uint32_t a = cls[w & 0xFF] + cls[256 + ((w >> 8) & 0xFF)] + cls[512 + ((w >> 16) & 0xFF)] + cls[768 + (w >> 24)];
    return tab[t + a];
  } else {
    uint32_t a0 = cls[w & 0xFF] + cls[256 + ((w >> 8) & 0xFF)];
    uint32_t a1 = cls[(w >> 16) & 0xFF] + cls[256 + (w >> 24)];
    t = tab[t + a0];
    return tab[t + a1];
  }
}

template <int MODE, int STRIDE>
__device__ __forceinline__ void chunk16s(LaneState &L, const FwdDfaDev &f, const uint8_t *cls, const uint16_t *tab,
                                         uint4 v, uint64_t pos) {
  if (L.fast) {
    uint32_t t = L.t;
    t = fastS<STRIDE>(t, v.x, cls, tab);
    t = fastS<STRIDE>(t, v.y, cls, tab);
    t = fastS<STRIDE>(t, v.z, cls, tab);
    t = fastS<STRIDE>(t, v.w, cls, tab);
    if (t != f.sent) { L.t = t; return; }
    L.s = L.t / f.P;  // real state at the chunk start (rare path)
    L.fast = false;
  }
  uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll 1
  for (int j = 0; j < 16; ++j) {
    careful_step<MODE>(L, f, (words[j >> 2] >> ((j & 3) * 8)) & 0xFF, pos + j);
    if (L.done) return;
  }
  if (L.s < f.hot_s) { L.t = L.s * f.P; L.fast = true; }
}

// Reverse DFA over text[lo..me] (exec.rs:651-661, dfa.rs:768-866): longest
// match, i.e. the smallest start.  Returns the start, NONE (reverse NoMatch)
// or QUITMARK.  Text bytes come from aligned 16-byte loads walked backwards;
// with `rlds` (the reverse DFA's hot table staged in LDS, same layout as the
// forward one) ordinary steps stay in LDS.
// QAM (quit_after_match, dfa.rs:805-812): return at the first match flag
// (is_match / shortest_match of DfaAnchoredReverse; any match position).
// reached (optional): set when the scan got to `lo` alive, i.e. its answer
// may depend on where the slice starts (with look-around, the EOF step at lo
// reads lo as the text's start).
template <bool QAM = false>
__device__ __forceinline__ uint64_t rev_scan(const RevDfaDev &r, const uint8_t *rlds, const uint8_t *base,
                                             uint64_t len, uint64_t lo, uint64_t me, bool *reached = nullptr) {
  uint32_t s = r.ustart1 ? r.ustart1 - 1 : r.start[rev_flag_index(base, lo, len, me)];
  if (s == r.dead) return NONE;
  const uint32_t hot = rlds ? r.hot : 0;
  const bool all = rlds && r.all;
  uint64_t rs = NONE;
  uint64_t a = me;
  while (a > lo) {
    const uintptr_t p = (uintptr_t)(base + a - 1);
    const uint4 v = *(const uint4 *)(p & ~(uintptr_t)15);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll 1
    for (int j = (int)(p & 15); j >= 0 && a > lo; --j) {
      const uint32_t b = (w[j >> 2] >> ((j & 3) * 8)) & 0xFF;
      --a;
      if (all) {
        s = rlds[__umul24(s, kRow) + b];
      } else {
        if (s < hot) {
          const uint32_t t = rlds[__umul24(s, kRow) + b];
          if (t != hot) { s = t; continue; }
        }
        s = r.full[(size_t)s * 256 + b];
      }
      if (s >= r.n_normal) {
        if (s < r.n_match_end) {
          rs = a + 1;
          if (QAM) return rs;
        } else if (s == r.dead) {
          return rs;
        } else {
          return QUITMARK;
        }
      }
    }
  }
  if (reached) *reached = true;
  if (r.eof[s]) rs = lo;
  return rs;
}

// Whether the 128 bytes of v hold one of the prefix first bytes (pfx_rep).
__device__ __forceinline__ uint32_t has_byte(uint32_t w, uint32_t rep) {
  const uint32_t x = w ^ rep;
  return (x - 0x01010101u) & ~x & 0x80808080u;
}
__device__ __forceinline__ bool prefix_hit(const FwdDfaDev &f, const uint4 *v) {
  uint32_t acc = 0;
  for (uint32_t i = 0; i < f.pfx_n; ++i) {
    const uint32_t rep = f.pfx_rep[i];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      acc |= has_byte(v[k].x, rep) | has_byte(v[k].y, rep) | has_byte(v[k].z, rep) | has_byte(v[k].w, rep);
  }
  return acc != 0;
}

// FwdDfaDev::rare_*: whether the 144 bytes of v (the burst and the next 16)
// hold a candidate start of the burst.
__device__ __forceinline__ bool rare_hit(const FwdDfaDev &f, const uint4 *v) {
  const uint32_t r1 = f.rare_rep[0], o1 = f.rare_or[0], r2 = f.rare_rep[1], o2 = f.rare_or[1];
  const uint32_t sh = 8 * f.rare_d;
  uint32_t acc = 0, a_prev = 0, b_prev = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t a = has_byte(w4[q] | o1, r1), b = has_byte(w4[q] | o2, r2);
      if (k + q > 0) acc |= a_prev & __builtin_amdgcn_alignbit(b, b_prev, sh);
      a_prev = a;
      b_prev = b;
    }
  }
  // the last word's class-2 bytes past the window count as hits
  acc |= a_prev & __builtin_amdgcn_alignbit(0x80808080u, b_prev, sh);
  return acc != 0;
}

// One lane's forward scan of text[at..end) (dfa.rs:576-764): 16-byte
// chunks through the LDS fast table, 128-byte bursts per lane.  No EOF step.
// PFX: with the start-state prefix skip (FwdDfaDev::pfx_*).  A separate
// instantiation: the skip loop costs the scan ~58 VGPRs (long_scan_kernel
// 82 -> 140, half the waves per SIMD), so kernels for regexes without a
// prefix set are built without it.
template <int MODE, bool PFX = false>
__device__ __forceinline__ void fwd_range(LaneState &L, const FwdDfaDev &f, const uint8_t *lds, const uint8_t *base,
                                          uint64_t at, uint64_t end) {
  // head: the bytes up to the next 16-byte boundary come from one aligned
  // 16-byte load (the haystack buffer is readable up to its 16-byte-rounded
  // end), not from a chain of byte loads
  if (!L.done && at < end && (((uintptr_t)(base + at)) & 15)) {
    const uintptr_t a = (uintptr_t)(base + at);
    const uint4 v = *(const uint4 *)(a & ~(uintptr_t)15);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t j = (uint32_t)(a & 15);
#pragma unroll 1
    for (; j < 16 && at < end && !L.done; ++j, ++at) step1<MODE>(L, f, lds, (w[j >> 2] >> ((j & 3) * 8)) & 0xFF, at);
  }
  // (Tried, round 6: a lane switching its skip off once half of 8 or 32
  // tested bursts held a candidate.  Worse: a lane that stops skipping still
  // runs this instantiation, with half the waves of the one without the skip
  // loop, so the first-byte skip lost 19-42 % where a few early bursts held
  // its byte; profiles/r06_prefix_ab.jsonl.)
  while (!L.done && at + 128 <= end) {
    if (PFX && (f.pfx_n || f.rare_on) && L.s + 1 == f.ustart1) {
      // start-state prefix skip (dfa.rs:700-711): bursts without a prefix
      // first byte cannot start a match, and the state stays the start state
      while (true) {
        uint4 t[9];
        const uint4 *q = (const uint4 *)(base + at);
        if (f.rare_on) {
          if (at + 144 > end) break;  // (the window's 16 bytes past the burst)
#pragma unroll
          for (int k = 0; k < 9; ++k) t[k] = q[k];
          if (rare_hit(f, t)) break;
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) t[k] = q[k];
          if (prefix_hit(f, t)) break;
        }
        at += 128;
        if (at + 128 > end) break;
      }
      if (at + 128 > end) break;
    }
    const uint4 *p = (const uint4 *)(base + at);
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p[k];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (!L.done) chunk16<MODE>(L, f, lds, v[k], at + 16 * k);
    at += 128;
  }
  while (!L.done && at + 16 <= end) {
    uint4 v = *(const uint4 *)(base + at);
    chunk16<MODE>(L, f, lds, v, at);
    at += 16;
  }
  while (!L.done && at < end) {
    step1<MODE>(L, f, lds, base[at], at);
    ++at;
  }
}

// Full forward scan of text[at..len] including the EOF step (dfa.rs:748-763).
template <int MODE, bool PFX = false>
__device__ __forceinline__ void fwd_run(LaneState &L, const FwdDfaDev &f, const uint8_t *lds, const uint8_t *base,
                                        uint64_t len, uint64_t at) {
  fwd_range<MODE, PFX>(L, f, lds, base, at, len);
  if (!L.done && f.eof[L.s]) L.last = len;
}

__device__ __forceinline__ void lane_start(LaneState &L, const FwdDfaDev &f, const uint8_t *base, uint64_t len,
                                           uint64_t at) {
  L.last = NONE;
  L.done = false;
  L.quit = false;
  L.fast = false;
  L.t = 0;
  if (at > len) {
    L.done = true;
    L.s = f.dead;
  } else {
    L.s = f.ustart1 ? f.ustart1 - 1 : f.start[fwd_flag_index(base, len, at)];
    if (L.s >= f.n_normal) L.done = true;  // dead start state (dfa.rs:484)
  }
}

// ExecNoSync::find_dfa_forward (exec.rs:632-662) for one lane: 0 = no
// match, 1 = match (ms, me), 2 = the DFA quit.
__device__ __forceinline__ int dfa_find(const FwdDfaDev &f, const RevDfaDev &r, const uint8_t *lds,
                                        const uint8_t *rlds, const uint8_t *base, uint64_t len, uint64_t at,
                                        uint64_t *ms, uint64_t *me) {
  LaneState L;
  lane_start(L, f, base, len, at);
  fwd_run<MODE_FIND>(L, f, lds, base, len, at);
  if (L.quit) return 2;
  if (L.last == NONE) return 0;
  *me = L.last;
  if (L.last == at) { *ms = at; return 1; }  // exec.rs:647
  const uint64_t rs = rev_scan(r, rlds, base, len, at, L.last);
  if (rs == QUITMARK) return 2;
  if (rs == NONE) return 0;  // exec.rs:656-660
  *ms = rs;
  return 1;
}

// dfa_find for a search that may not start a match at or after `cut`
// (at < cut): the state at cut - 1 is replaced by its copy without the `.*?`
// prefix (f.strip), so the scan stops once every match that started before
// the cut has been decided.  Used by the chunked find_iter: its result equals
// the unrestricted search whenever that search's match starts before the cut,
// and is "no match" otherwise.
// With look-around (f.looks): returns 3 when the reverse scan finds no start
// (exec.rs:656-660: the search's NoMatch, which ends the reference's
// iteration), and *reached (optional) says whether the answer may depend on
// the search start `at` (the reverse scan got to it alive, or the match is
// empty at it).
__device__ __forceinline__ int dfa_find_cut(const FwdDfaDev &f, const RevDfaDev &r, const uint8_t *lds,
                                            const uint8_t *rlds, const uint8_t *base, uint64_t len, uint64_t at,
                                            uint64_t cut, uint64_t *ms, uint64_t *me, bool *reached = nullptr) {
  LaneState L;
  lane_start(L, f, base, len, at);
  if (cut > at && cut - 1 <= len) {
    fwd_range<MODE_FIND>(L, f, lds, base, at, cut - 1);
    if (!L.done) {
      L.s = f.strip[L.s];
      if (L.s == f.dead) L.done = true;
    }
    fwd_range<MODE_FIND>(L, f, lds, base, cut - 1, len);
  } else {
    fwd_range<MODE_FIND>(L, f, lds, base, at, len);
  }
  if (!L.done && f.eof[L.s]) L.last = len;
  if (L.quit) return 2;
  if (L.last == NONE) return 0;
  *me = L.last;
  if (L.last == at) {
    if (reached) *reached = true;
    *ms = at;
    return 1;
  }
  const uint64_t rs = rev_scan(r, rlds, base, len, at, L.last, reached);
  if (rs == QUITMARK) return 2;
  if (rs == NONE) return f.looks ? 3 : 0;
  *ms = rs;
  return 1;
}

// Literal engine (find_iter pass 1 and find / is_match batches): the first
// literal, in leftmost-first priority order, that occurs at position i, or -1.
// The caller guarantees i + lit_k <= len (i below len + 1 - lit_minlen).
__device__ __forceinline__ int lit_verify(const FwdDfaDev &f, const uint8_t *lds, const uint8_t *base, uint64_t len,
                                          uint64_t i) {
  uint32_t key = 0;
  for (uint32_t j = 0; j < f.lit_k; ++j) key |= (uint32_t)base[i + j] << (8 * j);
  const uint32_t *keys = (const uint32_t *)(lds + kLitKeys);
  for (uint32_t x = 0; x < f.lit_n; ++x) {
    if (keys[x] != key) continue;
    const uint32_t ln = lds[kLitLens + x];
    if (i + ln > len) continue;
    const uint8_t *lb = lds + kLitBytes + x * kLitLen;
    uint32_t j = f.lit_k;
    while (j < ln && base[i + j] == lb[j]) ++j;
    if (j == ln) return (int)x;
  }
  return -1;
}


// Candidate starts of the 64 positions [a, a + 64) (a 16-byte aligned):
// bit j = the hash of the lit_k bytes at a + j is in the prefix bitmap (and,
// K8, the hash of bytes 4..7 in the second one).  Blocks at or past hi_blk
// read as zeros; each position is tested on its own, so the 64 LDS probes are
// independent (no dependent chain per byte).
template <bool K4, bool K8>
__device__ __forceinline__ uint64_t lit_cands64(uintptr_t a, uintptr_t hi_blk, const uint32_t *bitmap,
                                                const uint32_t *bitmap2, uint32_t kmask) {
  // 64 positions per step: 4 blocks and the first word after them
  uint32_t d[18];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (a + 16 * k < hi_blk) v = *(const uint4 *)(a + 16 * k);
    d[4 * k] = v.x;
    d[4 * k + 1] = v.y;
    d[4 * k + 2] = v.z;
    d[4 * k + 3] = v.w;
  }
  if (a + 64 < hi_blk) {
    const uint2 t2 = *(const uint2 *)(a + 64);
    d[16] = t2.x;
    d[17] = t2.y;
  } else {
    d[16] = d[17] = 0u;
  }
  uint32_t clo = 0, chi = 0;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const uint32_t w = (j & 3) ? __builtin_amdgcn_alignbyte(d[(j >> 2) + 1], d[j >> 2], j & 3) : d[j >> 2];
    const uint32_t hh = lit_hash(K4 ? w : (w & kmask));
    uint32_t bit = (bitmap[hh >> 5] >> (hh & 31)) & 1u;
    if (K8) {  // bytes 4..7 too: candidates of a small alphabet (DNA) stay rare
      const uint32_t w2 =
          (j & 3) ? __builtin_amdgcn_alignbyte(d[(j >> 2) + 2], d[(j >> 2) + 1], j & 3) : d[(j >> 2) + 1];
      const uint32_t h2 = lit_hash(w2);
      bit &= (bitmap2[h2 >> 5] >> (h2 & 31)) & 1u;
    }
    if (j < 32) clo |= bit << j;
    else chi |= bit << (j - 32);
  }
  return ((uint64_t)chi << 32) | clo;
}

}  // namespace rure_amd
