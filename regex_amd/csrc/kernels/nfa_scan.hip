// Wavefront Pike VM for gfx950 (MI355X).
//
// Reference: src/pikevm.rs (exec_ 130-223, step 237-280, add 284-352) over
// the byte input of src/input.rs (ByteInput, is_empty_match 268-318) with
// the UTF-8 helpers of src/utf8.rs:83-175.  Used where the DFA cannot
// answer: patterns with a Unicode word boundary on non-ASCII input (the DFA
// quits, dfa.rs:1491-1496, and exec.rs falls back to the NFA) and automata
// too large to materialise.
//
// One wavefront runs one haystack.  The ordered thread list of the Pike VM
// lives in LDS (or per-wave global scratch for very large programs); the
// epsilon walk of `add` is replaced by the precomputed closures of
// host/nfa_build.cpp, and each closure is appended 64 entries at a time:
// every lane tests one entry (assertions hold at this position? leaf not yet
// in the list?), then __ballot + mbcnt give the survivors their slots in
// priority order.  Threads are stepped 64 at a time; the first Match thread
// (ballot + ffs) cuts all lower-priority threads, exactly as the reference's
// `break` after a match for single regexes (pikevm.rs:202-212).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfa_scan.hpp"

namespace rure_amd {

namespace {

constexpr uint64_t NONE = ~0ull;
constexpr uint64_t QUITMARK = ~0ull - 1;
constexpr uint32_t NO_CHAR = 0xFFFFFFFFu;

enum : uint32_t {
  LK_START_LINE = 1u << 0, LK_END_LINE = 1u << 1, LK_START_TEXT = 1u << 2, LK_END_TEXT = 1u << 3,
  LK_WB = 1u << 4, LK_NWB = 1u << 5, LK_WB_ASCII = 1u << 6, LK_NWB_ASCII = 1u << 7,
};

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// utf8.rs:83-150
__device__ uint32_t dec_utf8(const uint8_t *s, uint64_t n) {
  if (n == 0) return NO_CHAR;
  uint32_t b0 = s[0];
  if (b0 <= 0x7F) return b0;
  if (b0 >= 0xC0 && b0 <= 0xDF) {
    if (n < 2 || (s[1] & 0xC0) != 0x80) return NO_CHAR;
    uint32_t cp = ((b0 & 0x1F) << 6) | (s[1] & 0x3F);
    return (cp < 0x80 || cp > 0x7FF) ? NO_CHAR : cp;
  }
  if (b0 >= 0xE0 && b0 <= 0xEF) {
    if (n < 3 || (s[1] & 0xC0) != 0x80 || (s[2] & 0xC0) != 0x80) return NO_CHAR;
    uint32_t cp = ((b0 & 0x0F) << 12) | ((uint32_t)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
    return (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF)) ? NO_CHAR : cp;
  }
  if (b0 >= 0xF0 && b0 <= 0xF7) {
    if (n < 4 || (s[1] & 0xC0) != 0x80 || (s[2] & 0xC0) != 0x80 || (s[3] & 0xC0) != 0x80) return NO_CHAR;
    uint32_t cp = ((b0 & 0x07) << 18) | ((uint32_t)(s[1] & 0x3F) << 12) | ((uint32_t)(s[2] & 0x3F) << 6) |
                  (s[3] & 0x3F);
    return (cp < 0x10000 || cp > 0x10FFFF) ? NO_CHAR : cp;
  }
  return NO_CHAR;
}

__device__ __forceinline__ uint32_t utf8_len(uint32_t cp) {
  return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4;
}

// utf8.rs:154-175 on text[..n]
__device__ uint32_t dec_last_utf8(const uint8_t *s, uint64_t n) {
  if (n == 0) return NO_CHAR;
  uint64_t start = n - 1;
  if (s[start] <= 0x7F) return s[start];
  uint64_t lim = n >= 4 ? n - 4 : 0;
  while (start > lim) {
    start -= 1;
    if ((s[start] & 0xC0) != 0x80) break;
  }
  uint32_t cp = dec_utf8(s + start, n - start);
  if (cp == NO_CHAR) return NO_CHAR;
  if (utf8_len(cp) < n - start) return NO_CHAR;
  return cp;
}

__device__ __forceinline__ bool ascii_word(uint32_t c) {
  return c == '_' || (c - '0') < 10u || ((c | 0x20) - 'a') < 26u;
}

// regex-syntax lib.rs:1729-1744 (PERLW, Unicode 10)
__device__ bool unicode_word(uint32_t c, const NfaDev &nf) {
  if (c == NO_CHAR) return false;
  if (c < 0x80) return ascii_word(c);
  uint32_t lo = 0, hi = nf.perlw_n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (c < nf.perlw[2 * mid]) hi = mid;
    else if (c > nf.perlw[2 * mid + 1]) lo = mid + 1;
    else return true;
  }
  return false;
}

// Which assertions hold at `pos` of text[..len] (input.rs:268-318, bytes
// input: only_utf8 = false).
__device__ uint32_t look_holds(const uint8_t *t, uint64_t len, uint64_t pos, const NfaDev &nf) {
  if (nf.looks == 0) return 0;
  uint32_t h = 0;
  if (pos == 0 || t[pos - 1] == '\n') h |= LK_START_LINE;
  if (pos == len || t[pos] == '\n') h |= LK_END_LINE;
  if (pos == 0) h |= LK_START_TEXT;
  if (pos == len) h |= LK_END_TEXT;
  // ASCII word boundary: Char::is_word_byte of the decoded neighbours is
  // exactly "the adjacent byte is an ASCII word byte".
  bool ap = pos > 0 && ascii_word(t[pos - 1]);
  bool an = pos < len && ascii_word(t[pos]);
  h |= (ap != an) ? LK_WB_ASCII : LK_NWB_ASCII;
  if (nf.unicode_wb) {
    bool wp = unicode_word(dec_last_utf8(t, pos), nf);
    bool wn = unicode_word(pos < len ? dec_utf8(t + pos, len - pos) : NO_CHAR, nf);
    h |= (wp != wn) ? LK_WB : LK_NWB;
  }
  return h;
}

struct Lists {
  uint32_t *stamp;
  uint32_t *leaf[2];
  uint64_t *st[2];
};

// Appends closure `cid` (filtered by the assertions `holds`) to a thread
// list in priority order, skipping leaves already in it (stamp == tag).
__device__ uint32_t append_closure(const NfaDev &nf, uint32_t cid, uint32_t holds, uint64_t stv, uint32_t *stamp,
                                   uint32_t tag, uint32_t *lleaf, uint64_t *lst, uint32_t cnt) {
  const uint32_t o0 = nf.cl_off[cid], o1 = nf.cl_off[cid + 1];
  const uint32_t lane = lane_id();
  for (uint32_t k0 = o0; k0 < o1; k0 += 64) {
    const uint32_t k = k0 + lane;
    bool pass = false;
    uint32_t leaf = 0;
    if (k < o1) {
      uint2 e = nf.entries[k];
      leaf = e.x;
      pass = ((e.y & 0xFF) & ~holds) == 0;
      uint32_t pv = e.y >> 8;
      while (pass && pv) {  // an earlier entry of the same leaf in this closure wins
        uint2 q = nf.entries[o0 + pv - 1];
        if (((q.y & 0xFF) & ~holds) == 0) pass = false;
        pv = q.y >> 8;
      }
      if (pass) pass = stamp[leaf] != tag;
    }
    const uint64_t bal = __ballot(pass);
    if (pass) {
      const uint32_t pos = cnt + mbcnt(bal);
      stamp[leaf] = tag;
      lleaf[pos] = leaf;
      lst[pos] = stv;
    }
    cnt += (uint32_t)__popcll(bal);
    wave_sync();
  }
  return cnt;
}

struct TagGen {
  uint32_t tag = 0;
  __device__ uint32_t next(uint32_t *stamp, uint32_t nleaves) {
    if (tag >= 0xFFFFFFF0u) {  // wrap: forget every stamp
      for (uint32_t i = lane_id(); i < nleaves; i += 64) stamp[i] = 0xFFFFFFFFu;
      wave_sync();
      tag = 0;
    }
    return tag++;
  }
};

// pikevm.rs:130-223 for one haystack (wave-uniform control flow).
template <int MODE>
__device__ void pike_one(const NfaDev &nf, Lists &W, TagGen &tg, const uint8_t *text, uint64_t len, uint64_t start,
                         uint64_t *r0, uint64_t *r1) {
  const uint32_t lane = lane_id();
  uint64_t ms = NONE, me = NONE, mask = 0;
  bool matched = false, all_matched = false;
  const uint64_t full = nf.nmatch >= 64 ? ~0ull : ((1ull << nf.nmatch) - 1);
  if (start > len) {
    *r0 = NONE;
    *r1 = NONE;
    if (MODE == MODE_SET || MODE == MODE_ISMATCH) *r0 = 0;
    return;
  }
  int c = 0;
  uint32_t nc = 0, ctag = tg.next(W.stamp, nf.nleaves);
  uint64_t at = start;
  while (true) {
    if (nc == 0 && ((matched && nf.single) || all_matched || (at != 0 && nf.anchored))) break;
    if (nc == 0 || (!nf.anchored && !all_matched))
      nc = append_closure(nf, nf.root, look_holds(text, len, at, nf), at, W.stamp, ctag, W.leaf[c], W.st[c], nc);
    const uint32_t b = at < len ? text[at] : 0x100u;
    const uint32_t ntag = tg.next(W.stamp, nf.nleaves);
    const uint32_t hnx = at < len ? look_holds(text, len, at + 1, nf) : 0;
    uint32_t nn = 0;
    bool stop = false, quit_now = false;
    for (uint32_t j0 = 0; j0 < nc && !stop; j0 += 64) {
      const uint32_t j = j0 + lane;
      const bool valid = j < nc;
      uint32_t w0 = 0;
      if (valid) w0 = nf.leaves[3 * W.leaf[c][j]];
      const bool is_m = valid && (w0 & 0xFF) == 1;
      const uint32_t lo = (w0 >> 8) & 0xFF, hi = (w0 >> 16) & 0xFF;
      const bool acc = valid && (w0 & 0xFF) == 0 && b >= lo && b <= hi;
      const uint64_t mb = __ballot(is_m);
      uint64_t ab = __ballot(acc);
      if (mb) {
        if (MODE == MODE_SET) {
          uint64_t m = mb;
          while (m) {
            const uint32_t t = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t slot = nf.leaves[3 * W.leaf[c][j0 + t] + 2];
            if (slot < 64) mask |= 1ull << slot;
          }
          matched = true;
          if (!all_matched) all_matched = (mask & full) == full;
          if (nf.single) {  // one Match instruction: leftmost-first cut
            ab &= (1ull << __builtin_ctzll(mb)) - 1;
            stop = true;
          }
        } else {
          const uint32_t t = (uint32_t)__builtin_ctzll(mb);
          ms = W.st[c][j0 + t];
          me = at;
          matched = true;
          all_matched = true;
          if (MODE != MODE_FIND) { quit_now = true; break; }  // quit_after_match
          ab &= (1ull << t) - 1;  // pikevm.rs:202-212: lower-priority threads are cut
          stop = true;
        }
      }
      while (ab) {
        const uint32_t t = (uint32_t)__builtin_ctzll(ab);
        ab &= ab - 1;
        const uint32_t cid = nf.leaves[3 * W.leaf[c][j0 + t] + 1];
        nn = append_closure(nf, cid, hnx, W.st[c][j0 + t], W.stamp, ntag, W.leaf[c ^ 1], W.st[c ^ 1], nn);
      }
    }
    if (quit_now) break;
    if (at >= len) break;
    ++at;
    c ^= 1;
    nc = nn;
    ctag = ntag;
  }
  if (MODE == MODE_SET) { *r0 = mask; return; }
  if (MODE == MODE_ISMATCH) { *r0 = matched ? 1 : 0; return; }
  *r0 = ms;
  *r1 = me;
}

template <int MODE, bool FALLBACK, bool STRIDED>
__global__ __launch_bounds__(64) void pike_kernel(BatchDev bt, NfaDev nf, void *out, uint8_t *scratch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *mem = scratch ? scratch + (size_t)blockIdx.x * nfa_wave_bytes(nf.nleaves) : lds;
  Lists W;
  const uint32_t N = nf.nleaves;
  W.st[0] = (uint64_t *)mem;
  W.st[1] = W.st[0] + N;
  W.stamp = (uint32_t *)(W.st[1] + N);
  W.leaf[0] = W.stamp + N;
  W.leaf[1] = W.leaf[0] + N;
  const uint32_t lane = lane_id();
  for (uint32_t i = lane; i < N; i += 64) W.stamp[i] = 0xFFFFFFFFu;
  wave_sync();
  TagGen tg;
  for (uint64_t g = blockIdx.x; g * 64 < bt.count; g += gridDim.x) {
    const uint64_t hh = g * 64 + lane;
    bool need = hh < bt.count;
    if (need && FALLBACK) {
      if (MODE == MODE_FIND) need = ((const uint64_t *)out)[2 * hh] == QUITMARK;
      else if (MODE == MODE_ISMATCH) need = ((const uint8_t *)out)[hh] == 2;
      else need = ((const uint64_t *)out)[hh] == QUITMARK;
    }
    uint64_t todo = __ballot(need);
    while (todo) {
      const uint32_t t = (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1;
      const uint64_t h = g * 64 + t;
      const uint8_t *base;
      uint64_t len;
      if (STRIDED) {
        base = bt.hay + h * bt.stride;
        len = bt.length;
      } else {
        const uint64_t o0 = bt.offs[h], o1 = bt.offs[h + 1];
        base = bt.hay + o0;
        len = o1 - o0;
      }
      uint64_t r0 = NONE, r1 = NONE;
      pike_one<MODE>(nf, W, tg, base, len, bt.start, &r0, &r1);
      if (lane == 0) {
        if (MODE == MODE_FIND) {
          ((uint64_t *)out)[2 * h] = r0;
          ((uint64_t *)out)[2 * h + 1] = r1;
        } else if (MODE == MODE_ISMATCH) {
          ((uint8_t *)out)[h] = (uint8_t)r0;
        } else if (MODE == MODE_SHORTEST) {
          ((uint64_t *)out)[h] = r1;
        } else {
          ((uint64_t *)out)[h] = r0;
        }
      }
    }
  }
}

template <int MODE, bool FALLBACK>
hipError_t launch_m(const BatchDev &b, const NfaDev &n, void *out, void *scratch, hipStream_t st, int grid) {
  const size_t lds = scratch ? 0 : nfa_wave_bytes(n.nleaves);
  if (lds > 64 * 1024) {
    hipError_t e = b.offs ? hipFuncSetAttribute((const void *)pike_kernel<MODE, FALLBACK, false>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
                          : hipFuncSetAttribute((const void *)pike_kernel<MODE, FALLBACK, true>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (b.offs)
    hipLaunchKernelGGL((pike_kernel<MODE, FALLBACK, false>), dim3(grid), dim3(64), lds, st, b, n, out,
                       (uint8_t *)scratch);
  else
    hipLaunchKernelGGL((pike_kernel<MODE, FALLBACK, true>), dim3(grid), dim3(64), lds, st, b, n, out,
                       (uint8_t *)scratch);
  return hipGetLastError();
}

template <int MODE>
hipError_t launch_f(bool fallback, const BatchDev &b, const NfaDev &n, void *out, void *scratch, hipStream_t st,
                    int grid) {
  return fallback ? launch_m<MODE, true>(b, n, out, scratch, st, grid)
                  : launch_m<MODE, false>(b, n, out, scratch, st, grid);
}

}  // namespace

hipError_t launch_pike(int mode, bool fallback, const BatchDev &b, const NfaDev &n, void *out, void *scratch,
                       hipStream_t st, int grid) {
  switch (mode) {
    case MODE_FIND: return launch_f<MODE_FIND>(fallback, b, n, out, scratch, st, grid);
    case MODE_ISMATCH: return launch_f<MODE_ISMATCH>(fallback, b, n, out, scratch, st, grid);
    case MODE_SHORTEST: return launch_f<MODE_SHORTEST>(fallback, b, n, out, scratch, st, grid);
    default: return launch_f<MODE_SET>(fallback, b, n, out, scratch, st, grid);
  }
}

}  // namespace rure_amd
