// Device side of the wavefront Pike VM (see nfa_scan.hip), shared with the
// find_iter kernels (iter_scan.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfa_scan.hpp"

namespace rure_amd {
namespace pike {
namespace {  // internal linkage: included by several kernel files

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
// nb: the byte the list's threads will step on (0x100 at the end of the
// text): a Bytes leaf that does not take it would die at that step, so it
// is not added (Match leaves always are) -- the order of the survivors, and
// so the leftmost-first priorities, are unchanged.  Inside a word of
// Unicode \w+ this keeps one or two threads of the class's hundreds of
// alternatives in the list instead of all of them.
__device__ uint32_t append_closure(const NfaDev &nf, uint32_t cid, uint32_t holds, uint64_t stv, uint32_t *stamp,
                                   uint32_t tag, uint32_t *lleaf, uint64_t *lst, uint32_t cnt, uint32_t nb) {
  if (nf.cl_info) {  // no entry can pass: skip the scan (uniform)
    const uint32_t *ci = nf.cl_info + (size_t)cid * 9;
    const uint32_t w = ci[8];
    const bool byte_ok = nb <= 0xFF && ((ci[nb >> 5] >> (nb & 31)) & 1u);
    if (((w & 0xFF) & ~holds) != 0 || (!(w & 0x100) && !byte_ok)) return cnt;
  }
  uint32_t o0 = nf.cl_off[cid], o1 = nf.cl_off[cid + 1];
  const uint2 *E = nf.entries;
  if (nf.cl_big && nb <= 0x100) {  // a big closure: only the next byte's bucket
    const uint32_t bi = nf.cl_big[cid];
    if (bi != 0xFFFFFFFFu) {
      const uint32_t *bo = nf.cl_boff + (size_t)bi * 258;
      o0 = bo[nb];
      o1 = bo[nb + 1];
      E = nf.cl_sub;
    }
  }
  const uint32_t lane = lane_id();
  for (uint32_t k0 = o0; k0 < o1; k0 += 64) {
    const uint32_t k = k0 + lane;
    bool pass = false;
    uint32_t leaf = 0;
    if (k < o1) {
      uint2 e = E[k];
      leaf = e.x;
      pass = ((e.y & 0xFF) & ~holds) == 0;
      uint32_t pv = e.y >> 8;
      while (pass && pv) {  // an earlier entry of the same leaf in this closure wins
        uint2 q = E[o0 + pv - 1];
        if (((q.y & 0xFF) & ~holds) == 0) pass = false;
        pv = q.y >> 8;
      }
      if (pass) {
        const uint32_t w0 = nf.leaves[3 * leaf];
        if ((w0 & 0xFF) == 0) pass = nb >= ((w0 >> 8) & 0xFF) && nb <= ((w0 >> 16) & 0xFF);
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
// cut (the chunked find_iter's unit end, > start): no thread starts at or
// after it, so the search ends once every thread that started before it has
// died or matched -- the unrestricted search's answer when that starts
// before the cut (an earlier start outranks every later one), else none.
template <int MODE>
__device__ void pike_one(const NfaDev &nf, Lists &W, TagGen &tg, const uint8_t *text, uint64_t len, uint64_t start,
                         uint64_t *r0, uint64_t *r1, uint64_t cut = ~0ull) {
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
    if (nc == 0 && ((matched && nf.single) || all_matched || (at != 0 && nf.anchored) || at >= cut)) break;
    if (at < cut && (nc == 0 || (!nf.anchored && !all_matched)))
      nc = append_closure(nf, nf.root, look_holds(text, len, at, nf), at, W.stamp, ctag, W.leaf[c], W.st[c], nc,
                          at < len ? text[at] : 0x100u);
    const uint32_t b = at < len ? text[at] : 0x100u;
    const uint32_t ntag = tg.next(W.stamp, nf.nleaves);
    const uint32_t hnx = at < len ? look_holds(text, len, at + 1, nf) : 0;
    const uint32_t nbx = at + 1 < len ? text[at + 1] : 0x100u;  // the next list's byte
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
        nn = append_closure(nf, cid, hnx, W.st[c][j0 + t], W.stamp, ntag, W.leaf[c ^ 1], W.st[c ^ 1], nn, nbx);
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

}  // namespace
}  // namespace pike
}  // namespace rure_amd
