// Batched replacen / split over device find_iter output (gfx950).
//
// Reference: bytes::Regex::replacen's literal path (re_bytes.rs:489-512: the
// text between matches is copied, each of the first `limit` matches becomes
// `rep`) and the Split / SplitN iterators (re_bytes.rs:699-749).  The matches
// come from the batched find_iter (iter_scan.hip), concatenated per haystack
// in order.
//
// replacen: a wave per haystack turns its matches into a layout (output
// length, and per match shift_j = bytes removed before match j minus j
// replacements), the lengths are prefix-summed, then every thread writes 16
// output bytes: it finds the last match whose replacement starts at or before
// its position (binary search on R_j = s_j - shift_j) and copies from the
// replacement or from the text after that match.  Balanced for any match
// density (the regex-dna strip pass removes 35 M short lines; the IUB
// substitutions touch a few bytes per 100 KB).
//
// split: the fields are the gaps between matches plus the tail, with the
// SplitN rule for a limit (its last field is the remainder of the text).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>
#include <rocprim/rocprim.hpp>
#include <stdint.h>

#include "dfa_scan.hpp"

namespace rure_amd {

namespace {

__device__ __forceinline__ void hay_of(const BatchDev &bt, uint64_t h, uint64_t *base, uint64_t *len) {
  if (bt.offs) {
    *base = bt.offs[h];
    *len = bt.offs[h + 1] - bt.offs[h];
  } else {
    *base = h * bt.stride;
    *len = bt.length;
  }
}

// First index i in [lo, hi) with a[i] > x (a non-decreasing).
__device__ __forceinline__ uint64_t upper_idx(const uint64_t *a, uint64_t lo, uint64_t hi, uint64_t x) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// The layout of replacen as a segmented scan over all matches of the batch
// (one thread per match, so a haystack with 35 M matches is as parallel as
// 35 M haystacks): val[g] = len(match g) - rep_len when g is among its
// haystack's first `limit` matches, else 0; S = exclusive scan of val over
// nm + 1 entries; shift[g] = S[g] - S[moff[h]] (bytes removed before match g
// minus its replacements so far, within haystack h) and out_len[h] = len_h -
// (S[moff[h] + k_h] - S[moff[h]]).
__global__ __launch_bounds__(256) void replace_vals_kernel(uint64_t n, const uint64_t *counts, const uint64_t *moff,
                                                           const uint64_t *m, uint64_t limit, uint64_t rep_len,
                                                           int64_t *val) {
  const uint64_t nm = moff[n];
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= nm; g += (uint64_t)gridDim.x * blockDim.x) {
    int64_t v = 0;
    if (g < nm) {
      const uint64_t h = upper_idx(moff, 0, n + 1, g) - 1;
      const uint64_t k = counts[h] < limit ? counts[h] : limit;
      if (g - moff[h] < k) v = (int64_t)(m[2 * g + 1] - m[2 * g]) - (int64_t)rep_len;
    }
    val[g] = v;
  }
}

__global__ __launch_bounds__(256) void replace_shift_kernel(BatchDev bt, const uint64_t *counts, const uint64_t *moff,
                                                            uint64_t limit, const int64_t *S, int64_t *shift,
                                                            uint64_t *out_len) {
  const uint64_t n = bt.count, nm = moff[n];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nm + n; g += stride) {
    if (g < nm) {
      const uint64_t h = upper_idx(moff, 0, n + 1, g) - 1;
      shift[g] = S[g] - S[moff[h]];
    } else {
      const uint64_t h = g - nm;
      uint64_t base, len;
      hay_of(bt, h, &base, &len);
      const uint64_t k = counts[h] < limit ? counts[h] : limit;
      out_len[h] = (uint64_t)((int64_t)len - (S[moff[h] + k] - S[moff[h]]));
    }
  }
}

// One haystack, every match replaced: the replacement starts G come
// straight out of one inclusive scan, G_0 = s_0 and G_j = G_(j-1) + s_j -
// e_(j-1) + rep_len (the text between two matches, then a replacement), read
// through GOne; with s_nm = the haystack length, G_nm is the output length.
// No shift array: the copy reads G as the replacement starts (CopyCtx::one).
struct GOne {
  const uint64_t *m, *offs;
  uint64_t nm, length;
  int64_t rep_len;
  __device__ int64_t operator()(uint64_t j) const {
    const int64_t s = j < nm ? (int64_t)m[2 * j] : (int64_t)(offs ? offs[1] - offs[0] : length);
    return j ? s - (int64_t)m[2 * j - 1] + rep_len : s;
  }
};

__global__ void replace_len1_kernel(const int64_t *G, uint64_t nm, uint64_t *out_len) {
  out_len[0] = (uint64_t)G[nm];
}

// 16 bytes from an arbitrary address, as two aligned 16-byte loads and a
// funnel shift (the second load is the aligned block holding p[15], so it
// stays inside the buffer's 16-byte-rounded end whenever p[0..16) does).
__device__ __forceinline__ uint4 load16u(const uint8_t *p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t off = (uint32_t)(a & 15);
  const uint4 x = *(const uint4 *)(a - off);
  if (off == 0) return x;
  const uint4 y = *(const uint4 *)(a - off + 16);
  const uint64_t w0 = ((uint64_t)x.y << 32) | x.x, w1 = ((uint64_t)x.w << 32) | x.z;
  const uint64_t w2 = ((uint64_t)y.y << 32) | y.x, w3 = ((uint64_t)y.w << 32) | y.z;
  uint64_t r0, r1;
  const uint32_t sh = off * 8;
  if (sh < 64) {
    r0 = (w0 >> sh) | (w1 << (64 - sh));
    r1 = (w1 >> sh) | (w2 << (64 - sh));
  } else if (sh == 64) {
    r0 = w1;
    r1 = w2;
  } else {
    const uint32_t s2 = sh - 64;
    r0 = (w1 >> s2) | (w2 << (64 - s2));
    r1 = (w2 >> s2) | (w3 << (64 - s2));
  }
  return make_uint4((uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32));
}

// replace_copy_kernel: a wave writes a 1 KiB window of the output per step,
// lane l its 16-byte block l (coalesced stores).  Every match's replacement
// start in global output coordinates (G, replace_index_kernel) is counted
// per window and the counts prefix-summed (widx[w] = matches with G below
// window w), so a lane searches only the few matches of its own window: a
// binary search over all matches per block or per window is a chain of ~25
// dependent loads (the kernel took 12-25 ms per regex-dna substitution).
constexpr uint32_t kWin = 1024;

__global__ __launch_bounds__(256) void replace_g_kernel(uint64_t n, const uint64_t *ooff, const uint64_t *moff,
                                                        const uint64_t *m, const int64_t *shift, uint64_t *G) {
  const uint64_t nm = moff[n];
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nm; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = n == 1 ? 0 : upper_idx(moff, 0, n + 1, g) - 1;
    G[g] = ooff[h] + (uint64_t)((int64_t)m[2 * g] - shift[g]);
  }
}

// widx[w] = the first match with G >= w * kWin (G is non-decreasing), for w
// in [0, nent): one independent binary search per window (a scatter from the
// matches would leave one thread to fill the windows of a long match-free
// stretch).
__global__ __launch_bounds__(256) void replace_widx_kernel(uint64_t n, const uint64_t *moff, const uint64_t *G,
                                                           uint64_t nent, uint64_t *widx) {
  const uint64_t nm = moff[n];
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nent; w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = w * kWin;
    uint64_t lo = 0, hi = nm;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (G[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    widx[w] = lo;
  }
}

// One output block at global position p0 (window w): the byte-by-byte
// path (a replacement edge, a haystack edge or the output end) or, when
// `fast`, one 16-byte load of the text.  Split in two so that the kernel can
// run four blocks' dependent load chains side by side.
struct CopyCtx {
  BatchDev bt;
  const uint64_t *ooff, *counts, *moff, *m, *G, *widx;
  const int64_t *shift;
  uint64_t limit, rep_len, total, cap;
  const uint8_t *rep;
  bool one;  // one haystack, every match replaced: G holds the replacement starts, no shift
  __device__ __forceinline__ uint64_t R(uint64_t j) const {
    return one ? G[j] : (uint64_t)((int64_t)m[2 * j] - shift[j]);
  }
};

struct BlockPlan {
  uint64_t h, jj, src;  // haystack, matches passed, text source (fast)
  bool fast;
};

__device__ __forceinline__ BlockPlan plan_block(const CopyCtx &c, uint64_t w, uint64_t p0) {
  BlockPlan b;
  uint64_t lo = c.widx[w], hi = c.widx[w + 1];
  while (lo < hi) {  // matches with G <= p0 among the window's few
    const uint64_t mid = (lo + hi) >> 1;
    if (c.G[mid] <= p0) lo = mid + 1;
    else hi = mid;
  }
  const uint64_t n = c.bt.count;
  b.h = n == 1 ? 0 : upper_idx(c.ooff, 0, n + 1, p0) - 1;
  const uint64_t hbeg = c.ooff[b.h], hend = c.ooff[b.h + 1];
  const uint64_t k = c.counts[b.h] < c.limit ? c.counts[b.h] : c.limit;
  const uint64_t m0 = c.moff[b.h];
  // matches of this haystack with R <= loc; only its first k are replaced
  // (matches past the limit keep their text: their G, still increasing,
  // counts above k and is clamped)
  uint64_t jj = lo > m0 ? lo - m0 : 0;
  b.jj = jj > k ? k : jj;
  const uint64_t loc = p0 - hbeg;
  b.fast = false;
  b.src = 0;
  if (p0 + 16 <= hend && p0 + 16 <= c.total) {
    const uint64_t nextR = b.jj < k ? c.R(m0 + b.jj) : ~0ull;
    const uint64_t r = b.jj ? c.R(m0 + b.jj - 1) : 0;
    if (loc + 16 <= nextR && (b.jj == 0 || loc - r >= c.rep_len)) {
      uint64_t base, len;
      hay_of(c.bt, b.h, &base, &len);
      b.src = base + (b.jj ? c.m[2 * (m0 + b.jj - 1) + 1] + (loc - r - c.rep_len) : loc);
      b.fast = true;
    }
  }
  return b;
}

// A block with replacement edges inside one haystack: the (at most four)
// matches it can touch are loaded together, then each byte's source address
// is computed on its own, so the 16 byte loads are independent (a walk per
// byte was a chain of three dependent loads per byte).  False: the generic
// walk must do it (a haystack or output edge, or more edges in the block).
__device__ __forceinline__ bool copy_block_edges(const CopyCtx &c, uint64_t p0, const BlockPlan &b, uint8_t *out) {
  const uint64_t hbeg = c.ooff[b.h], hend = c.ooff[b.h + 1];
  if (p0 + 16 > hend || p0 + 16 > c.total) return false;
  const uint64_t k = c.counts[b.h] < c.limit ? c.counts[b.h] : c.limit, m0 = c.moff[b.h];
  const uint64_t loc = p0 - hbeg;
  uint64_t base, len;
  hay_of(c.bt, b.h, &base, &len);
  // matches jj - 1 + t, t = 0..4: replacement starts and match ends
  uint64_t Rt[5], Et[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int64_t j = (int64_t)b.jj - 1 + t;
    const bool ok = j >= 0 && (uint64_t)j < k;
    Rt[t] = ok ? c.R(m0 + (uint64_t)j) : ~0ull;
    Et[t] = ok ? c.m[2 * (m0 + (uint64_t)j) + 1] : 0;
  }
  if (Rt[4] <= loc + 15) return false;  // more than three replacements start in the block
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint64_t lc = loc + i;
    const int idx = (Rt[1] <= lc) + (Rt[2] <= lc) + (Rt[3] <= lc);  // Rt[0] <= loc when jj > 0
    uint8_t ch;
    if (b.jj == 0 && idx == 0) {
      ch = c.bt.hay[base + lc];
    } else {
      // the last match passed is jj - 1 + idx, i.e. Rt[idx]
      const uint64_t rr = Rt[idx], off = lc - rr;
      ch = off < c.rep_len ? c.rep[off] : c.bt.hay[base + Et[idx] + (off - c.rep_len)];
    }
    w[i >> 2] |= (uint32_t)ch << (8 * (i & 3));
  }
  *(uint4 *)(out + p0) = make_uint4(w[0], w[1], w[2], w[3]);
  return true;
}

__device__ __noinline__ void copy_block_slow(const CopyCtx &c, uint64_t p0, const BlockPlan &b, uint8_t *out) {
  if (copy_block_edges(c, p0, b, out)) return;
  uint8_t v[16];
  uint64_t hh = b.h, he = c.ooff[b.h + 1], bb, ln;
  hay_of(c.bt, hh, &bb, &ln);
  uint64_t kk = c.counts[hh] < c.limit ? c.counts[hh] : c.limit, mm = c.moff[hh], j2 = b.jj;
  for (int i = 0; i < 16; ++i) {
    const uint64_t p = p0 + i;
    uint8_t ch = 0;
    if (p < c.total) {
      if (p >= he) {  // the next haystack (empty outputs skipped)
        while (p >= c.ooff[hh + 1]) ++hh;
        he = c.ooff[hh + 1];
        hay_of(c.bt, hh, &bb, &ln);
        kk = c.counts[hh] < c.limit ? c.counts[hh] : c.limit;
        mm = c.moff[hh];
        j2 = 0;
      }
      const uint64_t lc = p - c.ooff[hh];
      while (j2 < kk && c.R(mm + j2) <= lc) ++j2;
      if (j2 == 0) {
        ch = c.bt.hay[bb + lc];
      } else {
        const uint64_t j = mm + j2 - 1;
        const uint64_t rr = c.R(j);
        ch = lc - rr < c.rep_len ? c.rep[lc - rr] : c.bt.hay[bb + c.m[2 * j + 1] + (lc - rr - c.rep_len)];
      }
    }
    v[i] = ch;
  }
  if (p0 + 16 <= c.total) {
    uint4 x;
    x.x = v[0] | (v[1] << 8) | (v[2] << 16) | ((uint32_t)v[3] << 24);
    x.y = v[4] | (v[5] << 8) | (v[6] << 16) | ((uint32_t)v[7] << 24);
    x.z = v[8] | (v[9] << 8) | (v[10] << 16) | ((uint32_t)v[11] << 24);
    x.w = v[12] | (v[13] << 8) | (v[14] << 16) | ((uint32_t)v[15] << 24);
    *(uint4 *)(out + p0) = x;
  } else {
    for (int i = 0; i < 16 && p0 + i < c.total; ++i) out[p0 + i] = v[i];
  }
}

// A wave writes 4 KiB per step: lane l the 16-byte block l of each of four
// 1 KiB windows (coalesced stores), the four blocks' load chains (window
// index, its matches, the text) in flight together.
constexpr uint32_t kCopyILP = 4;

__global__ __launch_bounds__(256) void replace_copy_kernel(CopyCtx c, uint8_t *out) {
  const uint64_t n = c.bt.count;
  c.total = c.ooff[n] < c.cap ? c.ooff[n] : c.cap;
  const uint64_t nwin = (c.total + kWin - 1) / kWin;
  const uint64_t nsup = (nwin + kCopyILP - 1) / kCopyILP;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t sw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); sw < nsup; sw += nwaves) {
    BlockPlan b[kCopyILP];
    uint64_t p0[kCopyILP];
#pragma unroll
    for (uint32_t q = 0; q < kCopyILP; ++q) {
      const uint64_t w = sw * kCopyILP + q;
      p0[q] = w * kWin + 16 * (uint64_t)lane;
      if (w < nwin && p0[q] < c.total) b[q] = plan_block(c, w, p0[q]);
      else { b[q].fast = false; b[q].h = ~0ull; }
    }
    uint4 v[kCopyILP];
#pragma unroll
    for (uint32_t q = 0; q < kCopyILP; ++q)
      if (b[q].fast) v[q] = load16u(c.bt.hay + b[q].src);
#pragma unroll
    for (uint32_t q = 0; q < kCopyILP; ++q) {
      if (b[q].fast) *(uint4 *)(out + p0[q]) = v[q];
      else if (b[q].h != ~0ull) copy_block_slow(c, p0[q], b[q], out);
    }
  }
}

// A copy moving 1 KiB per wave per round (round 4's replace_copy1_kernel,
// deleted in round 5) ran the per-byte path of the blocks that hold a
// replacement edge for the whole wave: nearly every
// 1 KiB window of the regex-dna strip (an edge every ~61 bytes) or of an IUB
// substitution holds one, so the path ran for the whole wave with a few
// lanes active — 3.7 G VALU instructions per strip pass, 4.9-5.6 ms
// (profiles/r05_replace_pmc.txt).  Here a wave takes kGroupWin windows
// (4 KiB of output) per round with one staging of the group's matches in
// LDS, copies the blocks that lie in one text stretch (two aligned loads and
// a funnel shift, all four windows' loads in flight together), and gathers
// the group's edge blocks into an LDS list that the whole wave then works
// through, every lane busy (no global atomics: a single edge list counter
// for the grid serialised the waves, 25 ms).
constexpr uint32_t kGroupWin = 4, kGroupSlots = 128;

// 16 bytes from any address without a branch: both aligned blocks are always
// loaded (the second is the first again when p is aligned, so nothing past
// the block holding p[15] is read), then a funnel shift by 8 * (p & 15) bits.
__device__ __forceinline__ uint4 load16u_nb(const uint8_t *p) {
  const uint32_t off = (uint32_t)((uintptr_t)p & 15);
  const uint8_t *a0 = p - off;  // (pointer arithmetic keeps the global address space)
  const uint4 x = *(const uint4 *)a0;
  const uint4 y = *(const uint4 *)(a0 + (off ? 16 : 0));
  const uint64_t w0 = ((uint64_t)x.y << 32) | x.x, w1 = ((uint64_t)x.w << 32) | x.z;
  const uint64_t w2 = ((uint64_t)y.y << 32) | y.x, w3 = ((uint64_t)y.w << 32) | y.z;
  const bool hi = off >= 8;
  const uint64_t u0 = hi ? w1 : w0, u1 = hi ? w2 : w1, u2 = hi ? w3 : w2;
  const uint32_t sh = (off & 7) * 8;
  const uint64_t r0 = sh ? (u0 >> sh) | (u1 << (64 - sh)) : u0;
  const uint64_t r1 = sh ? (u1 >> sh) | (u2 << (64 - sh)) : u1;
  return make_uint4((uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32));
}

// Blocks the group cannot do with its staged records (a dense group, a block
// with more than three replacement starts: rare) go to a global list, done
// by replace_rest_kernel through the generic per-block path (plan_block,
// copy_block_slow: a function call would hold ~140 VGPRs in this kernel);
// past the list's capacity replace_rest_kernel redoes the whole output.
__device__ __forceinline__ void push_rest(uint32_t *rest, uint64_t rest_cap, unsigned long long *nrest, uint64_t p0) {
  const unsigned long long k = atomicAdd(nrest, 1ull);
  if (k < rest_cap) rest[k] = (uint32_t)(p0 >> 4);
}

__global__ __launch_bounds__(256, 5) void replace_copy4_kernel(CopyCtx c, uint8_t *out, uint32_t *rest, uint64_t rest_cap,
                                                            unsigned long long *nrest) {
  __shared__ uint64_t sR[4][kGroupSlots], sE[4][kGroupSlots];
  __shared__ uint16_t sEdge[4][kGroupWin * 64];
  __shared__ uint32_t sA[4][kGroupWin * 64];  // per block of the group: its matches with R <= the block start
  const uint64_t total = c.ooff[1] < c.cap ? c.ooff[1] : c.cap;
  c.total = total;
  const uint64_t nm = c.moff[1];
  const uint64_t nwin = (total + kWin - 1) / kWin;
  const uint64_t ngrp = (nwin + kGroupWin - 1) / kGroupWin;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t base, len;
  hay_of(c.bt, 0, &base, &len);
  const uint8_t *hay = c.bt.hay + base;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  // widx has nwin + 2 entries: windows past the end clamp to the last one
  auto wx = [&](uint64_t w) { return c.widx[w < nwin ? w : nwin]; };
  uint64_t grp = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  uint64_t lo = wx(grp * kGroupWin), hi = wx(grp * kGroupWin + kGroupWin);
  for (; grp < ngrp; grp += nwaves) {
    const uint64_t w0 = grp * kGroupWin;
    const uint64_t cnt = hi - lo;
    // the next group's window index, a round ahead
    const uint64_t lo_n = wx((grp + nwaves) * kGroupWin), hi_n = wx((grp + nwaves) * kGroupWin + kGroupWin);
    if (cnt + 5 > kGroupSlots) {  // dense group: the generic per-block path
#pragma unroll 1
      for (uint32_t q = 0; q < kGroupWin; ++q) {
        const uint64_t p0 = (w0 + q) * kWin + 16 * (uint64_t)lane;
        if (w0 + q < nwin && p0 < total) push_rest(rest, rest_cap, nrest, p0);
      }
      lo = lo_n;
      hi = hi_n;
      continue;
    }
    const uint64_t *R = sR[wv], *E = sE[wv];
    uint32_t *A = sA[wv];
    const uint64_t gs = w0 * kWin;
#pragma unroll
    for (uint32_t q = 0; q < kGroupWin; ++q) A[64 * q + lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (uint32_t s = lane; s < kGroupSlots; s += 64) {  // slot s = match lo - 1 + s
      const int64_t g = (int64_t)lo - 1 + (int64_t)s;
      const bool ok = g >= 0 && (uint64_t)g < nm && s < cnt + 5;
      const uint64_t Rg = ok ? c.G[g] : ~0ull;
      sR[wv][s] = Rg;
      sE[wv][s] = ok ? c.m[2 * g + 1] : 0;
      // the group's matches by the first block whose start is >= R
      // (R >= gs; the last bucket, past the group, is not counted)
      if (s >= 1 && s <= cnt) {
        const uint64_t bk = (Rg - gs + 15) >> 4;
        if (bk < kGroupWin * 64) atomicAdd(&A[bk], 1u);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {  // inclusive prefix over the group's blocks (lane: blocks 4 lane .. 4 lane + 3)
      const uint4 a4 = *(const uint4 *)(A + 4 * lane);
      const uint32_t t = a4.x + a4.y + a4.z + a4.w;
      uint32_t ex = t;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(ex, o);
        if (lane >= (uint32_t)o) ex += x;
      }
      ex -= t;
      *(uint4 *)(A + 4 * lane) = make_uint4(ex + a4.x, ex + a4.x + a4.y, ex + a4.x + a4.y + a4.z, ex + t);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint4 v[kGroupWin];
    uint32_t fastm = 0;
#pragma unroll
    for (uint32_t q = 0; q < kGroupWin; ++q) {
      const uint64_t p0 = (w0 + q) * kWin + 16 * (uint64_t)lane;
      const uint32_t a = A[64 * q + lane];
      const uint64_t jj = lo + a;
      const uint64_t nextR = R[a + 1];
      const uint64_t r = jj ? R[a] : 0;
      const bool fast = p0 + 16 <= total && p0 + 16 <= nextR && (jj == 0 || p0 - r >= c.rep_len);
      const uint64_t src = fast ? (jj ? E[a] + (p0 - r - c.rep_len) : p0) : 0;
      v[q] = load16u_nb(hay + src);
      fastm |= fast ? 1u << q : 0u;
    }
    // the group's other blocks (inside the output) onto the wave's LDS list
    uint32_t ne = 0;
#pragma unroll
    for (uint32_t q = 0; q < kGroupWin; ++q) {
      const uint64_t p0 = (w0 + q) * kWin + 16 * (uint64_t)lane;
      if (fastm >> q & 1) *(uint4 *)(out + p0) = v[q];
      const bool edge = !(fastm >> q & 1) && p0 < total;
      const uint64_t m = __ballot(edge);
      if (edge) sEdge[wv][ne + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)(64 * q + lane);
      ne += (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
    for (uint32_t r0 = 0; r0 < ne; r0 += 64) {
      if (r0 + lane >= ne) continue;
      const uint32_t id = sEdge[wv][r0 + lane];
      const uint64_t p0 = (w0 + (id >> 6)) * kWin + 16 * (uint64_t)(id & 63);
      const uint32_t a = A[id];
      const uint64_t jj = lo + a;
      // deletions (rep_len 0, the regex-dna strip: an edge every ~61 bytes):
      // the block is at most four text stretches, each one unaligned 16-byte
      // load at the source of the block's byte 0 had the stretch covered it,
      // merged by byte masks — 8 aligned loads and ~30 VALU instead of 16
      // dependent-free byte loads and their selects
      if (c.rep_len == 0 && p0 + 16 <= total && R[a + 4] > p0 + 15) {
        int64_t bs[4];
        uint32_t k[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint64_t Rq = R[a + q];
          const bool in = q == 0 || Rq <= p0 + 15;  // the stretch after match a + q starts in the block
          k[q] = q == 0 ? 0u : in ? (uint32_t)(Rq - p0) : 16u;
          bs[q] = q == 0 && jj == 0 ? (int64_t)p0 : in ? (int64_t)(E[a + q] - Rq + p0) : (int64_t)p0;
        }
        if (bs[0] >= 0 && bs[1] >= 0 && bs[2] >= 0 && bs[3] >= 0) {
          uint4 t[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) t[q] = load16u_nb(hay + bs[q]);
          uint32_t x[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            uint32_t r = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const uint32_t word = d == 0 ? t[q].x : d == 1 ? t[q].y : d == 2 ? t[q].z : t[q].w;
              // bytes of dword d at or after k[q] (the later stretches overwrite)
              const int lo = (int)k[q] - 4 * d;
              const uint32_t ge = lo <= 0 ? 0xFFFFFFFFu : lo >= 4 ? 0u : 0xFFFFFFFFu << (8 * lo);
              r = (r & ~ge) | (word & ge);
            }
            x[d] = r;
          }
          *(uint4 *)(out + p0) = make_uint4(x[0], x[1], x[2], x[3]);
          continue;
        }
      }
      if (p0 + 16 <= total && R[a + 4] > p0 + 15) {
        // at most three replacement starts in the block: each byte's source
        // from the staged records, the 16 byte loads independent
        const uint64_t R0 = R[a], R1 = R[a + 1], R2 = R[a + 2], R3 = R[a + 3];
        const uint64_t E0 = E[a], E1 = E[a + 1], E2 = E[a + 2], E3 = E[a + 3];
        uint32_t x[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint64_t lc = p0 + i;
          const uint32_t idx = (R1 <= lc) + (R2 <= lc) + (R3 <= lc);
          uint8_t ch;
          if (jj == 0 && idx == 0) {
            ch = hay[lc];
          } else {
            const uint64_t rr = idx == 0 ? R0 : idx == 1 ? R1 : idx == 2 ? R2 : R3;
            const uint64_t ee = idx == 0 ? E0 : idx == 1 ? E1 : idx == 2 ? E2 : E3;
            const uint64_t off = lc - rr;
            ch = off < c.rep_len ? c.rep[off] : hay[ee + (off - c.rep_len)];
          }
          x[i >> 2] |= (uint32_t)ch << (8 * (i & 3));
        }
        *(uint4 *)(out + p0) = make_uint4(x[0], x[1], x[2], x[3]);
      } else {
        push_rest(rest, rest_cap, nrest, p0);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    lo = lo_n;
    hi = hi_n;
  }
}

__global__ __launch_bounds__(256) void replace_rest_kernel(CopyCtx c, uint8_t *out, const uint32_t *rest,
                                                           uint64_t rest_cap, const unsigned long long *nrest) {
  c.total = c.ooff[1] < c.cap ? c.ooff[1] : c.cap;
  const uint64_t n = *nrest;
  const bool all = n > rest_cap;  // the list overflowed: every block
  const uint64_t cnt = all ? (c.total + 15) / 16 : n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t p0 = all ? i << 4 : (uint64_t)rest[i] << 4;
    const BlockPlan b = plan_block(c, p0 / kWin, p0);
    if (b.fast) *(uint4 *)(out + p0) = load16u(c.bt.hay + b.src);
    else copy_block_slow(c, p0, b, out);
  }
}

// SplitN (re_bytes.rs:699-749): with m = k matches + (tail non-empty), a limit
// of `lim` fields gives all m fields when lim - 1 > m, else lim - 1 fields and
// the remainder of the text after them.
__device__ __forceinline__ uint64_t split_fields(uint64_t k, uint64_t lastend, uint64_t len, uint64_t lim) {
  const uint64_t mm = k + (lastend < len ? 1 : 0);
  if (lim == 0) return 0;
  if (lim - 1 > mm) return mm;
  return lim;
}

__global__ __launch_bounds__(256) void split_count_kernel(BatchDev bt, const uint64_t *counts, const uint64_t *moff,
                                                          const uint64_t *m, uint64_t lim, uint64_t *fields) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < bt.count;
       h += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t base, len;
    hay_of(bt, h, &base, &len);
    const uint64_t k = counts[h];
    const uint64_t lastend = k ? m[2 * (moff[h] + k - 1) + 1] : 0;
    fields[h] = split_fields(k, lastend, len, lim);
  }
}

// Fields from matches: field i of haystack h = [e_{i-1} (0 for i = 0), s_i)
// for i < min(k, lim - 1); the final field (tail or remainder) per haystack.
__global__ __launch_bounds__(256) void split_emit_kernel(BatchDev bt, const uint64_t *counts, const uint64_t *moff,
                                                         const uint64_t *m, uint64_t lim, const uint64_t *foff,
                                                         uint64_t *pieces, uint64_t cap) {
  const uint64_t n = bt.count;
  const uint64_t nm = moff[n];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nm + n; g += stride) {
    if (g < nm) {
      const uint64_t h = upper_idx(moff, 0, n + 1, g) - 1;
      const uint64_t i = g - moff[h];
      if (lim == 0 || i >= lim - 1) continue;  // consumed by the remainder field
      const uint64_t o = foff[h] + i;
      if (o < cap) {
        pieces[2 * o] = i == 0 ? 0 : m[2 * (g - 1) + 1];
        pieces[2 * o + 1] = m[2 * g];
      }
    } else {
      const uint64_t h = g - nm;
      uint64_t base, len;
      hay_of(bt, h, &base, &len);
      const uint64_t k = counts[h];
      const uint64_t lastend = k ? m[2 * (moff[h] + k - 1) + 1] : 0;
      const uint64_t nf = split_fields(k, lastend, len, lim);
      if (nf == 0) continue;
      const uint64_t mm = k + (lastend < len ? 1 : 0);
      uint64_t a, e = len;
      if (lim - 1 > mm) {         // plain split: the tail field, if any
        if (lastend >= len) continue;
        a = lastend;
      } else {                    // the SplitN remainder after lim - 1 fields
        const uint64_t used = lim - 1;
        if (used == 0) a = 0;
        else if (used <= k) a = m[2 * (moff[h] + used - 1) + 1];
        else {                    // the tail was a field of its own: then an empty remainder
          a = len;
          const uint64_t ot = foff[h] + k;
          if (ot < cap) {
            pieces[2 * ot] = lastend;
            pieces[2 * ot + 1] = len;
          }
        }
      }
      const uint64_t o = foff[h] + nf - 1;
      if (o < cap) {
        pieces[2 * o] = a;
        pieces[2 * o + 1] = e;
      }
    }
  }
}

int grid_for_items(uint64_t items, int threads, int cus) {
  uint64_t g = (items + threads - 1) / threads;
  const uint64_t cap = (uint64_t)cus * 8;
  if (g > cap) g = cap;
  return (int)(g < 1 ? 1 : g);
}


// ---------------------------------------------- one byte class, replace_all
// A regex whose every match is one byte of a class C (`B`, `[KM]`; host
// class_replace_set) has as find_iter the positions of the C bytes, so its
// replace_all needs no match list: the output of input unit u (kClsUnit bytes)
// starts at u kClsUnit + (L - 1) (C bytes before the unit), a prefix sum of
// per-unit counts.  Pass 1 counts; pass 2 (a wave per unit) stages the unit's
// bytes and per-lane layout in LDS and writes the unit's output range: the
// 16-byte blocks inside it from LDS (a block in a stretch without a
// replacement is one unaligned 16-byte read of the staged text), the partial
// blocks at its two edges byte by byte (they share an aligned block with the
// neighbouring units' edges: byte stores do not race).
constexpr uint32_t kClsUnit = 4096;  // bytes per unit: 64 lanes x 64
constexpr uint32_t kClsSlow = 256;   // a wave's list of blocks that meet a replacement

// bit 7 of each byte of w equal to the byte of rep (rep = byte * 0x01010101;
// exact: no borrow between bytes)
__device__ __forceinline__ uint32_t eq_bytes(uint32_t w, uint32_t rep) {
  const uint32_t x = w ^ rep;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

// sw1 / sw2: a class of at most two bytes as repeated bytes (sw1 = 0: use the
// table): four bytes' bits per SWAR compare instead of a table read per byte
__device__ __forceinline__ uint64_t cls_mask(const uint8_t *cls, const uint4 *v, uint32_t avail, uint32_t sw1,
                                             uint32_t sw2) {
  if (sw1) {
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t z = (eq_bytes(w[d], sw1) | eq_bytes(w[d], sw2)) >> 7;  // bits 0, 8, 16, 24
        m |= (uint64_t)((z * 0x01020408u) >> 24 & 0xFu) << (16 * j + 4 * d);
      }
    }
    return avail >= 64 ? m : m & ((1ull << avail) - 1ull);
  }
  uint64_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t pos = 16 * j + i;
      const uint32_t c = cls[(w[i >> 2] >> (8 * (i & 3))) & 0xFF];
      m |= (uint64_t)(pos < avail ? c : 0u) << pos;
    }
  }
  return m;
}

// (loads without a branch: absent blocks re-read the haystack's first block
// and are masked off by avail in cls_mask, so a prefetch's loads stay in
// flight past this call)
__device__ __forceinline__ void cls_load(const uint8_t *hay, uint64_t n, uint64_t s0, uint4 *v, uint32_t *avail) {
  const uint64_t a = s0 < n ? n - s0 : 0;
  *avail = a > 64 ? 64u : (uint32_t)a;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = *(const uint4 *)(16u * j < *avail ? hay + s0 + 16 * j : hay);
}

// Coalesced: lane l loads the unit's 16-byte pieces l, l + 64, l + 128,
// l + 192 (each load instruction one contiguous KiB of the wave).  *avail =
// the unit's bytes (<= kClsUnit).
__device__ __forceinline__ void cls_load_co(const uint8_t *hay, uint64_t n, uint64_t u, uint32_t lane, uint4 *v,
                                            uint32_t *avail) {
  const uint64_t s0 = u * kClsUnit;
  const uint64_t a = s0 < n ? n - s0 : 0;
  *avail = a > kClsUnit ? kClsUnit : (uint32_t)a;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t o = 16 * lane + 1024 * j;
    v[j] = *(const uint4 *)(o < *avail ? hay + s0 + o : hay);
  }
}

// The class bytes of a unit loaded by cls_load_co (wave total).
__device__ __forceinline__ uint32_t cls_count_co(const uint8_t *cls, const uint4 *v, uint32_t ua, uint32_t lane,
                                                 uint32_t sw1, uint32_t sw2) {
  uint64_t m = cls_mask(cls, v, 64, sw1, sw2);
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // the pieces' bytes past the haystack
    const uint32_t o = 16 * lane + 1024 * j;
    const uint32_t a = o < ua ? min(ua - o, 16u) : 0u;
    m &= ~(((0xFFFFull << a) & 0xFFFFull) << (16 * j));
  }
  uint32_t k = (uint32_t)__popcll(m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o);
  return k;
}

__global__ __launch_bounds__(256) void replace_cls_count_kernel(const uint8_t *hay, uint64_t n, const uint8_t *cls_g,
                                                                uint64_t nunits, uint64_t *ucount, uint32_t sw1,
                                                                uint32_t sw2, const uint64_t *n_dev) {
  __shared__ uint8_t cls[256];
  cls[threadIdx.x] = cls_g[threadIdx.x];
  __syncthreads();
  if (n_dev) {  // chained calls: the length on the device (n, nunits: upper bounds; units past it count 0)
    n = *n_dev;
    nunits = min(nunits, max<uint64_t>(1, (n + kClsUnit - 1) / kClsUnit));
  }
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  // last unit first: the tail of the text is what the previous pass wrote
  // last (still in the last-level cache), and the head this pass reads last
  // is what the write pass reads first
  // (two units per round: both units' loads in flight together)
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < nunits; i += 2 * nw) {
    const uint64_t u0 = nunits - 1 - i, u1 = i + nw < nunits ? nunits - 1 - (i + nw) : nunits;
    uint4 v0[4], v1[4];
    uint32_t a0, a1;
    cls_load_co(hay, n, u0, lane, v0, &a0);
    cls_load_co(hay, n, u1, lane, v1, &a1);
    const uint32_t k0 = cls_count_co(cls, v0, a0, lane, sw1, sw2), k1 = cls_count_co(cls, v1, a1, lane, sw1, sw2);
    if (lane == 0) {
      ucount[u0] = k0;
      if (u1 < nunits) ucount[u1] = k1;
    }
  }
}

// total (device) = the output length; out_offsets = {0, total} (either may
// be null); n_dev (chained calls): the input length on the device
__global__ void replace_cls_total_kernel(uint64_t n, uint64_t rep_len, const uint64_t *uoff, uint64_t nunits,
                                         uint64_t *ooff, uint64_t *total, const uint64_t *n_dev) {
  if (n_dev) n = *n_dev;
  const uint64_t t = n + uoff[nunits] * rep_len - uoff[nunits];
  if (!ooff) {
    *total = t;
    return;
  }
  ooff[0] = 0;
  ooff[1] = t;
  *total = t;
}

// The staged text is swizzled: the 16-byte piece j of lane c's 64 bytes sits
// in slot (j + c / 4) % 4, so that a quarter wave's 16-byte stores (and the
// fast path's reads) fall on distinct banks.  tx: logical -> LDS offset.
__device__ __forceinline__ uint32_t tx(uint32_t o) {
  return (o & ~63u) | ((((o >> 4) + (o >> 8)) & 3u) << 4) | (o & 15u);
}

// The output byte at unit-relative output position r (< the unit's output
// length): lane x = the lane whose output chunk holds it (rel[x] <= r), then
// within its 64 input bytes the replacement or text byte (its C bytes in
// ascending order: at most a few).
__device__ __forceinline__ uint8_t cls_out_byte(uint32_t r, const uint32_t *rel, const uint64_t *msk,
                                                const uint8_t *txt, const uint8_t *rep, uint32_t L) {
  uint32_t x = min(r >> 6, 63u);
  while (x > 0 && rel[x] > r) --x;
  uint32_t p = r - rel[x];
  uint64_t m = msk[x];
  uint32_t cnt = 0;
  while (m) {
    const uint32_t c = (uint32_t)__builtin_ctzll(m);
    m &= m - 1;
    const uint32_t oc = c + (L - 1) * cnt;  // the output offset of C byte c in the chunk
    if (oc > p) break;
    if (p < oc + L) return rep[p - oc];
    ++cnt;
  }
  return txt[tx(64 * x + p - (L - 1) * cnt)];
}

// 16 bytes of the staged text from logical offset o (o + 16 <= kClsUnit +
// 16: the stage has 16 spare bytes, in no swizzled piece)
__device__ __forceinline__ uint4 lds16u(const uint8_t *txt, uint32_t o) {
  const uint32_t d = o & ~3u, sh = 8 * (o & 3);
  const uint32_t a = *(const uint32_t *)(txt + tx(d)), b = *(const uint32_t *)(txt + tx(d + 4)),
                 c = *(const uint32_t *)(txt + tx(d + 8)), e = *(const uint32_t *)(txt + tx(d + 12)),
                 f = *(const uint32_t *)(txt + tx(d + 16));
  return make_uint4(__builtin_amdgcn_alignbit(b, a, sh), __builtin_amdgcn_alignbit(c, b, sh),
                    __builtin_amdgcn_alignbit(e, c, sh), __builtin_amdgcn_alignbit(f, e, sh));
}

// The 16 output bytes from unit-relative output position r with a running
// state (the lane chunk, its C bytes passed), for blocks that meet a
// replacement: ~10 VALU per byte instead of a search per byte.
__device__ __forceinline__ uint4 cls_block_slow(uint32_t r, uint32_t T, const uint32_t *rel, const uint64_t *msk,
                                                const uint8_t *txt, const uint8_t *rep, uint32_t L) {
  uint32_t x = min(r >> 6, 63u);
  while (x > 0 && rel[x] > r) --x;
  uint32_t p = r - rel[x], lenx = rel[x + 1] - rel[x], cnt = 0;
  uint64_t m = msk[x];
  // next C byte of the chunk and its output offset (none: past the chunk)
  uint32_t cn = m ? (uint32_t)__builtin_ctzll(m) : 64u, ocn = cn;
  uint32_t b[4] = {0, 0, 0, 0};
#pragma unroll 1
  for (uint32_t j = 0; j < 16 && r + j < T; ++j) {
    while (p >= lenx) {  // into the next lane's chunk
      p -= lenx;
      ++x;
      lenx = rel[x + 1] - rel[x];
      m = msk[x];
      cnt = 0;
      cn = m ? (uint32_t)__builtin_ctzll(m) : 64u;
      ocn = cn;
    }
    while (m && p >= ocn + L) {  // past C byte cn's replacement
      m &= m - 1;
      ++cnt;
      cn = m ? (uint32_t)__builtin_ctzll(m) : 64u;
      ocn = cn + (L - 1) * cnt;
    }
    const uint32_t ch = (m && p >= ocn) ? rep[p - ocn] : txt[tx(64 * x + p - (L - 1) * cnt)];
    b[j >> 2] |= ch << (8 * (j & 3));
    ++p;
  }
  return make_uint4(b[0], b[1], b[2], b[3]);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A unit whose output spans at most kClsMap bytes from the aligned block
// before it and holds at most kClsRank C bytes gets a block map: the output
// offset of every replacement (P, by rank) and per 16-byte output block the
// replacements starting before it (prefix of counts).  A block with no
// replacement starting in it and the one before it ended is text only, read
// from staged offset (block start - (L - 1) * replacements before it); a
// block a replacement meets walks P from there byte by byte.
constexpr uint32_t kClsMap = 6144;
constexpr uint32_t kClsRank = 256;
#ifndef CLS_WAVES
#define CLS_WAVES 5
#endif
constexpr uint32_t kClsCW = kClsMap / 32 / 64;  // a lane's words of the count map
static_assert(kClsMap % 2048 == 0, "the map is worked by whole lanes");

// The 16 output bytes of block x0 (offset from the unit's aligned output
// base) with c0 replacements starting before it.
__device__ __forceinline__ uint4 cls_block_map(uint32_t x0, uint32_t c0, uint32_t K, const uint16_t *P, uint32_t o15,
                                               const uint8_t *txt, const uint8_t *rep, uint32_t L) {
  int idx = (int)c0 - 1;  // the last replacement starting at or before the byte
  uint32_t cur = idx >= 0 ? P[idx] : 0u, nxt = c0 < K ? P[c0] : ~0u;
  uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
#pragma unroll 1
  for (uint32_t j0 = 0; j0 < 16; j0 += 4) {  // a word per round, shifted in from the top
    uint32_t w = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t x = x0 + j0 + j;
      if (x >= nxt) {
        ++idx;
        cur = nxt;
        nxt = (uint32_t)(idx + 1) < K ? P[idx + 1] : ~0u;
      }
      const uint32_t ch =
          (idx >= 0 && x - cur < L) ? rep[x - cur] : txt[tx(x - o15 - (L - 1) * (uint32_t)(idx + 1))];
      w |= ch << (8 * j);
    }
    b0 = b1;
    b1 = b2;
    b2 = b3;
    b3 = w;
  }
  return make_uint4(b0, b1, b2, b3);
}

// The next substitution's class bytes (at most two byte values as SWAR
// compares, s1 != 0) among a lane's staged bytes, as a 64-bit mask (bytes
// past avail: none).
__device__ __forceinline__ uint64_t next_mask(const uint4 *v, uint32_t avail, uint32_t s1, uint32_t s2) {
  uint64_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t z = (eq_bytes(w[d], s1) | eq_bytes(w[d], s2)) >> 7;  // bits 0, 8, 16, 24
      m |= (uint64_t)((z * 0x01020408u) >> 24 & 0xFu) << (16 * j + 4 * d);
    }
  }
  return avail >= 64 ? m : m & ((1ull << avail) - 1ull);
}

struct ClsWave {
  uint8_t txt[kClsUnit + 32];
  uint32_t cnt[kClsMap / 32];  // per block pair: C bytes starting in the block (low, high half)
  uint16_t P[kClsRank];        // output offset of each replacement from the aligned base
  uint32_t rel[66];
  uint64_t msk[65];
  uint16_t slow[kClsSlow];
};

// n_dev (chained calls): the input length on the device (n, nunits: upper
// bounds); ncnt (chained calls): the next substitution's class bytes
// (nsw1 / nsw2) per 4 KiB unit of this output, added up here.
__global__ __launch_bounds__(256, CLS_WAVES) void replace_cls_write_kernel(const uint8_t *hay, uint64_t n, const uint8_t *cls_g,
                                                                uint64_t nunits, const uint64_t *uoff,
                                                                const uint8_t *rep_g, uint32_t L, uint8_t *out,
                                                                uint64_t cap, uint32_t sw1, uint32_t sw2,
                                                                const uint64_t *n_dev, uint32_t nsw1, uint32_t nsw2,
                                                                uint32_t nrep, unsigned long long *ncnt) {
  __shared__ uint8_t cls[256];
  __shared__ uint8_t rep[64];
  __shared__ __attribute__((aligned(16))) ClsWave sw[4];
  cls[threadIdx.x] = cls_g[threadIdx.x];
  if (threadIdx.x < 64) rep[threadIdx.x] = threadIdx.x < L ? rep_g[threadIdx.x] : 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  ClsWave &W = sw[threadIdx.x >> 6];
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  const uint64_t ulim = nunits;  // the count arrays' units (ncnt: this output's)
  if (n_dev) {
    n = *n_dev;
    nunits = min(nunits, max<uint64_t>(1, (n + kClsUnit - 1) / kClsUnit));
  }
  for (uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < nunits; u += nw) {
    // stage: the lane's 64 bytes, class mask, output offset in the unit
    // (loading the next unit here, behind this one's output, was slower:
    // profiles/r05_replace_class.txt)
    uint4 v[4];
    uint32_t ua;
    cls_load_co(hay, n, u, lane, v, &ua);
#pragma unroll
    for (int j = 0; j < 4; ++j) *(uint4 *)(W.txt + tx(16 * lane + 1024 * j)) = v[j];
    wave_sync();
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = *(const uint4 *)(W.txt + tx(64 * lane + 16 * j));
    const uint32_t avail = ua > 64 * lane ? min(ua - 64 * lane, 64u) : 0u;
    const uint64_t m = cls_mask(cls, v, avail, sw1, sw2);
    const uint32_t k = (uint32_t)__popcll(m);
    const uint32_t len = avail + (L - 1) * k;  // this lane's output bytes
    // (output bytes: < 2^19; C bytes, <= 4096, above them)
    uint32_t incl = len | k << 19;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o);
      if (lane >= (uint32_t)o) incl += x;
    }
    const uint32_t tot = __shfl(incl, 63);
    const uint32_t T = tot & 0x7FFFF, K = tot >> 19;  // the unit's output bytes, C bytes
    const uint32_t r0 = (incl & 0x7FFFF) - len, kex = (incl >> 19) - k;
    if (lane == 0) *(uint4 *)(W.txt + kClsUnit) = make_uint4(0, 0, 0, 0);
    W.rel[lane] = r0;
    W.msk[lane] = m;
    if (lane == 63) { W.rel[64] = T; W.rel[65] = T; W.msk[64] = 0; }
    const uint64_t ob = u * kClsUnit + uoff[u] * (L - 1);  // the unit's output start
    const uint32_t o15 = (uint32_t)(ob & 15);
    if (nsw1) {
      // the next substitution's class bytes in this lane's output, by 4 KiB
      // output unit (the next call's units): its text bytes outside this
      // class, plus the copies in each replacement (nrep of them); a lane
      // whose output crosses a unit edge places them byte by byte
      const uint64_t nm = next_mask(v, avail, nsw1, nsw2) & ~m;
      const uint64_t os = ob + r0, oe = os + len;
      uint32_t lo = 0, hi = 0;  // counts in unit os >> 12 and the one after
      if (len == 0 || (os >> 12) == ((oe - 1) >> 12)) {
        lo = (uint32_t)__popcll(nm) + k * nrep;
      } else {
        // bytes before e1 count in the lane's first unit, before e1 + 4096 in
        // the next; later ones (a lane's output is at most 64 * 64 bytes:
        // only long replacements reach that far) take an atomic each
        const uint64_t e1 = (os | 4095) + 1;
        auto put = [&](uint64_t q) {
          if (q < e1) ++lo;
          else if (q < e1 + 4096) ++hi;
          else if ((q >> 12) < ulim) atomicAdd(&ncnt[q >> 12], 1ull);
        };
        uint64_t pos = os;
        for (uint32_t i = 0; i < avail; ++i) {
          if ((m >> i) & 1) {
#pragma unroll 1
            for (uint32_t t = 0; t < L; ++t) {
              const uint32_t rb = rep[t] * 0x01010101u;
              if (rb == nsw1 || rb == nsw2) put(pos + t);
            }
            pos += L;
          } else {
            if ((nm >> i) & 1) put(pos);
            ++pos;
          }
        }
      }
      // lanes' first units are U0 or U0 + 1 (U0 + 2 for a few): two packed sums
      const uint64_t U0 = ob >> 12;
      const uint32_t d = (uint32_t)((os >> 12) - U0);
      uint32_t p01 = 0, p12 = 0;
      if (d == 0) p01 = lo | hi << 16;
      else if (d == 1) p12 = lo | hi << 16;
      else {
        if (lo) atomicAdd(&ncnt[min(os >> 12, ulim - 1)], (unsigned long long)lo);
        if (hi) atomicAdd(&ncnt[min((os >> 12) + 1, ulim - 1)], (unsigned long long)hi);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        p01 += __shfl_xor(p01, o);
        p12 += __shfl_xor(p12, o);
      }
      if (lane == 0) {  // (each half: at most 4096 + 64 * 63 per unit... fits 16 bits)
        const uint32_t c0 = p01 & 0xFFFF, c1 = (p01 >> 16) + (p12 & 0xFFFF), c2 = p12 >> 16;
        if (c0 && U0 < ulim) atomicAdd(&ncnt[U0], (unsigned long long)c0);
        if (c1 && U0 + 1 < ulim) atomicAdd(&ncnt[U0 + 1], (unsigned long long)c1);
        if (c2 && U0 + 2 < ulim) atomicAdd(&ncnt[U0 + 2], (unsigned long long)c2);
      }
    }
    const bool map = o15 + T + 16 <= kClsMap && K <= kClsRank;
    if (map) {
#pragma unroll
      for (uint32_t i = 0; i < kClsCW; ++i) W.cnt[kClsCW * lane + i] = 0;
      wave_sync();
      uint64_t mm = m;
      uint32_t P = o15 + r0, rk = kex;  // output offset of the next C byte from the aligned base, less c; its rank
      while (mm) {
        const uint32_t c = (uint32_t)__builtin_ctzll(mm);
        mm &= mm - 1;
        const uint32_t q = P + c;
        atomicAdd(&W.cnt[q >> 5], (q & 16) ? 0x10000u : 1u);
        W.P[rk++] = (uint16_t)q;
        P += L - 1;
      }
      wave_sync();
      // exclusive prefix over the blocks (lane: words kClsCW lane ..)
      uint32_t cw[kClsCW];
#pragma unroll
      for (uint32_t i = 0; i < kClsCW; ++i) cw[i] = W.cnt[kClsCW * lane + i];
      uint32_t tot = 0;
#pragma unroll
      for (uint32_t i = 0; i < kClsCW; ++i) tot += (cw[i] & 0xFFFF) + (cw[i] >> 16);
      uint32_t ex = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(ex, o);
        if (lane >= (uint32_t)o) ex += x;
      }
      ex -= tot;
#pragma unroll
      for (uint32_t i = 0; i < kClsCW; ++i) {
        const uint32_t lo = ex;
        ex += cw[i] & 0xFFFF;
        W.cnt[kClsCW * lane + i] = lo | ex << 16;
        ex += cw[i] >> 16;
      }
    }
    wave_sync();
    const uint64_t base = ob - o15, A = (ob + 15) & ~(uint64_t)15, E = ob + T, B = E & ~(uint64_t)15;
    // whole aligned blocks: text-only blocks from the staged text, the
    // others to the wave's slow list
    uint32_t ns = 0;
    for (uint64_t q0 = A; q0 < B; q0 += 1024) {
      const uint64_t q = q0 + 16 * (uint64_t)lane;
      bool sl = false;
      if (q < B) {
        const uint32_t r = (uint32_t)(q - ob);
        bool fast;
        uint32_t src;
        if (map) {
          const uint32_t bl = (uint32_t)(q - base) >> 4;
          const uint32_t c0 = (W.cnt[bl >> 1] >> (16 * (bl & 1))) & 0xFFFF,
                         c1 = (W.cnt[(bl + 1) >> 1] >> (16 * ((bl + 1) & 1))) & 0xFFFF;
          fast = c1 == c0 && (c0 == 0 || W.P[c0 - 1] + L <= 16 * bl);
          src = r - (L - 1) * c0;
        } else {
          uint32_t x = min(r >> 6, 63u);
          while (x > 0 && W.rel[x] > r) --x;
          const uint32_t p = r - W.rel[x];
          uint64_t mm = W.msk[x];
          uint32_t cnt = 0, cn = 64;
          bool inrep = false;
          while (mm) {
            const uint32_t c = (uint32_t)__builtin_ctzll(mm);
            const uint32_t oc = c + (L - 1) * cnt;
            if (oc > p) { cn = c; break; }
            if (p < oc + L) { inrep = true; break; }
            mm &= mm - 1;
            ++cnt;
          }
          const uint32_t t = p - (L - 1) * cnt;  // input offset of the block's first byte in lane x
          // the next C byte after it in unit input coordinates
          uint32_t nxt = 64 * x + cn;
          if (cn == 64 && x < 63)
            nxt = W.msk[x + 1] ? 64 * (x + 1) + (uint32_t)__builtin_ctzll(W.msk[x + 1]) : 64 * (x + 2);
          fast = !inrep && 64 * x + t + 16 <= nxt;
          src = 64 * x + t;
        }
        fast = fast && q + 16 <= cap;
        if (fast) *(uint4 *)(out + q) = lds16u(W.txt, src);
        sl = !fast;
      }
      const uint64_t bm = __ballot(sl);
      if (sl) W.slow[ns + __popcll(bm & ((1ull << lane) - 1ull))] = (uint16_t)((q - A) >> 4);
      ns += (uint32_t)__popcll(bm);
      // the list is worked off when full (a unit dense in replacements of a
      // long string has up to 256 L blocks) and after the unit's last round
      if (ns + 64 > kClsSlow || q0 + 1024 >= B) {
        wave_sync();
#pragma unroll 1
        for (uint32_t i0 = 0; i0 < ns; i0 += 64) {
          if (i0 + lane < ns) {
            const uint64_t qs = A + 16 * (uint64_t)W.slow[i0 + lane];
            uint4 o;
            if (map) {
              const uint32_t bl = (uint32_t)(qs - base) >> 4;
              o = cls_block_map(16 * bl, (W.cnt[bl >> 1] >> (16 * (bl & 1))) & 0xFFFF, K, W.P, o15, W.txt, rep, L);
            } else {
              o = cls_block_slow((uint32_t)(qs - ob), T, W.rel, W.msk, W.txt, rep, L);
            }
            if (qs + 16 <= cap) {
              *(uint4 *)(out + qs) = o;
            } else {  // the output buffer ends inside this block
              const uint32_t bb[4] = {o.x, o.y, o.z, o.w};
              for (uint32_t j = 0; qs + j < cap; ++j) out[qs + j] = (uint8_t)(bb[j >> 2] >> (8 * (j & 3)));
            }
          }
        }
        ns = 0;
        wave_sync();
      }
    }
    // the edges: [ob, min(A, E)) and [max(B, A), E), byte by byte
    const uint64_t h1 = min(A, E), t0 = max(B, A);
    const uint64_t pos = lane < 16 ? ob + lane : t0 + (lane - 16);
    const bool mine = lane < 16 ? pos < h1 : (lane < 32 && pos < E);
    if (mine && pos < cap) out[pos] = cls_out_byte((uint32_t)(pos - ob), W.rel, W.msk, W.txt, rep, L);
    wave_sync();
  }
}

// ------------------------------------------------------------------
// A chain of one-byte-class replace_all steps is a string homomorphism: step
// i maps each byte of its class to rep_i and every other byte to itself, so
// the chain maps each byte x to F(x) = h_n(...h_1(x)), a string the host
// composes (HMap).  The whole chain is then one count pass and one write
// pass (the sequential chain: a count and a write pass per step), and every
// intermediate length follows from the input's histogram of the bytes F
// changes: length_i = n + sum_x hist[x] (|F_i(x)| - 1).
struct HMapDev {
  const uint8_t *flen;    // 256: |F(x)| (1..64)
  const uint16_t *soff;   // 256: offset of F(x) in pool
  const uint8_t *aidx;    // 256: index of x among the bytes F changes, 0xFF if F(x) = x
  const uint8_t *pool;    // the strings (at most kHMapPool bytes)
  uint32_t pool_len;
  uint32_t nact;          // bytes F changes
};
constexpr uint32_t kHMapPool = kHMapPoolMax;
constexpr uint32_t kHMapOut = 8192;  // a wave's staged output per 4 KiB unit (beyond: direct byte stores)
constexpr uint32_t kHMapReg = 16;    // changed bytes counted in lane registers (more: LDS atomics)

// Per unit: the output bytes it adds (sum of |F(x)| - 1); the histogram of
// the changed bytes.  Coalesced loads (lane l: the unit's 16-byte pieces l,
// l + 64, l + 128, l + 192); one LDS read per byte (info: |F(x)| - 1 and the
// changed-byte index); a changed byte (rare) bumps one of kHMapReg 16-bit
// lane counters (packed two per register, the index selecting the register
// by compares: no register array indexed at run time), summed over the wave
// and added to hist at the end — atomics per byte serialised on the few
// counters (0.94 ms per 2 GiB).  Past kHMapReg changed bytes: LDS atomics.
__global__ __launch_bounds__(256) void hmap_count_kernel(const uint8_t *in, uint64_t n, uint64_t nunits, HMapDev h,
                                                         uint64_t *ucount, unsigned long long *hist) {
  __shared__ uint32_t info[256];
  __shared__ uint8_t alist[256];
  __shared__ uint32_t lh[256];
  __shared__ __attribute__((aligned(16))) uint8_t txt[4][4096];
  {
    const uint32_t x = threadIdx.x, a = h.aidx[x];
    info[x] = (uint32_t)(h.flen[x] - 1) | a << 16;
    if (a != 0xFF) alist[a] = (uint8_t)x;
    lh[x] = 0;
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint8_t *T = txt[threadIdx.x >> 6];
  const bool reg = h.nact <= kHMapReg;
  uint32_t c[kHMapReg / 2];
#pragma unroll
  for (uint32_t k = 0; k < kHMapReg / 2; ++k) c[k] = 0;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  uint32_t rounds = 0;
  for (uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < nunits; u += nw) {
    const uint64_t s0 = u * 4096;
    const uint64_t av = s0 < n ? n - s0 : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // coalesced: lane l the pieces l, l + 64, ...
      const uint64_t o = 16 * (uint64_t)lane + 1024 * j;
      *(uint4 *)(T + o) = o < av ? *(const uint4 *)(in + s0 + o) : make_uint4(0, 0, 0, 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // lane l counts dwords l, l + 64, ... (conflict-free reads); the changed
    // bytes (rare, but in nearly every step of some lane) are marked and
    // counted after the loop, so the loop has no branch
    uint32_t extra = 0;
    uint64_t chg = 0;
#pragma unroll 4
    for (uint32_t i = 0; i < 16; ++i) {
      const uint32_t d = lane + 64 * i, w = ((const uint32_t *)T)[d];
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t inf = 4 * d + b < av ? info[(w >> (8 * b)) & 0xFF] : 0xFF0000u;
        extra += inf & 0xFFFF;
        chg |= (uint64_t)((inf >> 16) != 0xFF) << (4 * i + b);
      }
    }
    while (chg) {
      const uint32_t t = (uint32_t)__builtin_ctzll(chg);
      chg &= chg - 1;
      const uint32_t a = info[T[4 * (lane + 64 * (t >> 2)) + (t & 3)]] >> 16;
      if (reg) {
#pragma unroll
        for (uint32_t k = 0; k < kHMapReg / 2; ++k) c[k] += (a >> 1) == k ? 1u << (16 * (a & 1)) : 0u;
      } else {
        atomicAdd(&lh[alist[a]], 1u);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) extra += __shfl_xor(extra, o);
    if (lane == 0) ucount[u] = extra;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (16-bit lane counters: at most 64 per unit; emptied every 512 units)
    if (reg && ++rounds == 512) {
      rounds = 0;
#pragma unroll
      for (uint32_t a = 0; a < kHMapReg; ++a) {
        uint32_t t = (c[a >> 1] >> (16 * (a & 1))) & 0xFFFF;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
        if (lane == 0 && t && a < h.nact) atomicAdd(&lh[alist[a]], t);
      }
#pragma unroll
      for (uint32_t k = 0; k < kHMapReg / 2; ++k) c[k] = 0;
    }
  }
  if (reg) {
#pragma unroll
    for (uint32_t a = 0; a < kHMapReg; ++a) {
      uint32_t t = (c[a >> 1] >> (16 * (a & 1))) & 0xFFFF;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
      if (lane == 0 && t && a < h.nact) atomicAdd(&lh[alist[a]], t);
    }
  }
  __syncthreads();
  if (lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)lh[threadIdx.x]);
}

// Per unit: each lane holds its 64 bytes in registers (the next unit's
// already in flight: the kernel waits on memory otherwise, 3-4 waves per SIMD
// with one HBM round trip per unit) and writes their images into the wave's
// output stage at the unit's output alignment — every byte's first image
// byte in one branch-free pass, the longer images' other bytes from a wave
// list (ballot slots) by one lane each — then whole aligned 16-byte blocks
// are stored by consecutive lanes and the two edge blocks byte by byte (they
// share an aligned block with the neighbouring units: byte stores do not
// race).  uoff = exclusive sums of the units' added bytes.
struct HMapWave {
  uint8_t out[kHMapOut + 32];
  uint32_t rest[128];  // images longer than one byte: output offset << 8 | byte
};

__device__ __forceinline__ void hmap_lane_load(const uint8_t *in, uint64_t n, uint64_t u, uint32_t lane, uint4 *g) {
  const uint64_t s0 = u * 4096 + 64 * (uint64_t)lane;
  const uint64_t av = s0 < n ? n - s0 : 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) g[j] = 16u * j < av ? *(const uint4 *)(in + s0 + 16 * j) : make_uint4(0, 0, 0, 0);
}

__global__ __launch_bounds__(256) void hmap_write_kernel(const uint8_t *in, uint64_t n, uint64_t nunits, HMapDev h,
                                                         const uint64_t *uoff, uint8_t *out, uint64_t cap) {
  __shared__ uint32_t info[256];  // |F(x)| | (F(x) = x) << 7 | offset << 8
  __shared__ __attribute__((aligned(16))) HMapWave sw[4];
  extern __shared__ __attribute__((aligned(16))) uint8_t pool[];  // (dynamic: pool_len)
  {
    const uint32_t x = threadIdx.x;
    info[x] = (uint32_t)h.flen[x] | (h.aidx[x] == 0xFF ? 0x80u : 0u) | (uint32_t)h.soff[x] << 8;
  }
  for (uint32_t i = threadIdx.x; i < h.pool_len; i += blockDim.x) pool[i] = h.pool[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  HMapWave &W = sw[threadIdx.x >> 6];
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint4 gn[4];
  hmap_lane_load(in, n, u, lane, gn);
  for (; u < nunits; u += nw) {
    uint4 g[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = gn[j];
    hmap_lane_load(in, n, u + nw < nunits ? u + nw : u, lane, gn);  // the next unit, in flight
    const uint64_t s0 = u * 4096;
    const uint64_t lb = s0 + 64 * (uint64_t)lane;
    const uint32_t avail = n > lb ? (uint32_t)min<uint64_t>(n - lb, 64) : 0u;
    uint32_t len = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      const uint4 q = g[k >> 2];
      const uint32_t w = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
#pragma unroll 1
      for (uint32_t b = 0; b < 4; ++b) len += 4 * k + b < avail ? info[(w >> (8 * b)) & 0xFF] & 0x7F : 0u;
    }
    uint32_t incl = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o);
      if (lane >= (uint32_t)o) incl += x;
    }
    const uint32_t T = __shfl(incl, 63), r0 = incl - len;
    const uint64_t ob = s0 + uoff[u];  // the unit's output start
    const uint32_t o15 = (uint32_t)(ob & 15);
    if (o15 + T + 16 > kHMapOut) {  // a unit that grows past the stage: byte stores, in order
      uint64_t p = ob + r0;
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint4 q = g[k >> 2];
        const uint32_t w = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
#pragma unroll 1
        for (uint32_t b = 0; b < 4 && 4 * k + b < avail; ++b) {
          const uint32_t inf = info[(w >> (8 * b)) & 0xFF], l = inf & 0x7F, off = inf >> 8;
          for (uint32_t t = 0; t < l; ++t, ++p)
            if (p < cap) out[p] = pool[off + t];
        }
      }
      continue;
    }
    {
      uint32_t pos = o15 + r0, nrest = 0;
      auto flush = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t e = lane; e < nrest; e += 64) {
          const uint32_t r = W.rest[e], inf = info[r & 0xFF], l = inf & 0x7F, off = inf >> 8;
          uint8_t *d = W.out + (r >> 8);
          for (uint32_t j = 1; j < l; ++j) d[j] = pool[off + j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        nrest = 0;
      };
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint4 q = g[k >> 2];
        const uint32_t w = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
#pragma unroll 1
        for (uint32_t b = 0; b < 4; ++b) {
          const bool in_ = 4 * k + b < avail;
          const uint32_t x = (w >> (8 * b)) & 0xFF, inf = info[x];
          const uint32_t l = in_ ? inf & 0x7F : 0u;
          if (in_) W.out[pos] = (inf & 0x80) ? (uint8_t)x : pool[inf >> 8];
          const bool lg = l > 1;
          const uint64_t m = __ballot(lg);
          if (lg) W.rest[nrest + __popcll(m & ((1ull << lane) - 1ull))] = pos << 8 | x;
          nrest += (uint32_t)__popcll(m);
          pos += l;
          if (nrest > 64) flush();  // (at most 64 join per byte step: the list holds 128)
        }
      }
      if (nrest) flush();
    }
    const uint64_t base = ob - o15, E = ob + T;
    const uint64_t A = (ob + 15) & ~(uint64_t)15, B = E & ~(uint64_t)15;
    for (uint64_t q = A + 16 * (uint64_t)lane; q < B; q += 1024) {
      const uint4 x = *(const uint4 *)(W.out + (q - base));
      if (q + 16 <= cap) *(uint4 *)(out + q) = x;
      else for (uint32_t j = 0; q + j < cap; ++j) out[q + j] = W.out[q - base + j];
    }
    // the edges: [ob, min(A, E)) and [max(B, A), E)
    const uint64_t h1 = min(A, E), t0 = max(B, A);
    const uint64_t pos = lane < 16 ? ob + lane : t0 + (lane - 16);
    const bool mine = lane < 16 ? pos < h1 : (lane < 32 && pos < E);
    if (mine && pos < cap) out[pos] = W.out[pos - base];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// lengths[i + 1] = n + sum_x hist[x] * dlen[i * 256 + x] (dlen = |F_i(x)| - 1
// for the bytes F changes), one thread per step
__global__ void hmap_lengths_kernel(uint64_t n, int steps, const unsigned long long *hist, const uint32_t *dlen,
                                    uint64_t *lengths) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i == 0) lengths[0] = n;
  if (i >= steps) return;
  uint64_t t = n;
  for (int x = 0; x < 256; ++x) t += (uint64_t)hist[x] * dlen[(size_t)i * 256 + x];
  lengths[i + 1] = t;
}

}  // namespace

hipError_t exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t st) {
  size_t tmp = 0;
  hipError_t e = rocprim::exclusive_scan(nullptr, tmp, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), st);
  if (e != hipSuccess) return e;
  void *buf = nullptr;
  if ((e = scratch_malloc(&buf, tmp, st)) != hipSuccess) return e;
  e = rocprim::exclusive_scan(buf, tmp, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), st);
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

hipError_t launch_replace_plan(const BatchDev &b, const uint64_t *counts, const uint64_t *moff, const uint64_t *m,
                               uint64_t limit, uint64_t rep_len, int64_t *shift, uint64_t *out_len, hipStream_t st,
                               int cus, uint64_t nm) {
  if (b.count == 1 && limit == ~0ull) {  // one scan into shift's nm + 1 entries: G (GOne)
    auto in = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint64_t>(0),
                                               GOne{m, b.offs, nm, b.length, (int64_t)rep_len});
    size_t tmp = 0;
    hipError_t e = rocprim::inclusive_scan(nullptr, tmp, in, shift, (size_t)(nm + 1), rocprim::plus<int64_t>(), st);
    void *buf = nullptr;
    if (e == hipSuccess) e = scratch_malloc(&buf, tmp, st);
    if (e == hipSuccess)
      e = rocprim::inclusive_scan(buf, tmp, in, shift, (size_t)(nm + 1), rocprim::plus<int64_t>(), st);
    if (buf) { hipError_t e2 = scratch_free(buf, st); if (e == hipSuccess) e = e2; }
    if (e == hipSuccess) {
      hipLaunchKernelGGL(replace_len1_kernel, dim3(1), dim3(1), 0, st, shift, nm, out_len);
      e = hipGetLastError();
    }
    return e;
  }
  int64_t *val = nullptr, *S = nullptr;
  hipError_t e = scratch_malloc((void **)&val, (nm + 1) * 8, st);
  if (e == hipSuccess) e = scratch_malloc((void **)&S, (nm + 1) * 8, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(replace_vals_kernel, dim3(grid_for_items(nm + 1, 256, cus)), dim3(256), 0, st, b.count, counts,
                       moff, m, limit, rep_len, val);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    size_t tmp = 0;
    e = rocprim::exclusive_scan(nullptr, tmp, val, S, (int64_t)0, (size_t)(nm + 1), rocprim::plus<int64_t>(), st);
    void *buf = nullptr;
    if (e == hipSuccess) e = scratch_malloc(&buf, tmp, st);
    if (e == hipSuccess)
      e = rocprim::exclusive_scan(buf, tmp, val, S, (int64_t)0, (size_t)(nm + 1), rocprim::plus<int64_t>(), st);
    if (buf) { hipError_t e2 = scratch_free(buf, st); if (e == hipSuccess) e = e2; }
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(replace_shift_kernel, dim3(grid_for_items(nm + b.count, 256, cus)), dim3(256), 0, st, b, counts,
                       moff, limit, S, shift, out_len);
    e = hipGetLastError();
  }
  if (val) { hipError_t e2 = scratch_free(val, st); if (e == hipSuccess) e = e2; }
  if (S) { hipError_t e2 = scratch_free(S, st); if (e == hipSuccess) e = e2; }
  return e;
}

hipError_t launch_replace_copy(const BatchDev &b, const uint64_t *ooff, const uint64_t *counts, const uint64_t *moff,
                               const uint64_t *m, const int64_t *shift, uint64_t limit, const uint8_t *rep,
                               uint64_t rep_len, uint8_t *out, uint64_t cap, uint64_t total_hint, hipStream_t st,
                               int cus, uint64_t nm) {
  // total_hint bounds the bytes written (the output is at most the text
  // plus the replacements, and at most cap)
  const uint64_t nwin = (total_hint + kWin - 1) / kWin;
  // one haystack, every match replaced: launch_replace_plan left G in shift
  const bool one = b.count == 1 && limit == ~0ull;
  uint64_t *G = one ? (uint64_t *)shift : nullptr, *gbuf = nullptr, *widx = nullptr;
  hipError_t e = one ? hipSuccess : scratch_malloc((void **)&gbuf, std::max<uint64_t>(nm, 1) * 8, st);
  if (!one) G = gbuf;
  if (e == hipSuccess) e = scratch_malloc((void **)&widx, (nwin + 2) * 8, st);
  if (e == hipSuccess && nm == 0) e = hipMemsetAsync(widx, 0, (nwin + 2) * 8, st);
  if (e == hipSuccess && nm) {
    if (!one)
      hipLaunchKernelGGL(replace_g_kernel, dim3(grid_for_items(nm, 256, cus)), dim3(256), 0, st, b.count, ooff, moff,
                         m, shift, G);
    hipLaunchKernelGGL(replace_widx_kernel, dim3(grid_for_items(nwin + 1, 256, cus)), dim3(256), 0, st, b.count, moff,
                       G, nwin + 1, widx);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    CopyCtx c;
    c.bt = b;
    c.ooff = ooff;
    c.counts = counts;
    c.moff = moff;
    c.m = m;
    c.G = G;
    c.widx = widx;
    c.shift = shift;
    c.limit = limit;
    c.rep_len = rep_len;
    c.total = 0;
    c.cap = cap;
    c.rep = rep;
    c.one = one;
    if (b.count == 1 && limit == ~0ull && knob(Knob::ReplaceGeneric) != 1 && total_hint < (1ull << 36)) {
      const uint64_t nblk = (total_hint + 15) / 16, rcap = std::max<uint64_t>(4096, nblk / 16);
      uint32_t *rest = nullptr;
      e = scratch_malloc((void **)&rest, rcap * 4 + 256, st);  // (u32 block indices: outputs < 64 GiB)
      unsigned long long *nrest = rest ? (unsigned long long *)(rest + ((rcap + 1) & ~(uint64_t)1)) : nullptr;
      if (e == hipSuccess) e = hipMemsetAsync(nrest, 0, 8, st);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(replace_copy4_kernel, dim3(grid_for_items((total_hint + 63) / 64, 256, cus)), dim3(256), 0,
                           st, c, out, rest, rcap, nrest);
        hipLaunchKernelGGL(replace_rest_kernel, dim3(grid_for_items(nblk / 64 + 1, 256, cus)), dim3(256), 0, st, c,
                           out, rest, rcap, nrest);
        e = hipGetLastError();
      }
      if (rest) { hipError_t e2 = scratch_free(rest, st); if (e == hipSuccess) e = e2; }
    }
    else
      hipLaunchKernelGGL(replace_copy_kernel,
                         dim3(grid_for_items((total_hint + 16 * kCopyILP - 1) / (16 * kCopyILP), 256, cus)),
                         dim3(256), 0, st, c, out);
    if (e == hipSuccess) e = hipGetLastError();
  }
  for (uint64_t *q : {gbuf, widx})
    if (q) { hipError_t e2 = scratch_free(q, st); if (e == hipSuccess) e = e2; }
  return e;
}

hipError_t launch_split(const BatchDev &b, const uint64_t *counts, const uint64_t *moff, const uint64_t *m,
                        uint64_t lim, uint64_t *fields, uint64_t *foff, uint64_t *pieces, uint64_t cap,
                        uint64_t nmatches, hipStream_t st, int cus) {
  hipLaunchKernelGGL(split_count_kernel, dim3(grid_for_items(b.count, 256, cus)), dim3(256), 0, st, b, counts, moff, m,
                     lim, fields);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if ((e = exclusive_scan_u64(fields, foff, b.count + 1, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(split_emit_kernel, dim3(grid_for_items(nmatches + b.count, 256, cus)), dim3(256), 0, st, b,
                     counts, moff, m, lim, foff, pieces, cap);
  return hipGetLastError();
}


// replace_all of a one-byte-class regex over one haystack (16-byte aligned,
// search from 0): cls[256] (device) = the class, rep (device) at most 64
// bytes.  Writes out (at most cap bytes), out_offsets {0, total}, *total.
// The class replace kernels' resident blocks per CU, per device (computed
// once per device under a lock: the launch may come from several threads
// and devices)
static hipError_t cls_occupancy(int dev, int *occ_c, int *occ_w) {
  static std::mutex mu;
  static std::vector<std::pair<int, int>> cache;
  std::lock_guard<std::mutex> g(mu);
  if ((int)cache.size() <= dev) cache.resize(dev + 1, {0, 0});
  if (!cache[dev].first) {
    int c = 0, w = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&c, replace_cls_count_kernel, 256, 0);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&w, replace_cls_write_kernel, 256, 0);
    if (e != hipSuccess) return e;
    cache[dev] = {std::max(1, c), std::max(1, w)};
  }
  *occ_c = cache[dev].first;
  *occ_w = cache[dev].second;
  return hipSuccess;
}

hipError_t launch_replace_class(const uint8_t *hay, uint64_t n, const uint8_t *cls, const uint8_t *rep,
                                uint32_t rep_len, uint8_t *out, uint64_t cap, uint64_t *ooff, uint64_t *total,
                                hipStream_t st, int cus, uint32_t sw1, uint32_t sw2) {
  if (((uintptr_t)hay & 15) || rep_len > 64 || rep_len == 0) return hipErrorNotSupported;
  const uint64_t nunits = std::max<uint64_t>(1, (n + kClsUnit - 1) / kClsUnit);
  // resident blocks only (a grid-stride loop over more blocks than the
  // CUs hold runs the rest as a tail at low occupancy)
  int dev = 0, occ_c = 0, occ_w = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if ((e = cls_occupancy(dev, &occ_c, &occ_w)) != hipSuccess) return e;
  uint64_t *buf = nullptr;
  if ((e = scratch_malloc((void **)&buf, (2 * nunits + 2) * 8, st)) != hipSuccess) return e;
  uint64_t *ucount = buf, *uoff = buf + nunits + 1;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((nunits + 7) / 8, (uint64_t)cus * occ_c));
  const int gridw = (int)std::max<uint64_t>(1, std::min<uint64_t>((nunits + 3) / 4, (uint64_t)cus * occ_w));
  do {
    if ((e = hipMemsetAsync(ucount + nunits, 0, 8, st)) != hipSuccess) break;
    hipLaunchKernelGGL(replace_cls_count_kernel, dim3(grid), dim3(256), 0, st, hay, n, cls, nunits, ucount, sw1, sw2,
                       (const uint64_t *)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = exclusive_scan_u64(ucount, uoff, nunits + 1, st)) != hipSuccess) break;
    hipLaunchKernelGGL(replace_cls_total_kernel, dim3(1), dim3(1), 0, st, n, (uint64_t)rep_len, uoff, nunits, ooff,
                       total, (const uint64_t *)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if (cap) {
      hipLaunchKernelGGL(replace_cls_write_kernel, dim3(gridw), dim3(256), 0, st, hay, n, cls, nunits, uoff, rep,
                         rep_len, out, cap, sw1, sw2, (const uint64_t *)nullptr, 0u, 0u, 0u,
                         (unsigned long long *)nullptr);
      e = hipGetLastError();
    }
  } while (false);
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

// The chain as one byte -> string map (see HMapDev): per byte |F(x)| (256
// u8), offsets (256 u16), changed-byte indices (256 u8, 0xFF: unchanged;
// nact of them), the pool, then per step i |F_i(x)| - 1 as 256 u32 (device,
// one blob); the final text goes to out.
hipError_t launch_replace_hmap(const uint8_t *in, uint64_t n, int steps, const uint8_t *blob, uint32_t pool_len,
                               uint32_t nact, uint8_t *out, uint64_t cap, uint64_t *lengths, hipStream_t st,
                               int cus) {
  HMapDev h;
  h.flen = blob;
  h.soff = (const uint16_t *)(blob + 256);
  h.aidx = blob + 768;
  h.pool = blob + 1024;
  h.pool_len = pool_len;
  h.nact = nact;
  const uint32_t *dlen = (const uint32_t *)(blob + 1024 + kHMapPool);
  if (pool_len > kHMapPool) return hipErrorNotSupported;
  const uint64_t nunits = std::max<uint64_t>(1, (n + 4095) / 4096);
  uint64_t *buf = nullptr;
  hipError_t e = scratch_malloc((void **)&buf, (2 * (nunits + 1) + 256) * 8, st);
  if (e != hipSuccess) return e;
  uint64_t *ucount = buf, *uoff = buf + nunits + 1;
  unsigned long long *hist = (unsigned long long *)(uoff + nunits + 1);
  do {
    if ((e = hipMemsetAsync(ucount + nunits, 0, 8, st)) != hipSuccess) break;
    if ((e = hipMemsetAsync(hist, 0, 256 * 8, st)) != hipSuccess) break;
    const int g = grid_for_items((nunits + 3) / 4 * 256, 256, cus);
    const int gw = std::min(g, cus * 4);  // (the write kernel's LDS stages: 4 blocks per CU)
    hipLaunchKernelGGL(hmap_count_kernel, dim3(g), dim3(256), 0, st, in, n, nunits, h, ucount, hist);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = exclusive_scan_u64(ucount, uoff, nunits + 1, st)) != hipSuccess) break;
    hipLaunchKernelGGL(hmap_write_kernel, dim3(gw), dim3(256), (pool_len + 15) & ~15u, st, in, n, nunits, h, uoff,
                       out, cap);
    if ((e = hipGetLastError()) != hipSuccess) break;
    hipLaunchKernelGGL(hmap_lengths_kernel, dim3(1), dim3(std::max(64, (steps + 63) / 64 * 64)), 0, st, n, steps,
                       (const unsigned long long *)hist, dlen, lengths);
    e = hipGetLastError();
  } while (false);
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

// A chain of replace_all calls of one-byte-class regexes over one haystack
// (the IUB substitutions), step i reading step i - 1's output: buffers
// alternate out0, out1, out0, ...  The input of step i > 0 is counted by step
// i - 1's write kernel as it writes it (the next class as SWAR bytes,
// nxt[i][0..1], when the class has at most two bytes), so only step 0 and
// steps after a wider class run the count pass; the lengths stay on the
// device (lengths[i + 1] = the output length of step i) and nothing is read
// back.  Outputs past cap are cut (the lengths still count them; a step whose
// input was cut reads garbage past cap, so the caller checks lengths[steps]
// <= cap: replacements are never shorter than the byte they replace, so the
// lengths only grow).
hipError_t launch_replace_class_chain(const uint8_t *hay, uint64_t n0, int steps, const uint8_t *const *cls,
                                      const uint8_t *const *rep, const uint32_t *rep_len, const uint32_t (*sw)[2],
                                      const uint32_t *nrep, uint8_t *out0, uint8_t *out1, uint64_t cap,
                                      uint64_t *lengths, hipStream_t st, int cus) {
  if (steps <= 0) return hipSuccess;
  if (((uintptr_t)hay & 15) || ((uintptr_t)out0 & 15) || ((uintptr_t)out1 & 15)) return hipErrorNotSupported;
  for (int i = 0; i < steps; ++i)
    if (rep_len[i] > 64 || rep_len[i] == 0) return hipErrorNotSupported;
  int dev = 0, occ_c = 0, occ_w = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if ((e = cls_occupancy(dev, &occ_c, &occ_w)) != hipSuccess) return e;
  // units: enough for the largest input (n0 or cap)
  const uint64_t nmax = std::max<uint64_t>(n0, cap);
  const uint64_t nunits = std::max<uint64_t>(1, (nmax + kClsUnit - 1) / kClsUnit);
  uint64_t *buf = nullptr;
  if ((e = scratch_malloc((void **)&buf, (3 * (nunits + 1) + 1) * 8, st)) != hipSuccess) return e;
  uint64_t *cnt[2] = {buf, buf + nunits + 1}, *uoff = buf + 2 * (nunits + 1);
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((nunits + 7) / 8, (uint64_t)cus * occ_c));
  const int gridw = (int)std::max<uint64_t>(1, std::min<uint64_t>((nunits + 3) / 4, (uint64_t)cus * occ_w));
  do {
    if ((e = hipMemcpyAsync(lengths, &n0, 8, hipMemcpyHostToDevice, st)) != hipSuccess) break;
    bool counted = false;  // cnt[i & 1] holds step i's unit counts
    for (int i = 0; i < steps && e == hipSuccess; ++i) {
      const uint8_t *in = i == 0 ? hay : (i & 1) ? out0 : out1;
      uint8_t *out = (i & 1) ? out1 : out0;
      const uint64_t n = i == 0 ? n0 : nmax;  // (an upper bound past step 0: the kernels read lengths[i])
      const uint64_t *n_dev = i == 0 ? nullptr : lengths + i;
      uint64_t *c = cnt[i & 1], *cn = cnt[(i + 1) & 1];
      if (!counted) {
        if ((e = hipMemsetAsync(c, 0, (nunits + 1) * 8, st)) != hipSuccess) break;
        hipLaunchKernelGGL(replace_cls_count_kernel, dim3(grid), dim3(256), 0, st, in, n, cls[i], nunits, c,
                           sw[i][0], sw[i][1], n_dev);
        if ((e = hipGetLastError()) != hipSuccess) break;
      }
      if ((e = exclusive_scan_u64(c, uoff, nunits + 1, st)) != hipSuccess) break;
      const bool chain = i + 1 < steps && sw[i + 1][0] != 0;
      if (chain && (e = hipMemsetAsync(cn, 0, (nunits + 1) * 8, st)) != hipSuccess) break;
      hipLaunchKernelGGL(replace_cls_write_kernel, dim3(gridw), dim3(256), 0, st, in, n, cls[i], nunits, uoff, rep[i],
                         rep_len[i], out, cap, sw[i][0], sw[i][1], n_dev, chain ? sw[i + 1][0] : 0u,
                         chain ? sw[i + 1][1] : 0u, chain ? nrep[i] : 0u,
                         chain ? (unsigned long long *)cn : (unsigned long long *)nullptr);
      if ((e = hipGetLastError()) != hipSuccess) break;
      hipLaunchKernelGGL(replace_cls_total_kernel, dim3(1), dim3(1), 0, st, n, (uint64_t)rep_len[i], uoff, nunits,
                         (uint64_t *)nullptr, lengths + i + 1, n_dev);
      e = hipGetLastError();
      counted = chain;
    }
  } while (false);
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

}  // namespace rure_amd
