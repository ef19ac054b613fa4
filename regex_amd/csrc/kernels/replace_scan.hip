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

#include <cstdlib>
#include <cstring>
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

// One wave per haystack: shift_j for its first k matches and the output length.
// (Replaced by replace_vals / replace_shift: a haystack's matches were one
// wave's sequential loop, 0.4 s for the regex-dna strip's 35 M matches.)
__global__ __launch_bounds__(256) void replace_plan_kernel(BatchDev bt, const uint64_t *counts, const uint64_t *moff,
                                                           const uint64_t *m, uint64_t limit, uint64_t rep_len,
                                                           int64_t *shift, uint64_t *out_len) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t h = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); h < bt.count; h += nw) {
    uint64_t base, len;
    hay_of(bt, h, &base, &len);
    const uint64_t k = counts[h] < limit ? counts[h] : limit;
    const uint64_t m0 = moff[h];
    uint64_t carry = 0;  // bytes removed by the matches before this chunk of 64
    for (uint64_t j0 = 0; j0 < k; j0 += 64) {
      const uint64_t j = j0 + lane;
      uint64_t d = 0;
      if (j < k) d = m[2 * (m0 + j) + 1] - m[2 * (m0 + j)];
      uint64_t incl = d;  // inclusive wave scan
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t v = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += v;
      }
      if (j < k) shift[m0 + j] = (int64_t)(carry + incl - d) - (int64_t)(j * rep_len);
      carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) out_len[h] = len - carry + k * rep_len;
  }
}

__global__ __launch_bounds__(256) void replace_copy_kernel(BatchDev bt, const uint64_t *ooff, const uint64_t *counts,
                                                           const uint64_t *moff, const uint64_t *m,
                                                           const int64_t *shift, uint64_t limit, const uint8_t *rep,
                                                           uint64_t rep_len, uint8_t *out, uint64_t cap) {
  const uint64_t n = bt.count;
  const uint64_t total = ooff[n] < cap ? ooff[n] : cap;
  const uint64_t nblk = (total + 15) / 16;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nblk; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t p0 = q * 16;
    uint64_t h = upper_idx(ooff, 0, n + 1, p0) - 1;  // ooff[h] <= p0 < ooff[h+1]
    uint8_t v[16];
    uint64_t hh = ~0ull, base = 0, k = 0, m0 = 0, jj = 0;  // jj = matches whose replacement starts <= position
    for (int i = 0; i < 16; ++i) {
      const uint64_t p = p0 + i;
      if (p >= total) { v[i] = 0; continue; }
      while (p >= ooff[h + 1]) ++h;  // haystacks with empty output are skipped
      const uint64_t loc = p - ooff[h];
      if (h != hh) {
        hh = h;
        uint64_t len;
        hay_of(bt, h, &base, &len);
        k = counts[h] < limit ? counts[h] : limit;
        m0 = moff[h];
        uint64_t lo = 0, hi = k;
        while (lo < hi) {
          const uint64_t mid = (lo + hi) >> 1;
          if ((uint64_t)((int64_t)m[2 * (m0 + mid)] - shift[m0 + mid]) <= loc) lo = mid + 1;
          else hi = mid;
        }
        jj = lo;
      }
      while (jj < k && (uint64_t)((int64_t)m[2 * (m0 + jj)] - shift[m0 + jj]) <= loc) ++jj;
      uint8_t c;
      if (jj == 0) {
        c = bt.hay[base + loc];
      } else {
        const uint64_t j = m0 + jj - 1;
        const uint64_t r = (uint64_t)((int64_t)m[2 * j] - shift[j]);
        c = loc - r < rep_len ? rep[loc - r] : bt.hay[base + m[2 * j + 1] + (loc - r - rep_len)];
      }
      v[i] = c;
    }
    if (p0 + 16 <= total) {
      uint4 w;
      w.x = v[0] | (v[1] << 8) | (v[2] << 16) | ((uint32_t)v[3] << 24);
      w.y = v[4] | (v[5] << 8) | (v[6] << 16) | ((uint32_t)v[7] << 24);
      w.z = v[8] | (v[9] << 8) | (v[10] << 16) | ((uint32_t)v[11] << 24);
      w.w = v[12] | (v[13] << 8) | (v[14] << 16) | ((uint32_t)v[15] << 24);
      *(uint4 *)(out + p0) = w;
    } else {
      for (int i = 0; i < 16 && p0 + i < total; ++i) out[p0 + i] = v[i];
    }
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
  if (getenv("RURE_AMD_REPLACE_WAVE")) {  // the previous wave-per-haystack plan (A/B)
    hipLaunchKernelGGL(replace_plan_kernel, dim3(grid_for_items(b.count, 4, cus)), dim3(256), 0, st, b, counts, moff,
                       m, limit, rep_len, shift, out_len);
    return hipGetLastError();
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
                               int cus) {
  hipLaunchKernelGGL(replace_copy_kernel, dim3(grid_for_items((total_hint + 15) / 16, 256, cus)), dim3(256), 0, st, b,
                     ooff, counts, moff, m, shift, limit, rep, rep_len, out, cap);
  return hipGetLastError();
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

}  // namespace rure_amd
