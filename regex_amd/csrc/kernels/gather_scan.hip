// Match-record compaction for the multi-GPU gather.
//
// A rank's batched find leaves one (start, end) pair per haystack, SIZE_MAX
// where there is no match.  The only data-path exchange of the sharded scan is
// an all-gather of the matches, so they are compacted on the device first —
// (base + haystack, start, end) records in haystack order plus their count —
// without a host round trip (a `nonzero` would synchronise every step).
//
// count_kernel writes the number of matching haystacks of every 1024-haystack
// block; write_kernel sums the counts of the blocks before its own (up to
// 4096 blocks: a few thousand u64 read by 256 threads; beyond, a rocPRIM
// exclusive scan of the counts runs in between), scans its block in
// registers / LDS and writes its records.  The last block also writes the
// total.  Deterministic order; the find output is read twice.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dfa_scan.hpp"

namespace rure_amd {

namespace {

constexpr uint32_t kCompactPer = 4;                    // haystacks per thread
constexpr uint32_t kCompactBlock = 256 * kCompactPer;  // haystacks per block

__device__ __forceinline__ uint32_t hits4(const uint64_t *found, uint64_t n, uint64_t h0, uint32_t *mask) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCompactPer; ++k) {
    const uint64_t h = h0 + k;
    if (h < n && found[2 * h] != ~(uint64_t)0) m |= 1u << k;
  }
  *mask = m;
  return __popc(m);
}

// Exclusive prefix of v over the 256 threads of the block; *total = the sum.
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *total) {
  __shared__ uint32_t wsum[4];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(incl, o, 64);
    if (lane >= (uint32_t)o) incl += x;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    before += j < w ? wsum[j] : 0;
    all += wsum[j];
  }
  *total = all;
  return before + incl - v;
}

__global__ __launch_bounds__(256) void compact_count_kernel(const uint64_t *found, uint64_t n, uint64_t *blk) {
  const uint64_t h0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * kCompactPer;
  uint32_t m, total;
  block_excl(hits4(found, n, h0, &m), &total);
  if (threadIdx.x == 0) blk[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void compact_write_kernel(const uint64_t *found, uint64_t n, uint64_t base,
                                                            const uint64_t *blk, const uint64_t *excl, uint64_t *rec,
                                                            uint64_t cap, uint64_t *count) {
  // records before this block
  __shared__ uint64_t red[4];
  uint64_t s = 0;
  if (excl) s = threadIdx.x == 0 ? excl[blockIdx.x] : 0;
  else
    for (uint32_t j = threadIdx.x; j < blockIdx.x; j += 256) s += blk[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const uint64_t off = red[0] + red[1] + red[2] + red[3];
  const uint64_t h0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * kCompactPer;
  uint32_t m, total;
  uint64_t o = off + block_excl(hits4(found, n, h0, &m), &total);
  while (m) {
    const uint32_t k = __ffs(m) - 1;
    m &= m - 1;
    if (o < cap) {
      const uint64_t h = h0 + k;
      rec[3 * o] = base + h;
      rec[3 * o + 1] = found[2 * h];
      rec[3 * o + 2] = found[2 * h + 1];
    }
    ++o;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *count = off + total;
}

__global__ __launch_bounds__(256) void mask_column_kernel(const uint8_t *s8, const uint64_t *s64, uint64_t n,
                                                          uint64_t *dst, uint64_t words, uint64_t w) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    dst[i * words + w] = s8 ? (uint64_t)(s8[i] != 0) : s64[i];
}

// find_iter of a regex whose every match ends at the end of the text
// (DfaAnchoredReverse): at most the find result (dispatch.cpp run_find_iter).
__global__ __launch_bounds__(256) void one_match_counts_kernel(const uint64_t *found, uint64_t n, uint64_t *cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    cnt[i] = found[2 * i] != ~(uint64_t)0 ? 1 : 0;
}

__global__ __launch_bounds__(256) void one_match_write_kernel(const uint64_t *found, uint64_t n, const uint64_t *off,
                                                              uint64_t *counts, uint64_t *m, uint64_t cap,
                                                              uint64_t *total) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t c = off[i + 1] - off[i];
    counts[i] = c;
    if (c && off[i] < cap) {
      m[2 * off[i]] = found[2 * i];
      m[2 * off[i] + 1] = found[2 * i + 1];
    }
    if (i + 1 == n) *total = off[n];
  }
}

}  // namespace

hipError_t launch_find_to_iter(const uint64_t *found, uint64_t n, uint64_t *counts, uint64_t *matches, uint64_t cap,
                               uint64_t *total, hipStream_t st) {
  uint64_t *buf = nullptr;
  hipError_t e = scratch_malloc((void **)&buf, (n + 1) * 16, st);
  if (e != hipSuccess) return e;
  const uint32_t g = (uint32_t)std::min<uint64_t>((n + 255) / 256 ? (n + 255) / 256 : 1, 8192);
  e = hipMemsetAsync(buf + n, 0, 8, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(one_match_counts_kernel, dim3(g), dim3(256), 0, st, found, n, buf);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = exclusive_scan_u64(buf, buf + n + 1, n + 1, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(one_match_write_kernel, dim3(g), dim3(256), 0, st, found, n, buf + n + 1, counts, matches, cap,
                       total);
    e = hipGetLastError();
  }
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

hipError_t launch_mask_column(const uint8_t *s8, const uint64_t *s64, uint64_t n, uint64_t *dst, uint64_t words,
                              uint64_t w, hipStream_t st) {
  const uint64_t g = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(mask_column_kernel, dim3((uint32_t)(g ? g : 1)), dim3(256), 0, st, s8, s64, n, dst, words, w);
  return hipGetLastError();
}

hipError_t launch_compact_matches(const uint64_t *found, uint64_t n, uint64_t base, uint64_t *rec, uint64_t cap,
                                  uint64_t *count, hipStream_t st) {
  const uint64_t nb = n ? (n + kCompactBlock - 1) / kCompactBlock : 1;
  if (nb > 0x7fffffffull) return hipErrorInvalidValue;
  const bool scan = nb > 4096;
  uint64_t *blk = nullptr;
  hipError_t e = scratch_malloc((void **)&blk, nb * 8 * (scan ? 2 : 1), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(compact_count_kernel, dim3((uint32_t)nb), dim3(256), 0, st, found, n, blk);
  e = hipGetLastError();
  if (e == hipSuccess && scan) e = exclusive_scan_u64(blk, blk + nb, nb, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(compact_write_kernel, dim3((uint32_t)nb), dim3(256), 0, st, found, n, base, blk,
                       scan ? blk + nb : nullptr, rec, cap, count);
    e = hipGetLastError();
  }
  hipError_t e2 = scratch_free(blk, st);
  return e != hipSuccess ? e : e2;
}

}  // namespace rure_amd
