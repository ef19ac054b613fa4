// find_iter of a regex that is one byte class repeated, C+ (\w+, [a-z]+,
// \S+, \d+, \pL+ on ASCII text): the reference's iteration (re_trait.rs:
// 197-221) restarts each search at the previous match end, and for such a
// regex the leftmost-first match from p is the maximal run of C bytes that
// begins at the first C byte at or after p (build.cpp run_class proves it on
// the find_iter DFA: the anchored automaton is the run automaton, and the
// first-byte rule holds).  So the matches are exactly the maximal runs: a run
// starts at i when text[i] is in C and text[i-1] is not (or i = start), and
// ends at the first byte after it not in C.  No DFA walk, no reverse scan:
// every byte is one LDS class lookup, independent of every other byte.
//
// A wave takes a unit of 4 KiB of one haystack, lane l its 64 bytes
// [c0 + 64 l, c0 + 64 l + 64) as four 16-byte loads; the bytes' class bits
// form a 64-bit mask per lane, run starts are mask & ~(mask << 1 | the
// previous byte's bit), and a run's end is the first zero bit after it — in
// the lane, in a later lane of the wave (a suffix minimum over the lanes), or
// past the unit (a serial look-ahead by the owning lane).  Two passes: counts
// per unit, a scan, then the records at their final places.
//
// The class table marks bytes that quit with bit 1 (the ASCII shadow of a
// Unicode class: a byte >= 0x80 may belong to a multi-byte match): any such
// byte in a unit raises the quit flag, and the caller answers the batch with
// the full automaton.
//
// A Unicode class (cp: its code point bitmap, 0x110000 bits; the table
// marks every byte >= 0x80 with bit 2) needs no quit: the Unicode-mode
// program matches only valid UTF-8 encodings of C's code points, so a byte
// is "in C" when it belongs to such an encoding, and the maximal runs of
// those bytes are again the matches (no two valid encodings overlap, and a
// run's first byte is a lead byte).  A lane holding a byte >= 0x80 (rare on
// mostly-ASCII text) decodes around each such byte: back over at most three
// continuation bytes to the lead (never before the search start: the search
// does not see earlier bytes), then the sequence's validity (no overlong
// form, no surrogate, at most U+10FFFF) and its code point's bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "dfa_scan.hpp"

namespace rure_amd {

namespace {

constexpr uint32_t kRunUnit = 4096;  // bytes per wave unit: 64 lanes x 64 bytes
constexpr uint32_t kRunWin = 256;    // records per wave staged in LDS by the emit pass (4 KiB)

// Whether byte q of the haystack at base (bytes [lo, len) visible) belongs
// to a valid UTF-8 encoding of a code point in the bitmap cp.
__device__ __noinline__ bool utf8_in_class(const uint8_t *base, uint64_t lo, uint64_t len, uint64_t q,
                                           const uint32_t *cp) {
  uint64_t p = q;
  for (int k = 0; k < 3 && p > lo && (base[p] & 0xC0) == 0x80; ++k) --p;
  const uint32_t b0 = base[p];
  uint32_t n, c;
  if (b0 >= 0xC2 && b0 <= 0xDF) n = 2, c = b0 & 0x1F;
  else if (b0 >= 0xE0 && b0 <= 0xEF) n = 3, c = b0 & 0x0F;
  else if (b0 >= 0xF0 && b0 <= 0xF4) n = 4, c = b0 & 0x07;
  else return false;  // ASCII, a continuation byte or an invalid lead
  if (p + n <= q || p + n > len) return false;
  for (uint32_t i = 1; i < n; ++i) {
    const uint32_t bi = base[p + i];
    if ((bi & 0xC0) != 0x80) return false;
    if (i == 1) {  // the second byte's range excludes overlong forms, surrogates and > U+10FFFF
      if ((b0 == 0xE0 && bi < 0xA0) || (b0 == 0xED && bi > 0x9F) || (b0 == 0xF0 && bi < 0x90) ||
          (b0 == 0xF4 && bi > 0x8F))
        return false;
    }
    c = (c << 6) | (bi & 0x3F);
  }
  return (cp[c >> 5] >> (c & 31)) & 1u;
}

// The 64 bytes of a lane at p (16-byte aligned): class bits (bit 0: in C)
// of the bytes before `len` into a 64-bit mask; *q = any byte's bits 1
// (quit) and 2 (decode: a byte >= 0x80 of a Unicode class).
__device__ __forceinline__ uint64_t run_mask(const uint8_t *cls, const uint8_t *p, uint64_t avail, uint32_t *q) {
  uint64_t m = 0;
  uint32_t qq = 0;
  const uint4 *v = (const uint4 *)p;
  uint4 blk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) blk[j] = 16u * j < avail ? v[j] : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t w[4] = {blk[j].x, blk[j].y, blk[j].z, blk[j].w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t c = cls[(w[i >> 2] >> (8 * (i & 3))) & 0xFF];
      const uint32_t pos = 16 * j + i;
      const uint32_t ok = pos < avail ? c : 0u;
      m |= (uint64_t)(ok & 1u) << pos;
      qq |= ok;
    }
  }
  *q = qq & 6u;
  return m;
}

// The decode bits of a lane whose bytes include some >= 0x80 (Unicode class).
__device__ __noinline__ uint64_t run_mask_utf8(uint64_t m, const uint8_t *base, uint64_t s0, uint64_t lo,
                                               uint64_t len, const uint32_t *cp) {
  for (uint32_t i = 0; i < 64 && s0 + i < len; ++i)
    if (base[s0 + i] >= 0x80 && utf8_in_class(base, lo, len, s0 + i, cp)) m |= 1ull << i;
  return m;
}

// EMIT = false: the runs starting in each unit (ucount) and the first byte
// not in C of each unit as a batch position (ufz: h * stride + i; the
// haystack's last unit at most its end; 2^63: none), the quit flag.
// EMIT = true: the records, a run that continues past its unit ending at the
// first byte not in C after the unit (ufz suffix minima: uzs).
template <bool EMIT>
__global__ __launch_bounds__(256) void run_iter_kernel(BatchDev b, const uint8_t *cls_g, const uint32_t *cp,
                                                       uint64_t nk, uint64_t nunits, uint64_t *ucount, uint64_t *ufz,
                                                       const uint64_t *uoff, const uint64_t *uzs, uint64_t *matches,
                                                       uint64_t cap, uint32_t *quit) {
  __shared__ uint8_t cls[256];
  // EMIT: a window of kRunWin records per wave, written to LDS by the lanes
  // that own them and copied out as whole 1 KiB stores (lanes write their
  // runs' records at scattered indices, 16 B at a time otherwise)
  __shared__ uint4 recs[EMIT ? 4 * kRunWin : 1];
  if (threadIdx.x < 256) cls[threadIdx.x] = cls_g[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint4 *wrec = recs + (EMIT ? (threadIdx.x >> 6) * kRunWin : 0);
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t u = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); u < nunits; u += nwaves) {
    const uint64_t h = u / nk, k = u - h * nk;
    const uint8_t *base = b.hay + h * b.stride;
    const uint64_t len = b.length;
    const uint64_t c0 = b.start + k * kRunUnit;
    const uint64_t s0 = c0 + 64 * (uint64_t)lane;
    const uint64_t avail = s0 < len ? len - s0 : 0;
    uint32_t q = 0;
    uint64_t m = run_mask(cls, base + s0, avail, &q);
    if (q & 4u) m = run_mask_utf8(m, base, s0, b.start, len, cp);
    // the byte before the lane's first: lane l - 1's bit 63; lane 0 reads it
    // (not in C at the search start: the search begins there)
    uint64_t pm = (uint64_t)__shfl_up((unsigned)(m >> 63), 1);
    if (lane == 0) {
      pm = 0;
      if (c0 > b.start && c0 - 1 < len) {
        const uint32_t x = cls[base[c0 - 1]];
        pm = (x & 4u) ? (utf8_in_class(base, b.start, len, c0 - 1, cp) ? 1u : 0u) : (x & 1u);
      }
    }
    const uint64_t starts = m & ~((m << 1) | pm);
    const uint32_t n = (uint32_t)__popcll(starts);
    const uint64_t nz = ~m;  // (bytes past the haystack are not in C)
    const uint64_t fz = nz ? s0 + (uint64_t)__builtin_ctzll(nz) : (1ull << 63);
    if (!EMIT) {
      if (__any((q & 2u) != 0)) {
        if (lane == 0) atomicOr(quit, 1u);
      }
      uint32_t tot = n;
      uint64_t mz = fz;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        tot += __shfl_xor(tot, o);
        mz = min(mz, (uint64_t)__shfl_xor(mz, o));
      }
      if (k + 1 == nk) mz = min(mz, len);
      if (lane == 0) {
        ucount[u] = tot;
        ufz[u] = mz == (1ull << 63) ? mz : h * b.stride + mz;
      }
      continue;
    }
    // the record index of this lane's first run in the unit: the runs of the
    // lanes before it
    uint32_t incl = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o);
      if (lane >= (uint32_t)o) incl += x;
    }
    const uint32_t T = __shfl(incl, 63);  // the unit's runs
    const uint64_t at0 = uoff[u];
    const bool a16 = ((uintptr_t)matches & 15) == 0;
    uint32_t r = incl - n;
    // the first byte not in C in the lanes after this one (suffix minimum)
    uint64_t after = __shfl_down(fz, 1);
    if (lane == 63) after = 1ull << 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t x = __shfl_down(after, o);
      if (lane + o < 64) after = min(after, x);
    }
    uint64_t st = starts;
    for (uint32_t w0 = 0; w0 < T; w0 += kRunWin) {
      while (st && r < w0 + kRunWin) {  // this lane's records in the window
        const uint32_t i = (uint32_t)__builtin_ctzll(st);
        st &= st - 1;
        const uint64_t rest = nz >> i;  // bit 0 = byte i itself (in C)
        uint64_t e;
        if (rest) {
          e = s0 + i + (uint64_t)__builtin_ctzll(rest);
        } else if (after != (1ull << 63)) {
          e = after;
        } else if (k + 1 == nk) {  // the haystack's last unit: its end
          e = len;
        } else {  // the run continues past the unit
          e = uzs[u + 1] - h * b.stride;
        }
        if (e > len) e = len;
        const uint64_t sp = s0 + i;
        wrec[r - w0] = make_uint4((uint32_t)sp, (uint32_t)(sp >> 32), (uint32_t)e, (uint32_t)(e >> 32));
        ++r;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint32_t nrec = min(kRunWin, T - w0);
      for (uint32_t j = lane; j < nrec; j += 64) {
        const uint64_t g = at0 + w0 + j;
        if (g < cap) {
          const uint4 v = wrec[j];
          if (a16) {
            *(uint4 *)(matches + 2 * g) = v;
          } else {  // records only 8-byte aligned
            matches[2 * g] = (uint64_t)v.x | (uint64_t)v.y << 32;
            matches[2 * g + 1] = (uint64_t)v.z | (uint64_t)v.w << 32;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

// counts[h] = the runs of haystack h (its units' counts), *total = all
__global__ void run_counts_kernel(uint64_t n, uint64_t nk, const uint64_t *uoff, uint64_t *counts, uint64_t *total) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h <= n; h += (uint64_t)gridDim.x * blockDim.x) {
    if (h < n) counts[h] = uoff[(h + 1) * nk] - uoff[h * nk];
    else *total = uoff[n * nk];
  }
}

}  // namespace

hipError_t exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t st);

// Fixed-stride batches whose searched bytes start 16-byte aligned (single
// haystacks from start 0).  quit (host) = a byte with the quit class was
// read: the results are then not the answer (one read-back of a flag).
hipError_t launch_find_iter_runs(const BatchDev &b, const uint8_t *cls, const uint32_t *cp, const IterOut &o,
                                 hipStream_t st, int cus, bool can_quit, bool *quit) {
  if (quit) *quit = false;
  if (b.offs || (((uintptr_t)(b.hay + b.start)) & 15) || (b.count > 1 && (b.stride & 15)))
    return hipErrorNotSupported;
  const uint64_t span = b.length > b.start ? b.length - b.start : 0;
  const uint64_t nk = std::max<uint64_t>(1, (span + kRunUnit - 1) / kRunUnit);
  const uint64_t nunits = b.count * nk;
  uint64_t *buf = nullptr;
  // unit counts and their offsets (nunits + 1 each), first non-C bytes and
  // their suffix minima (nunits each), the quit flag
  hipError_t e = scratch_malloc((void **)&buf, (4 * (nunits + 1) + 2) * 8, st);
  if (e != hipSuccess) return e;
  uint64_t *ucount = buf, *uoff = buf + nunits + 1, *ufz = uoff + nunits + 1, *uzs = ufz + nunits + 1;
  uint32_t *qf = (uint32_t *)(uzs + nunits + 1);
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((nunits + 3) / 4, (uint64_t)cus * 8));
  void *tmp = nullptr;
  do {
    if ((e = hipMemsetAsync(ucount + nunits, 0, 8, st)) != hipSuccess) break;
    if ((e = hipMemsetAsync(qf, 0, 4, st)) != hipSuccess) break;
    hipLaunchKernelGGL(run_iter_kernel<false>, dim3(grid), dim3(256), 0, st, b, cls, cp, nk, nunits, ucount, ufz,
                       (const uint64_t *)nullptr, (const uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t)0, qf);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if (can_quit && quit) {
      uint32_t hq = 0;
      if ((e = hipMemcpyAsync(&hq, qf, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) break;
      if ((e = hipStreamSynchronize(st)) != hipSuccess) break;
      if (hq) { *quit = true; break; }
    }
    if ((e = exclusive_scan_u64(ucount, uoff, nunits + 1, st)) != hipSuccess) break;
    {  // uzs[u] = min(ufz[u..]): a suffix scan as a scan of the reversed sequence
      auto in = rocprim::make_reverse_iterator(ufz + nunits);
      auto out = rocprim::make_reverse_iterator(uzs + nunits);
      size_t tb = 0;
      if ((e = rocprim::inclusive_scan(nullptr, tb, in, out, (size_t)nunits, rocprim::minimum<uint64_t>(), st)) !=
          hipSuccess)
        break;
      if ((e = scratch_malloc(&tmp, tb, st)) != hipSuccess) break;
      if ((e = rocprim::inclusive_scan(tmp, tb, in, out, (size_t)nunits, rocprim::minimum<uint64_t>(), st)) !=
          hipSuccess)
        break;
    }
    hipLaunchKernelGGL(run_iter_kernel<true>, dim3(grid), dim3(256), 0, st, b, cls, cp, nk, nunits, ucount, ufz, uoff,
                       uzs, o.matches, o.cap, qf);
    if ((e = hipGetLastError()) != hipSuccess) break;
    const int g2 = (int)std::max<uint64_t>(1, std::min<uint64_t>((b.count + 256) / 256, (uint64_t)cus * 4));
    hipLaunchKernelGGL(run_counts_kernel, dim3(g2), dim3(256), 0, st, b.count, nk, uoff, o.counts, o.total);
    e = hipGetLastError();
  } while (false);
  if (tmp) { hipError_t e3 = scratch_free(tmp, st); if (e == hipSuccess) e = e3; }
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

}  // namespace rure_amd
