// Batched DFA scans of automata too large for the u16 tables (BigDfaDev):
// u32 next states in column form, the hot rows in LDS, the rest read from
// global memory (L2 / Infinity Cache resident for tables of tens of MB).
//
// Reference semantics restated (src/dfa.rs): exec_at (576-764, one-byte
// delayed match flag, EOF step), exec_at_reverse (768-866, longest match
// -> leftmost start), start_flags (1415-1464); dispatch find_dfa_forward
// (exec.rs:632-662) and shortest_dfa (exec.rs:692-694).  The reference
// builds such automata lazily in a bounded cache; the host materialises them
// eagerly (dfa_build.cpp, column form) so a lane only reads tables.
//
// Execution: one lane per haystack.  A 16-byte chunk's columns come from the
// LDS column map first (independent of the state), then the dependent chain
// is one table read per byte: LDS for hot states, global otherwise.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfa_device.hpp"

namespace rure_amd {
namespace {

constexpr uint32_t kBigLdsBytes = 64 * 1024;  // hot rows (u32)

__device__ __forceinline__ uint32_t big_next(const BigDfaDev &f, const uint32_t *hot_rows, uint32_t s, uint32_t c) {
  return s < f.hot ? hot_rows[s * f.ncol + c] : f.trans[(size_t)s * f.ncol + c];
}

// Reverse scan over text[lo..me) (rev_scan with the big reverse DFA).
__device__ uint64_t big_rev_scan(const BigDfaDev &r, const uint8_t *base, uint64_t len, uint64_t lo, uint64_t me) {
  uint32_t s = r.ustart1 ? r.ustart1 - 1 : r.start[rev_flag_index(base, lo, len, me)];
  if (s == r.dead) return NONE;
  uint64_t rs = NONE;
  for (uint64_t a = me; a > lo;) {
    --a;
    s = r.trans[(size_t)s * r.ncol + r.colmap[base[a]]];
    if (s >= r.n_normal) {
      if (s < r.n_match_end) rs = a + 1;
      else return rs;  // dead (no quit state in the big automata)
    }
  }
  if (r.eof[s]) rs = lo;
  return rs;
}

template <int MODE, bool STRIDED>
__global__ __launch_bounds__(1024) void big_dfa_kernel(BatchDev bt, BigDfaDev f, BigDfaDev r, void *out) {
  __shared__ __attribute__((aligned(16))) uint32_t hot_rows[kBigLdsBytes / 4];
  __shared__ uint8_t colmap[256];
  const uint32_t nhot = f.hot * f.ncol;
  for (uint32_t i = threadIdx.x; i < nhot; i += blockDim.x) hot_rows[i] = f.trans[i];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) colmap[i] = f.colmap[i];
  __syncthreads();
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < bt.count; h += nthreads) {
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
    const uint64_t at = bt.start;
    uint64_t last = NONE;
    bool done = at > len;
    uint32_t s = f.dead;
    if (!done) {
      s = f.ustart1 ? f.ustart1 - 1 : f.start[fwd_flag_index(base, len, at)];
      done = s >= f.n_normal;  // dead start state (dfa.rs:484)
    }
    uint64_t p = at;
    // head to the 16-byte boundary, then whole chunks, then the tail
    while (!done && p < len) {
      const uintptr_t a = (uintptr_t)(base + p);
      const uint4 v = *(const uint4 *)(a & ~(uintptr_t)15);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const uint32_t j0 = (uint32_t)(a & 15);
      const uint32_t n = (uint32_t)min<uint64_t>(16 - j0, len - p);
      uint32_t cols[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) cols[j] = colmap[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
#pragma unroll
      for (uint32_t j = 0; j < 16; ++j) {
        if (j < j0 || j >= j0 + n || done) continue;
        s = big_next(f, hot_rows, s, cols[j]);
        if (s >= f.n_normal) {
          if (s < f.n_match_end) {  // dfa.rs:658-668: Match(at - 1)
            last = p + (j - j0);
            if (MODE != MODE_FIND) done = true;  // quit_after_match
          } else {
            done = true;  // dead
          }
        }
      }
      p += n;
    }
    if (!done && f.eof[s]) last = len;  // dfa.rs:748-763
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = last != NONE ? 1 : 0;
      continue;
    }
    if (MODE == MODE_SHORTEST) {
      ((uint64_t *)out)[h] = last;
      continue;
    }
    uint64_t ms = NONE, me = NONE;
    if (last != NONE) {
      me = last;
      if (me == at) {
        ms = at;  // exec.rs:647
      } else {
        const uint64_t rs = big_rev_scan(r, base, len, at, me);
        if (rs == NONE) ms = me = NONE;  // exec.rs:656-660
        else ms = rs;
      }
    }
    ((uint64_t *)out)[2 * h] = ms;
    ((uint64_t *)out)[2 * h + 1] = me;
  }
}

template <int MODE>
hipError_t launch_big_m(const BatchDev &b, const BigDfaDev &f, const BigDfaDev &r, void *out, hipStream_t st,
                        int cus) {
  const uint64_t blocks = (b.count + 1023) / 1024;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)cus * 2));
  if (b.offs)
    hipLaunchKernelGGL((big_dfa_kernel<MODE, false>), dim3(grid), dim3(1024), 0, st, b, f, r, out);
  else
    hipLaunchKernelGGL((big_dfa_kernel<MODE, true>), dim3(grid), dim3(1024), 0, st, b, f, r, out);
  return hipGetLastError();
}

// The on-demand DFA (LazyDfaDev): one lane per haystack as big_dfa_kernel;
// a lane that meets a row not built yet records where it stopped and parks
// (the host builds the rows the parked lanes need and runs another round
// from there, as the reference's lazy DFA builds a state when a search
// first steps into it, dfa.rs:910-1048).
constexpr uint32_t kLazyMatchBit = 0x80000000u, kLazyUnknownEntry = 0x7FFFFFFFu;
template <int MODE, bool STRIDED>
__global__ __launch_bounds__(1024) void lazy_dfa_kernel(BatchDev bt, LazyDfaDev f, RevDfaDev r, const LazyPark *in,
                                                        uint64_t nin, LazyPark *park, unsigned long long *npark,
                                                        void *out) {
  __shared__ __attribute__((aligned(16))) uint32_t hot_rows[kBigLdsBytes / 4];
  __shared__ uint8_t colmap[256];
  const uint32_t nhot = f.hot * f.ncol;
  for (uint32_t i = threadIdx.x; i < nhot; i += blockDim.x) hot_rows[i] = f.trans[i];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) colmap[i] = f.colmap[i];
  __syncthreads();
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x, nl = in ? nin : bt.count;
  for (uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; l < nl; l += nthreads) {
    uint64_t h = l;
    if (in) h = in[l].h;
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
    const uint64_t at = bt.start;
    uint64_t last = NONE, p = at;
    bool done = at > len, parked = false;
    uint32_t s = 0;
    if (in) {
      p = in[l].p;
      last = in[l].last;
      s = in[l].s;
    } else if (!done) {
      s = f.start[fwd_flag_index(base, len, at)];
      done = s == 0;  // dead start state (dfa.rs:484)
    }
    while (!done && p < len) {
      const uintptr_t a = (uintptr_t)(base + p);
      const uint4 v = *(const uint4 *)(a & ~(uintptr_t)15);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const uint32_t j0 = (uint32_t)(a & 15);
      const uint32_t n = (uint32_t)min<uint64_t>(16 - j0, len - p);
      uint32_t j = j0;
      for (; j < j0 + n; ++j) {
        const uint32_t c = colmap[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
        const uint32_t e = s < f.hot ? hot_rows[s * f.ncol + c] : f.trans[(size_t)s * f.ncol + c];
        if (e == kLazyUnknownEntry) {
          parked = true;
          break;
        }
        if (e == 0) {
          done = true;  // dead
          break;
        }
        s = e & ~kLazyMatchBit;
        if (e & kLazyMatchBit) {  // dfa.rs:658-668: Match(at - 1)
          last = p + (j - j0);
          if (MODE != MODE_FIND) {
            done = true;  // quit_after_match
            break;
          }
        }
      }
      p += j - j0;
      if (parked) break;
    }
    if (parked) {
      const unsigned long long k = atomicAdd(npark, 1ull);
      LazyPark x;
      x.h = h;
      x.p = p;
      x.last = last;
      x.s = s;
      x.pad = 0;
      park[k] = x;
      continue;
    }
    if (!done && f.eof[s]) last = len;  // dfa.rs:748-763
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = last != NONE ? 1 : 0;
      continue;
    }
    if (MODE == MODE_SHORTEST) {
      ((uint64_t *)out)[h] = last;
      continue;
    }
    uint64_t ms = NONE, me = NONE;
    if (last != NONE) {
      me = last;
      if (me == at) {
        ms = at;  // exec.rs:647
      } else {
        const uint64_t rs = rev_scan(r, nullptr, base, len, at, me);
        if (rs == NONE) ms = me = NONE;  // exec.rs:656-660
        else ms = rs;
      }
    }
    ((uint64_t *)out)[2 * h] = ms;
    ((uint64_t *)out)[2 * h + 1] = me;
  }
}

template <int MODE>
hipError_t launch_lazy_m(const BatchDev &b, const LazyDfaDev &f, const RevDfaDev &r, const LazyPark *in,
                         uint64_t nin, LazyPark *park, unsigned long long *npark, void *out, hipStream_t st,
                         int cus) {
  const uint64_t lanes = in ? nin : b.count;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((lanes + 1023) / 1024, (uint64_t)cus * 2));
  if (b.offs)
    hipLaunchKernelGGL((lazy_dfa_kernel<MODE, false>), dim3(grid), dim3(1024), 0, st, b, f, r, in, nin, park, npark,
                       out);
  else
    hipLaunchKernelGGL((lazy_dfa_kernel<MODE, true>), dim3(grid), dim3(1024), 0, st, b, f, r, in, nin, park, npark,
                       out);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_lazy_dfa(int mode, const BatchDev &b, const LazyDfaDev &f, const RevDfaDev &r, const LazyPark *in,
                           uint64_t nin, LazyPark *park, unsigned long long *npark, void *out, hipStream_t st,
                           int cus) {
  if (b.count == 0 || (in && nin == 0)) return hipSuccess;
  note_fwd_path(-10);
  switch (mode) {
    case MODE_FIND: return launch_lazy_m<MODE_FIND>(b, f, r, in, nin, park, npark, out, st, cus);
    case MODE_ISMATCH: return launch_lazy_m<MODE_ISMATCH>(b, f, r, in, nin, park, npark, out, st, cus);
    default: return launch_lazy_m<MODE_SHORTEST>(b, f, r, in, nin, park, npark, out, st, cus);
  }
}

uint32_t lazy_dfa_hot_rows(uint32_t ncol) { return kBigLdsBytes / 4 / std::max<uint32_t>(ncol, 1); }

uint32_t big_dfa_hot_rows(uint32_t ncol, uint32_t nstates) {
  return std::min<uint32_t>(nstates, kBigLdsBytes / 4 / std::max<uint32_t>(ncol, 1));
}

hipError_t launch_big_dfa(int mode, const BatchDev &b, const BigDfaDev &f, const BigDfaDev &r, void *out,
                          hipStream_t st, int cus) {
  if (b.count == 0) return hipSuccess;
  note_fwd_path(-6);
  switch (mode) {
    case MODE_FIND: return launch_big_m<MODE_FIND>(b, f, r, out, st, cus);
    case MODE_ISMATCH: return launch_big_m<MODE_ISMATCH>(b, f, r, out, st, cus);
    default: return launch_big_m<MODE_SHORTEST>(b, f, r, out, st, cus);
  }
}

}  // namespace rure_amd
