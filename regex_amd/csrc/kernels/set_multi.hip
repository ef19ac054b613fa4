// Sets as several core-form automata in one pass (MultiCoreDev): the
// reference runs one DfaMany search per haystack whatever the number of
// patterns (exec.rs:998-1038, dfa.rs:525-570); a set of more than 64
// patterns here is split into groups of 64 (one mask word each, the
// patterns a haystack matches do not depend on the other patterns), and this
// kernel steps every group's chain over each 16-byte chunk of the haystack
// read once, instead of one pass over the batch per group.
//
// Per group and chunk the step is set_core_kernel's (dfa_scan.hip): 16
// state-independent class lookups (u16 LDS map holding the row address), then
// the dependent chain of u16 LDS lookups (entry = next core << 6 | output
// code), the codes collected in a 64-bit bag and decoded at the end of the
// haystack; a chunk that leaves the hot cores is redone from its first byte
// against the global tables.  The groups' chains are independent, so they
// interleave byte by byte.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dfa_device.hpp"

namespace rure_amd {
namespace {

typedef __attribute__((address_space(3))) const uint16_t lds16_t;
typedef __attribute__((address_space(3))) const uint64_t lds64_t;
__device__ __forceinline__ uint32_t lds_u16(uint32_t a) { return *(lds16_t *)(uintptr_t)a; }
__device__ __forceinline__ uint64_t lds_u64(uint32_t a) { return *(lds64_t *)(uintptr_t)a; }

// Group g's careful step on class k from core c (global tables): returns
// true when the group is done (dead, or every pattern of it matched).
__device__ __forceinline__ bool multi_careful(const MultiGroupDev &d, uint32_t &c, uint64_t &mask, uint32_t k) {
  const size_t i = (size_t)c * d.K + k;
  mask |= d.gout[i];
  c = d.gcore[i];
  if (c == d.dead || c == d.quit) return true;
  return (mask & d.all) == d.all;
}

template <int G>
__device__ __forceinline__ void multi_chunk(const MultiCoreDev &f, uint32_t (&c)[G], uint64_t (&mask)[G],
                                            uint64_t (&codes)[G], uint32_t &live, uint32_t &quit, uint4 v,
                                            uint32_t k0, uint32_t kend) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t kc[G][16];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const MultiGroupDev &d = f.g[g];
    const uint32_t ident = d.rows_off + 2 * d.K;  // identity column: inactive bytes
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t b = (w[j >> 2] >> ((j & 3) * 8)) & 0xFF;
      const uint32_t k = d.rows_off + lds_u16(d.cls_off + 2 * b);  // (the map holds 2k)
      kc[g][j] = ((uint32_t)j >= k0 && (uint32_t)j < kend) ? k : ident;
    }
  }
  uint32_t t[G];
  uint64_t bag[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    t[g] = c[g] < f.g[g].hot ? c[g] : f.g[g].hot;
    bag[g] = 0;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t K2 = 2 * (f.g[g].K + 1);
      const uint32_t e = lds_u16(__umul24(t[g], K2) + kc[g][j]);
      bag[g] |= 1ull << (e & 63);
      t[g] = e >> 6;
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (!((live >> g) & 1u)) continue;
    const MultiGroupDev &d = f.g[g];
    if (c[g] < d.hot && t[g] != d.hot) {
      if (bag[g] >> 63) {  // code 63: masks from the global table, off the chain
        const uint32_t K2 = 2 * (d.K + 1);
        uint32_t x = c[g];
        for (int j = 0; j < 16; ++j) {
          const uint32_t e = lds_u16(__umul24(x, K2) + kc[g][j]);
          if ((e & 63) == 63) mask[g] |= d.gout[(size_t)x * d.K + ((kc[g][j] - d.rows_off) >> 1)];
          x = e >> 6;
        }
      }
      codes[g] |= bag[g];
      c[g] = t[g];
      if (c[g] == d.dead || c[g] == d.quit) live &= ~(1u << g);
      if (c[g] == d.quit) quit |= 1u << g;
      continue;
    }
    // left the hot cores (or started outside them): redo exactly
    for (uint32_t j = k0; j < kend; ++j) {
      if (multi_careful(d, c[g], mask[g], (kc[g][j] - d.rows_off) >> 1)) {
        live &= ~(1u << g);
        if (c[g] == d.quit) quit |= 1u << g;
        break;
      }
    }
  }
}

template <int G, bool STRIDED>
__global__ __launch_bounds__(1024) void set_multi_kernel(BatchDev bt, MultiCoreDev f, uint64_t *out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint32_t i = threadIdx.x * 16; i < f.lds_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(f.lds_image + i);
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
    uint32_t c[G];
    uint64_t mask[G], codes[G];
    uint32_t live = 0, quit = 0;
    uint32_t fi = 0;
    if (at <= len) {
      const uint32_t prev = at > 0 ? base[at - 1] : 0u;
      const uint32_t cur = at < len ? base[at] : 0u;
      const bool start = at == 0, end = len == 0;
      const bool wl = at > 0 && word_byte((uint8_t)prev), wn = at < len && word_byte((uint8_t)cur);
      fi = (start ? 1u : 0u) | (end ? 2u : 0u) | ((start || prev == '\n') ? 4u : 0u) | (end ? 8u : 0u) |
           (wl != wn ? 16u : 32u) | (wl ? 64u : 0u);  // dfa.rs:1415-1434
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      mask[g] = codes[g] = 0;
      c[g] = f.g[g].dead;
      if (at <= len) {
        c[g] = lds_u16(f.g[g].st_off + 2 * fi);
        if (c[g] != f.g[g].dead) live |= 1u << g;
      if (c[g] == f.g[g].quit) { live &= ~(1u << g); quit |= 1u << g; }
      }
    }
    uint64_t p = at;
    while (live && p < len) {
      const uintptr_t a = (uintptr_t)(base + p);
      const uint4 v = *(const uint4 *)(a & ~(uintptr_t)15);
      const uint32_t k0 = (uint32_t)(a & 15);
      const uint32_t kend = (uint32_t)min<uint64_t>(16, k0 + (len - p));
      multi_chunk<G>(f, c, mask, codes, live, quit, v, k0, kend);
      p += kend - k0;
    }
    uint64_t wout[kMultiMaxGroups] = {0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const MultiGroupDev &d = f.g[g];
      uint64_t m = mask[g];
      uint64_t bb = codes[g] & 0x7FFFFFFFFFFFFFFEull;
      while (bb) {
        const uint32_t i = (uint32_t)__builtin_ctzll(bb);
        bb &= bb - 1;
        m |= lds_u64(d.mt_off + 8 * i);
      }
      // the EOF step (dfa.rs:1004-1015) unless the group is done
      if (((live >> g) & 1u) && (m & d.all) != d.all)
        m |= c[g] < d.hot ? lds_u64(d.he_off + 8 * c[g]) : d.eof[c[g]];
#pragma unroll
      for (int w = 0; w < kMultiMaxGroups; ++w)
        if ((uint32_t)w == d.word) wout[w] |= m << d.shift;
    }
    if (quit) {  // the Pike VM redoes these words (unicode \b on a non-ASCII byte)
      if (bt.quit_flag) atomicOr(bt.quit_flag, 1u);
#pragma unroll
      for (int g = 0; g < G; ++g)
        if ((quit >> g) & 1u) {
#pragma unroll
          for (int w = 0; w < kMultiMaxGroups; ++w)
            if ((uint32_t)w == (f.split ? 0u : f.g[g].word)) wout[w] = QUITMARK;
        }
    }
    for (uint32_t w = 0; w < f.words; ++w) out[h * f.words + w] = wout[w < kMultiMaxGroups ? w : 0];
  }
}

template <int G>
hipError_t launch_g(const BatchDev &b, const MultiCoreDev &f, uint64_t *out, hipStream_t st, int cus) {
  const int bs = 1024;
  const uint64_t blocks = (b.count + bs - 1) / bs;
  const int per_cu = std::max<int>(1, std::min<int>(2, (int)((160u * 1024u) / std::max<uint32_t>(f.lds_bytes, 1))));
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)cus * per_cu));
  auto go = [&](auto kern) -> hipError_t {
    hipError_t e;
    if (f.lds_bytes > 64 * 1024 &&
        (e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)f.lds_bytes)) !=
            hipSuccess)
      return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), f.lds_bytes, st, b, f, out);
    return hipGetLastError();
  };
  return b.offs ? go(set_multi_kernel<G, false>) : go(set_multi_kernel<G, true>);
}

}  // namespace

hipError_t launch_set_multi(const BatchDev &b, const MultiCoreDev &f, uint64_t *out, hipStream_t st, int cus) {
  if (b.count == 0) return hipSuccess;
  if (f.words > (uint32_t)kMultiMaxGroups) return hipErrorInvalidValue;
  note_fwd_path(-7);
  switch (f.G) {
    case 1: return launch_g<1>(b, f, out, st, cus);
    case 2: return launch_g<2>(b, f, out, st, cus);
    case 3: return launch_g<3>(b, f, out, st, cus);
    case 4: return launch_g<4>(b, f, out, st, cus);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace rure_amd
