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

#include "nfa_device.hpp"

namespace rure_amd {

namespace {

using namespace pike;

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
