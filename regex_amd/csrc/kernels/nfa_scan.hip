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
  // the DFA pass flagged no quit: nothing to redo
  if (FALLBACK && bt.quit_flag && __atomic_load_n(bt.quit_flag, __ATOMIC_RELAXED) == 0) return;
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
      else need = ((const uint64_t *)out)[hh * bt.out_stride] == QUITMARK;
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
          ((uint64_t *)out)[h * bt.out_stride] = r0;
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


// ------------------------------------------------------------- captures
// Thread lists carry one capture-slot row per thread (pikevm.rs Threads::caps).
// A thread added from a closure entry inherits its parent's row with the
// entry's Saves set to the position of the add (add_step's Save arm,
// pikevm.rs:326-335); root threads start from the caller's slots, which are
// all unset until the first match (after which a single regex adds no more
// root threads).  A Match copies the thread's row to the output
// (pikevm.rs:250-256).
__device__ uint32_t append_caps(const NfaDev &nf, uint32_t cid, uint32_t holds, const uint64_t *pcaps, uint64_t at,
                                uint32_t *stamp, uint32_t tag, uint32_t *lleaf, uint64_t *lcaps, uint32_t ns,
                                uint32_t cnt) {
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
      while (pass && pv) {
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
      uint64_t *row = lcaps + (size_t)pos * ns;
      for (uint32_t i = 0; i < ns; ++i) row[i] = pcaps ? pcaps[i] : NONE;
      for (uint32_t q = nf.save_off[k], qe = nf.save_off[k + 1]; q < qe; ++q) {
        const uint32_t sl = nf.save_slot[q];
        if (sl < ns) row[sl] = at;
      }
    }
    cnt += (uint32_t)__popcll(bal);
    wave_sync();
  }
  return cnt;
}

// pikevm.rs:130-223 with slots (one regex, quit_after_match = false).
__device__ void pike_caps(const NfaDev &nf, uint32_t *stamp, uint32_t *leaf[2], uint64_t *caps[2], uint32_t ns,
                          TagGen &tg, const uint8_t *text, uint64_t len, uint64_t start, uint64_t *out) {
  const uint32_t lane = lane_id();
  if (start > len) return;
  bool matched = false;
  int c = 0;
  uint32_t nc = 0, ctag = tg.next(stamp, nf.nleaves);
  uint64_t at = start;
  while (true) {
    if (nc == 0 && (matched || (at != 0 && nf.anchored))) break;
    if (nc == 0 || (!nf.anchored && !matched))
      nc = append_caps(nf, nf.root, look_holds(text, len, at, nf), nullptr, at, stamp, ctag, leaf[c], caps[c], ns, nc);
    const uint32_t b = at < len ? text[at] : 0x100u;
    const uint32_t ntag = tg.next(stamp, nf.nleaves);
    const uint32_t hnx = at < len ? look_holds(text, len, at + 1, nf) : 0;
    uint32_t nn = 0;
    bool stop = false;
    for (uint32_t j0 = 0; j0 < nc && !stop; j0 += 64) {
      const uint32_t j = j0 + lane;
      const bool valid = j < nc;
      uint32_t w0 = 0;
      if (valid) w0 = nf.leaves[3 * leaf[c][j]];
      const bool is_m = valid && (w0 & 0xFF) == 1;
      const uint32_t lo = (w0 >> 8) & 0xFF, hi = (w0 >> 16) & 0xFF;
      const bool acc = valid && (w0 & 0xFF) == 0 && b >= lo && b <= hi;
      const uint64_t mb = __ballot(is_m);
      uint64_t ab = __ballot(acc);
      if (mb) {
        const uint32_t t = (uint32_t)__builtin_ctzll(mb);
        const uint64_t *row = caps[c] + (size_t)(j0 + t) * ns;
        for (uint32_t i = lane; i < ns; i += 64) out[i] = row[i];
        matched = true;
        ab &= (1ull << t) - 1;  // leftmost-first: lower-priority threads are cut
        stop = true;
      }
      while (ab) {
        const uint32_t t = (uint32_t)__builtin_ctzll(ab);
        ab &= ab - 1;
        const uint32_t cid = nf.leaves[3 * leaf[c][j0 + t] + 1];
        nn = append_caps(nf, cid, hnx, caps[c] + (size_t)(j0 + t) * ns, at + 1, stamp, ntag, leaf[c ^ 1],
                         caps[c ^ 1], ns, nn);
      }
    }
    if (at >= len) break;
    ++at;
    c ^= 1;
    nc = nn;
    ctag = ntag;
  }
}

// utf8.rs:24-39
__device__ __forceinline__ uint64_t next_utf8(const uint8_t *t, uint64_t len, uint64_t i) {
  if (i >= len) return i + 1;
  const uint32_t b = t[i];
  return i + (b <= 0x7F ? 1 : b <= 0xDF ? 2 : b <= 0xEF ? 3 : 4);
}

// exec.rs:555-567 + 861-875: with a DFA match (s, e) the NFA runs from s
// over text[..min(next_utf8(next_utf8(e)), len)]; where the DFA quit, or for
// an anchored-start program, over the whole haystack from `start`.
template <bool STRIDED>
__global__ __launch_bounds__(64) void caps_kernel(BatchDev bt, NfaDev nf, const uint64_t *found, uint64_t *slots,
                                                  uint32_t ns, uint8_t *scratch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t N = nf.nleaves;
  uint8_t *mem = scratch ? scratch + (size_t)blockIdx.x * caps_wave_bytes(N, ns) : lds;
  uint64_t *caps[2];
  caps[0] = (uint64_t *)mem;
  caps[1] = caps[0] + (size_t)N * ns;
  uint32_t *stamp = (uint32_t *)(caps[1] + (size_t)N * ns);
  uint32_t *leaf[2] = {stamp + N, stamp + 2 * N};
  const uint32_t lane = lane_id();
  for (uint32_t i = lane; i < N; i += 64) stamp[i] = 0xFFFFFFFFu;
  wave_sync();
  TagGen tg;
  for (uint64_t h = blockIdx.x; h < bt.count; h += gridDim.x) {
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
    uint64_t *o = slots + h * ns;
    for (uint32_t i = lane; i < ns; i += 64) o[i] = NONE;
    uint64_t n = len, st = bt.start;
    if (found) {
      const uint64_t fs = found[2 * h];
      if (fs == NONE) continue;
      if (fs != QUITMARK) {
        const uint64_t e = found[2 * h + 1];
        const uint64_t lim = next_utf8(base, len, next_utf8(base, len, e));
        n = lim < len ? lim : len;
        st = fs;
      }
    }
    pike_caps(nf, stamp, leaf, caps, ns, tg, base, n, st, o);
  }
}

template <bool STRIDED>
hipError_t launch_caps_s(const BatchDev &b, const NfaDev &n, const uint64_t *found, uint64_t *slots, uint32_t ns,
                         void *scratch, hipStream_t st, int grid) {
  const size_t lds = scratch ? 0 : caps_wave_bytes(n.nleaves, ns);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void *)caps_kernel<STRIDED>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((caps_kernel<STRIDED>), dim3(grid), dim3(64), lds, st, b, n, found, slots, ns,
                     (uint8_t *)scratch);
  return hipGetLastError();
}
}  // namespace

hipError_t launch_captures(const BatchDev &b, const NfaDev &n, const uint64_t *found, uint64_t *slots,
                           uint32_t nslots, void *scratch, hipStream_t st, int grid) {
  return b.offs ? launch_caps_s<false>(b, n, found, slots, nslots, scratch, st, grid)
                : launch_caps_s<true>(b, n, found, slots, nslots, scratch, st, grid);
}

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
