// Batched lazy-DFA-equivalent scan kernels for gfx950 (MI355X).
//
// Reference hot loops restated here (src/dfa.rs):
//   forward  exec_at           dfa.rs:576-764  (one-byte-delayed match, EOF step)
//   reverse  exec_at_reverse   dfa.rs:768-866  (longest match -> leftmost start)
//   dispatch find_dfa_forward  exec.rs:632-662, shortest_dfa exec.rs:692-694
//   start    start_flags(_reverse) dfa.rs:1415-1464
//
// Layout / execution model:
//   * one lane scans one haystack; lanes of a wave take consecutive haystacks,
//     so a batch of N haystacks needs N/64 waves spread over all 256 CUs;
//   * the "hot" part of the forward DFA (normal states reachable through
//     ASCII bytes, up to 255) is staged once per workgroup into LDS as a
//     256-column u8 table; row `hot` is an absorbing sentinel meaning "leave
//     the fast path" (cold state, match state, dead or quit);
//   * the fast path is one v_perm_b32 (next LDS address = state<<8 | byte)
//     plus one ds_read_u8 per byte; a 16-byte chunk that hits the sentinel is
//     re-run byte by byte from its first state against the full u16 table in
//     global memory (L2-resident), which records match ends exactly like
//     exec_at's match-state branch;
//   * haystack bytes arrive as 64-byte per-lane bursts (4 x global_load_dwordx4)
//     so every 128-byte line is consumed by one lane before it can be evicted.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfa_scan.hpp"

namespace rure_amd {

__device__ __forceinline__ bool word_byte(uint32_t b) {
  return b == '_' || (b - '0') < 10u || ((b | 0x20) - 'a') < 26u;
}

// dfa.rs:1415-1434
__device__ __forceinline__ uint32_t fwd_flag_index(const uint8_t *base, uint64_t len, uint64_t at) {
  bool start = at == 0, end = len == 0;
  bool start_line = at == 0 || base[at - 1] == '\n';
  bool wl = at > 0 && word_byte(base[at - 1]);
  bool wn = at < len && word_byte(base[at]);
  return (start ? 1u : 0u) | (end ? 2u : 0u) | (start_line ? 4u : 0u) | (end ? 8u : 0u) |
         (wl != wn ? 16u : 32u) | (wl ? 64u : 0u);
}

// dfa.rs:1440-1464, on the slice text[lo..] with the search ending at `at`.
__device__ __forceinline__ uint32_t rev_flag_index(const uint8_t *base, uint64_t lo, uint64_t len,
                                                   uint64_t at) {
  bool start = at == len, end = lo == len;
  bool start_line = at == len || base[at] == '\n';
  bool wl = at < len && word_byte(base[at]);
  bool wn = at > lo && word_byte(base[at - 1]);
  return (start ? 1u : 0u) | (end ? 2u : 0u) | (start_line ? 4u : 0u) | (end ? 8u : 0u) |
         (wl != wn ? 16u : 32u) | (wl ? 64u : 0u);
}

struct LaneState {
  uint32_t s;
  uint64_t last;   // last match end (NONE if none)
  bool done;
  bool quit;
};

static constexpr uint64_t NONE = ~0ull;
static constexpr uint64_t QUITMARK = ~0ull - 1;

// Full-table step for one byte at haystack position `pos` (careful path).
template <int MODE>
__device__ __forceinline__ void careful_step(LaneState &L, const FwdDfaDev &f, uint32_t b, uint64_t pos) {
  uint32_t s = f.full[(size_t)L.s * 256 + b];
  L.s = s;
  if (s >= f.n_normal) {
    if (s < f.n_match_end) {                 // dfa.rs:658-668: Match(at - 1)
      L.last = pos;
      if (MODE != MODE_FIND) L.done = true;  // quit_after_match
    } else if (s == f.dead) {                // dfa.rs:728-731
      L.done = true;
    } else {                                 // STATE_QUIT (dfa.rs:713-715)
      L.quit = true;
      L.done = true;
    }
  }
}

template <int MODE>
__device__ __forceinline__ void step1(LaneState &L, const FwdDfaDev &f, const uint8_t *lds,
                                      uint32_t b, uint64_t pos) {
  if (L.s < f.hot) {
    uint32_t t = lds[(L.s << 8) | b];
    if (t != f.hot) { L.s = t; return; }
  }
  careful_step<MODE>(L, f, b, pos);
}

// 4 fast-path steps on the bytes of `w` (little endian).  v_perm_b32 builds
// state<<8 | byte_k in one instruction.
__device__ __forceinline__ uint32_t fast4(uint32_t s, uint32_t w, const uint8_t *lds) {
  s = lds[__builtin_amdgcn_perm(s, w, 0x0c0c0400u)];
  s = lds[__builtin_amdgcn_perm(s, w, 0x0c0c0401u)];
  s = lds[__builtin_amdgcn_perm(s, w, 0x0c0c0402u)];
  s = lds[__builtin_amdgcn_perm(s, w, 0x0c0c0403u)];
  return s;
}

template <int MODE>
__device__ __forceinline__ void chunk16(LaneState &L, const FwdDfaDev &f, const uint8_t *lds,
                                        uint4 v, uint64_t pos) {
  if (L.s < f.hot) {
    uint32_t t = L.s;
    t = fast4(t, v.x, lds);
    t = fast4(t, v.y, lds);
    t = fast4(t, v.z, lds);
    t = fast4(t, v.w, lds);
    if (t != f.hot) { L.s = t; return; }
  }
  // Re-run the chunk exactly, byte by byte.
  uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll 1
  for (int j = 0; j < 16; ++j) {
    step1<MODE>(L, f, lds, (words[j >> 2] >> ((j & 3) * 8)) & 0xFF, pos + j);
    if (L.done) return;
  }
}

template <int MODE, bool STRIDED>
__global__ __launch_bounds__(256) void dfa_fwd_kernel(BatchDev bt, FwdDfaDev f, RevDfaDev r, void *out) {
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
      uint64_t o0 = bt.offs[h], o1 = bt.offs[h + 1];
      base = bt.hay + o0;
      len = o1 - o0;
    }
    uint64_t at = bt.start;
    LaneState L;
    L.last = NONE;
    L.done = false;
    L.quit = false;
    if (at > len) {
      L.done = true;
      L.s = f.dead;
    } else {
      L.s = f.start[fwd_flag_index(base, len, at)];
      if (L.s >= f.n_normal) L.done = true;  // dead start state (dfa.rs:484)
    }
    // head: single bytes until 16-byte aligned
    while (!L.done && at < len && (((uintptr_t)(base + at)) & 15)) {
      step1<MODE>(L, f, lds, base[at], at);
      ++at;
    }
    // body: 64-byte bursts per lane
    while (!L.done && at + 64 <= len) {
      const uint4 *p = (const uint4 *)(base + at);
      uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
      chunk16<MODE>(L, f, lds, v0, at);
      if (!L.done) chunk16<MODE>(L, f, lds, v1, at + 16);
      if (!L.done) chunk16<MODE>(L, f, lds, v2, at + 32);
      if (!L.done) chunk16<MODE>(L, f, lds, v3, at + 48);
      at += 64;
    }
    while (!L.done && at + 16 <= len) {
      uint4 v = *(const uint4 *)(base + at);
      chunk16<MODE>(L, f, lds, v, at);
      at += 16;
    }
    while (!L.done && at < len) {
      step1<MODE>(L, f, lds, base[at], at);
      ++at;
    }
    // EOF sentinel step (dfa.rs:748-763)
    if (!L.done && f.eof[L.s]) L.last = len;

    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = L.quit ? 2 : (L.last != NONE ? 1 : 0);
      continue;
    }
    if (MODE == MODE_SHORTEST) {
      ((uint64_t *)out)[h] = L.quit ? QUITMARK : L.last;
      continue;
    }
    uint64_t ms = NONE, me = NONE;
    if (L.quit) {
      ms = me = QUITMARK;
    } else if (L.last != NONE) {
      me = L.last;
      const uint64_t lo = bt.start;
      if (me == lo) {
        ms = lo;                              // exec.rs:647
      } else {
        // reverse scan over text[lo..me] (exec.rs:651-661, dfa.rs:768-866)
        uint32_t s = r.start[rev_flag_index(base, lo, len, me)];
        uint64_t rs = NONE;
        bool dead = s >= r.n_normal && s == r.dead;
        bool rq = false;
        uint64_t a = me;
        while (!dead && a > lo) {
          --a;
          s = r.full[(size_t)s * 256 + base[a]];
          if (s >= r.n_normal) {
            if (s < r.n_match_end) rs = a + 1;
            else if (s == r.dead) dead = true;
            else { rq = true; dead = true; }
          }
        }
        if (!dead && r.eof[s]) rs = lo;
        if (rq) { ms = me = QUITMARK; }
        else ms = rs;
      }
    }
    ((uint64_t *)out)[2 * h] = ms;
    ((uint64_t *)out)[2 * h + 1] = me;
  }
}

// ---------------------------------------------------------------- sets
// RegexSet::matches (re_set.rs:184-213 -> exec.rs:998-1038 ->
// dfa.rs:525-570 forward_many).  Match instructions are carried forward in
// set states (dfa.rs:984-994), so the answer is the Match set visible after
// the final EOF step (dfa.rs:1004-1015): eof_mask[final state].  Absorbing
// states ([n_normal, n_match_end)) end the scan early (dfa.rs:675-682).
__device__ __forceinline__ bool set_careful(uint32_t &s, const SetDfaDev &f, uint32_t b, bool &quit) {
  s = f.full[(size_t)s * 256 + b];
  if (s >= f.n_normal) {
    if (s == f.quit) quit = true;
    return true;
  }
  return false;
}

__device__ __forceinline__ bool set_step1(uint32_t &s, const SetDfaDev &f, const uint8_t *lds, uint32_t b,
                                          bool &quit) {
  if (s < f.hot) {
    uint32_t t = lds[(s << 8) | b];
    if (t != f.hot) { s = t; return false; }
  }
  return set_careful(s, f, b, quit);
}

template <bool STRIDED>
__global__ __launch_bounds__(256) void dfa_set_kernel(BatchDev bt, SetDfaDev f, uint64_t *out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint32_t i = threadIdx.x * 16; i < f.lds_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(f.lds_image + i);
  __syncthreads();
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < bt.count; h += nthreads) {
    const uint8_t *base;
    uint64_t len;
    if (STRIDED) { base = bt.hay + h * bt.stride; len = bt.length; }
    else { uint64_t o0 = bt.offs[h], o1 = bt.offs[h + 1]; base = bt.hay + o0; len = o1 - o0; }
    uint64_t at = bt.start;
    bool quit = false, done = false;
    uint32_t s;
    if (at > len) { s = f.dead; done = true; }
    else { s = f.start[fwd_flag_index(base, len, at)]; done = s >= f.n_normal; }
    while (!done && at < len && (((uintptr_t)(base + at)) & 15)) {
      done = set_step1(s, f, lds, base[at], quit);
      ++at;
    }
    while (!done && at + 16 <= len) {
      uint4 v = *(const uint4 *)(base + at);
      uint32_t s0 = s;
      if (s < f.hot) {
        uint32_t t = s;
        t = fast4(t, v.x, lds); t = fast4(t, v.y, lds); t = fast4(t, v.z, lds); t = fast4(t, v.w, lds);
        if (t != f.hot) { s = t; at += 16; continue; }
      }
      s = s0;
      uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll 1
      for (int j = 0; j < 16 && !done; ++j) done = set_step1(s, f, lds, (words[j >> 2] >> ((j & 3) * 8)) & 0xFF, quit);
      at += 16;
    }
    while (!done && at < len) {
      done = set_step1(s, f, lds, base[at], quit);
      ++at;
    }
    uint64_t m;
    if (quit) m = QUITMARK;
    else if (s == f.dead) m = 0;
    else m = f.eof_mask[s];
    out[h] = m;
  }
}

// ------------------------------------------------------------------ launch
template <int MODE, bool STRIDED>
static hipError_t launch_fwd(const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out,
                             hipStream_t st, int grid) {
  hipLaunchKernelGGL((dfa_fwd_kernel<MODE, STRIDED>), dim3(grid), dim3(256), f.lds_bytes, st, b, f, r, out);
  return hipGetLastError();
}

hipError_t launch_dfa_fwd(int mode, const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out,
                          hipStream_t st, int grid) {
  const bool strided = b.offs == nullptr;
  switch (mode) {
    case MODE_FIND: return strided ? launch_fwd<MODE_FIND, true>(b, f, r, out, st, grid)
                                   : launch_fwd<MODE_FIND, false>(b, f, r, out, st, grid);
    case MODE_ISMATCH: return strided ? launch_fwd<MODE_ISMATCH, true>(b, f, r, out, st, grid)
                                      : launch_fwd<MODE_ISMATCH, false>(b, f, r, out, st, grid);
    default: return strided ? launch_fwd<MODE_SHORTEST, true>(b, f, r, out, st, grid)
                            : launch_fwd<MODE_SHORTEST, false>(b, f, r, out, st, grid);
  }
}

hipError_t launch_dfa_set(const BatchDev &b, const SetDfaDev &f, uint64_t *out, hipStream_t st, int grid) {
  if (b.offs == nullptr)
    hipLaunchKernelGGL((dfa_set_kernel<true>), dim3(grid), dim3(256), f.lds_bytes, st, b, f, out);
  else
    hipLaunchKernelGGL((dfa_set_kernel<false>), dim3(grid), dim3(256), f.lds_bytes, st, b, f, out);
  return hipGetLastError();
}

}  // namespace rure_amd
