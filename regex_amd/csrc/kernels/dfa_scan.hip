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

#include <atomic>
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "dfa_device.hpp"

namespace rure_amd {

__device__ __forceinline__ void note_quit(uint32_t *flag) {
  if (flag) atomicOr(flag, 1u);
}

template <int MODE>
__device__ __forceinline__ void finish_lane(const LaneState &L, const RevDfaDev &r, const uint8_t *base,
                                            uint64_t len, uint64_t lo, uint64_t h, void *out, uint32_t *qf,
                                            const uint8_t *rlds = nullptr) {
  if (L.quit) note_quit(qf);
  if (MODE == MODE_ISMATCH) {
    ((uint8_t *)out)[h] = L.quit ? 2 : (L.last != NONE ? 1 : 0);
    return;
  }
  if (MODE == MODE_SHORTEST) {
    ((uint64_t *)out)[h] = L.quit ? QUITMARK : L.last;
    return;
  }
  uint64_t ms = NONE, me = NONE;
  if (L.quit) {
    ms = me = QUITMARK;
  } else if (L.last != NONE) {
    me = L.last;
    if (me == lo) {
      ms = lo;                              // exec.rs:647
    } else {
      const uint64_t rs = rev_scan(r, rlds, base, len, lo, me);
      if (rs == QUITMARK) note_quit(qf);
      if (rs == QUITMARK) ms = me = QUITMARK;
      else if (rs == NONE) ms = me = NONE;  // exec.rs:656-660: reverse NoMatch -> no match
      else ms = rs;
    }
  }
  ((uint64_t *)out)[2 * h] = ms;
  ((uint64_t *)out)[2 * h + 1] = me;
}

template <int MODE, bool STRIDED, bool PFX>
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
    LaneState L;
    lane_start(L, f, base, len, bt.start);
    fwd_run<MODE, PFX>(L, f, lds, base, len, bt.start);
    finish_lane<MODE>(L, r, base, len, bt.start, h, out, bt.quit_flag);
  }
}

static std::atomic<int> g_last_fwd_path{-1};
int last_fwd_path() { return g_last_fwd_path.load(); }
void note_fwd_path(int path) { g_last_fwd_path.store(path); }

// Kernel timer (bench diagnostics, rure_amd_kernel_timer): while on, the
// launches a caller brackets with ktimer_begin / ktimer_end (the find_iter
// speculative kernels) get a HIP event pair on their own stream, so the
// bench can report that kernel's average duration measured live.
namespace {
struct KTimer {
  std::mutex mu;
  bool on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t used = 0;
};
KTimer &ktimer() {
  static KTimer *t = new KTimer();
  return *t;
}
}  // namespace

void ktimer_begin(hipStream_t st) {
  KTimer &t = ktimer();
  std::lock_guard<std::mutex> g(t.mu);
  if (!t.on) return;
  if (t.used == t.ev.size()) {
    std::pair<hipEvent_t, hipEvent_t> p{nullptr, nullptr};
    if (hipEventCreate(&p.first) != hipSuccess || hipEventCreate(&p.second) != hipSuccess) return;
    t.ev.push_back(p);
  }
  (void)hipEventRecord(t.ev[t.used].first, st);
}

void ktimer_end(hipStream_t st) {
  KTimer &t = ktimer();
  std::lock_guard<std::mutex> g(t.mu);
  if (!t.on || t.used >= t.ev.size()) return;
  (void)hipEventRecord(t.ev[t.used].second, st);
  ++t.used;
}

int ktimer_set(int on) {
  KTimer &t = ktimer();
  std::lock_guard<std::mutex> g(t.mu);
  t.on = on != 0;
  t.used = 0;
  return 0;
}

double ktimer_read(uint64_t *launches) {
  KTimer &t = ktimer();
  std::lock_guard<std::mutex> g(t.mu);
  double sum = 0;
  for (size_t i = 0; i < t.used; ++i) {
    float ms = 0;
    if (hipEventSynchronize(t.ev[i].second) != hipSuccess ||
        hipEventElapsedTime(&ms, t.ev[i].first, t.ev[i].second) != hipSuccess)
      return -1.0;
    sum += ms;
  }
  if (launches) *launches = t.used;
  return t.used ? sum / (double)t.used : 0.0;
}

// ------------------------------------------------------- literal engine
// MatchType::Literal for find / is_match batches (exec.rs:601-625 find_literals,
// dispatched by exec.rs:1148-1166 when the regex is a complete finite string
// set).  The regex's literals (host/literals.hpp, leftmost-first priority
// order, non-empty, no look-around) live in the find_iter DFA's literal image;
// f must be that DFA.  One lane per haystack walks 64 start positions per
// step through the prefix-hash bitmap (lit_cands64: 64 independent LDS probes
// instead of a dependent DFA chain) and stops at the first position where a
// literal occurs: the leftmost start, and there the first literal in priority
// order is the leftmost-first match.  No reverse scan: the literal's length
// gives the end.
template <int MODE, bool STRIDED, bool K4, bool K8>
__global__ __launch_bounds__(256) void lit_find_kernel(BatchDev bt, FwdDfaDev f, void *out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint32_t i = threadIdx.x * 16; i < f.lit_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(f.lit_image + i);
  __syncthreads();
  const uint32_t *bitmap = (const uint32_t *)lds;
  const uint32_t *bitmap2 = (const uint32_t *)(lds + kLitBitmap2);
  const uint32_t kmask = K4 ? 0xFFFFFFFFu : ((1u << (8 * f.lit_k)) - 1);
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
    uint64_t ms = NONE, me = NONE;
    // candidate starts [start, iend): room for the shortest literal
    const uint64_t iend = len + 1 >= f.lit_minlen ? len + 1 - f.lit_minlen : 0;
    if (iend > bt.start) {
      const uintptr_t hi_blk = (uintptr_t)(base + len);
      const uintptr_t aend = (uintptr_t)(base + iend);
      for (uintptr_t a = (uintptr_t)(base + bt.start) & ~(uintptr_t)15; a < aend && ms == NONE; a += 64) {
        uint64_t cand = lit_cands64<K4, K8>(a, hi_blk, bitmap, bitmap2, kmask);
        const int64_t p0 = (int64_t)(a - (uintptr_t)base);
        while (cand) {
          const int j = __builtin_ctzll(cand);
          cand &= cand - 1;
          const int64_t i = p0 + j;
          if (i < (int64_t)bt.start || (uint64_t)i >= iend) continue;
          const int x = lit_verify(f, lds, base, len, (uint64_t)i);
          if (x < 0) continue;
          ms = (uint64_t)i;
          me = ms + lds[kLitLens + x];
          break;
        }
      }
    }
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = ms != NONE ? 1 : 0;
    } else {
      ((uint64_t *)out)[2 * h] = ms;
      ((uint64_t *)out)[2 * h + 1] = me;
    }
  }
}

template <int MODE, bool STRIDED>
static hipError_t launch_lit_find_m(const BatchDev &b, const FwdDfaDev &f, void *out, hipStream_t st, int grid) {
  if (f.lit_k8)
    hipLaunchKernelGGL((lit_find_kernel<MODE, STRIDED, true, true>), dim3(grid), dim3(256), kLitImage, st, b, f, out);
  else if (f.lit_k == 4)
    hipLaunchKernelGGL((lit_find_kernel<MODE, STRIDED, true, false>), dim3(grid), dim3(256), kLitImage, st, b, f, out);
  else
    hipLaunchKernelGGL((lit_find_kernel<MODE, STRIDED, false, false>), dim3(grid), dim3(256), kLitImage, st, b, f,
                       out);
  return hipGetLastError();
}

hipError_t launch_lit_find(int mode, const BatchDev &b, const FwdDfaDev &f, void *out, hipStream_t st) {
  if (!f.lit_n || (mode != MODE_FIND && mode != MODE_ISMATCH)) return hipErrorInvalidValue;
  const uint64_t blocks = (b.count + 255) / 256;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)f.cus * 32));
  g_last_fwd_path.store(-3);
  const bool strided = b.offs == nullptr;
  if (mode == MODE_FIND)
    return strided ? launch_lit_find_m<MODE_FIND, true>(b, f, out, st, grid)
                   : launch_lit_find_m<MODE_FIND, false>(b, f, out, st, grid);
  return strided ? launch_lit_find_m<MODE_ISMATCH, true>(b, f, out, st, grid)
                 : launch_lit_find_m<MODE_ISMATCH, false>(b, f, out, st, grid);
}

// ------------------------------------------------------- coalesced tiles
// Fixed-stride batches (stride % 16 == 0, search start 0, hot set <= 63
// states): a wave owns 64 consecutive haystacks and walks them in lockstep
// 128 bytes at a time.  The 8 KiB tile is fetched with coalesced loads (one
// wave-instruction = 8 haystacks x one whole 128-byte line, instead of 64
// scattered lines), transposed through a per-wave LDS buffer (rows XOR-
// swizzled so the ds_read_b128 of 16 lanes hit 16 distinct bank groups), and
// each lane then steps its own row through the DFA.  The next tile's loads
// are in flight while the current one is scanned.
static constexpr int kTileTab = 64 * kRow + 256;   // largest LDS fast table of the tile path (hot + 1 <= 64 rows)
static constexpr int kTileTabSmall = 16 * kRow + 96; // hot + 1 <= 16 rows

template <int MODE, int TAB, int STRIDE>
__global__ __launch_bounds__(256) void dfa_fwd_tile_kernel(BatchDev bt, FwdDfaDev f, RevDfaDev r, void *out,
                                                           uint64_t gscatter) {
  __shared__ __attribute__((aligned(16))) uint8_t tab[TAB];
  const uint8_t *img = STRIDE == 1 ? f.lds_image : f.lds_image_s;
  const uint32_t img_bytes = STRIDE == 1 ? f.lds_bytes : f.lds_bytes_s;
  __shared__ __attribute__((aligned(16))) uint4 stage[4][64 * 8];
  for (uint32_t i = threadIdx.x * 16; i < img_bytes; i += blockDim.x * 16)
    *(uint4 *)(tab + i) = *(const uint4 *)(img + i);
  __syncthreads();
  const uint16_t *tab16 = (const uint16_t *)(tab + 1024);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  const uint64_t L = bt.length, S = bt.stride, n = bt.count;
  const uint64_t L128 = L & ~(uint64_t)127;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const int src_h = lane >> 3, src_seg = lane & 7;
  const uint64_t ngroups = (n + 63) / 64;
  for (uint64_t gi = (uint64_t)blockIdx.x * 4 + w; gi < ngroups; gi += nwaves) {
    // Scattered group order: waves that run at the same time work on
    // haystack groups far apart in memory.  With power-of-two strides,
    // neighbouring groups progressing in lockstep concentrate the chip's
    // requests on a few HBM channels (tools/tile_diag.hip: 4.75 -> 5.38 TB/s).
    const uint64_t g = gscatter ? (gi * gscatter) % ngroups : gi;
    const uint64_t h = g * 64 + lane;
    const bool valid = h < n;
    const uint8_t *base = bt.hay + (valid ? h : 0) * S;
    LaneState L_;
    L_.last = NONE;
    L_.quit = false;
    L_.done = !valid;
    L_.s = valid ? f.start[fwd_flag_index(base, L, 0)] : f.dead;
    if (L_.s >= f.n_normal) L_.done = true;
    L_.fast = STRIDE > 1 && !L_.done && L_.s < f.hot_s;
    L_.t = L_.fast ? L_.s * f.P : 0;
    // this lane's share of each coalesced tile load: haystack g*64 + 8k + src_h,
    // 16-byte segment src_seg (rows past the batch end re-read row n-1; unused)
    uint64_t hh0 = g * 64 + src_h;
    const uint8_t *src0 = bt.hay + (hh0 < n ? hh0 : n - 1) * S + 16 * src_seg;
    const uint64_t kstep = 8 * S;                     // wave-uniform
    const uint64_t klast = (n - 1) * S + 16 * src_seg;  // clamp rows past the batch end
    uint4 n0, n1, n2, n3, n4, n5, n6, n7;
    uint64_t at = 0;
#define RURE_SRC(k) ((g * 64 + 8 * (k) + src_h < n) ? src0 + (k) * kstep : bt.hay + klast)
#define RURE_LOAD_TILE(a)                                                          \
  n0 = *(const uint4 *)(RURE_SRC(0) + (a)); n1 = *(const uint4 *)(RURE_SRC(1) + (a));  \
  n2 = *(const uint4 *)(RURE_SRC(2) + (a)); n3 = *(const uint4 *)(RURE_SRC(3) + (a));  \
  n4 = *(const uint4 *)(RURE_SRC(4) + (a)); n5 = *(const uint4 *)(RURE_SRC(5) + (a));  \
  n6 = *(const uint4 *)(RURE_SRC(6) + (a)); n7 = *(const uint4 *)(RURE_SRC(7) + (a));
#define RURE_STAGE(k, v) buf[(8 * (k) + src_h) * 8 + (src_seg ^ (((8 * (k) + src_h) >> 1) & 7))] = (v);
    if (L128) { RURE_LOAD_TILE(0) }
    const int sw = (lane >> 1) & 7;
    for (; at < L128; at += 128) {
      if (!__any(!L_.done)) break;
      // stage the tile (rows XOR-swizzled), then prefetch the next one
      RURE_STAGE(0, n0) RURE_STAGE(1, n1) RURE_STAGE(2, n2) RURE_STAGE(3, n3)
      RURE_STAGE(4, n4) RURE_STAGE(5, n5) RURE_STAGE(6, n6) RURE_STAGE(7, n7)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint64_t an = (at + 128 < L128) ? at + 128 : at;
      RURE_LOAD_TILE(an)
      uint4 cur = buf[lane * 8 + sw];
      if (STRIDE == 1) {
        // Branch-free pass over the tile's 128 bytes through the LDS table:
        // the sentinel row (`hot`) is absorbing, so a lane that leaves the
        // hot states (or is done, or starts outside them) just rides the
        // sentinel; the first chunk it entered the sentinel in and the state
        // at that chunk's start are kept with selects.  Per byte the wave
        // issues one v_mad + one ds_read_u8 and no scalar work.
        const uint32_t hot = f.hot;
        uint32_t t = (L_.done || L_.s >= hot) ? hot : L_.s;
        uint32_t bad = (L_.done || L_.s < hot) ? 8u : 0u;  // first chunk to redo exactly
        uint32_t sbad = L_.s;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const uint4 nx = buf[lane * 8 + ((m + 1 < 8 ? m + 1 : 7) ^ sw)];
          const uint32_t t0 = t;
          t = fast4(t, cur.x, tab);
          t = fast4(t, cur.y, tab);
          t = fast4(t, cur.z, tab);
          t = fast4(t, cur.w, tab);
          const bool hit = (t == hot) & (t0 != hot);
          bad = hit ? (uint32_t)m : bad;
          sbad = hit ? t0 : sbad;
          cur = nx;
        }
        if (bad < 8) {  // rare: redo exactly from the chunk that left the hot states
          L_.s = sbad;
#pragma unroll 1
          for (uint32_t m = bad; m < 8 && !L_.done; ++m) {
            const uint4 v = buf[lane * 8 + (m ^ sw)];
            const uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll 1
            for (int j = 0; j < 16 && !L_.done; ++j)
              step1<MODE>(L_, f, tab, (words[j >> 2] >> ((j & 3) * 8)) & 0xFF, at + 16 * m + j);
          }
        } else if (!L_.done) {
          L_.s = t;
        }
      } else {
#pragma unroll 1
        for (int m = 0; m < 8; ++m) {
          uint4 nx = buf[lane * 8 + ((m + 1 < 8 ? m + 1 : 7) ^ sw)];
          if (!L_.done) chunk16s<MODE, STRIDE>(L_, f, tab, tab16, cur, at + 16 * m);
          cur = nx;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#undef RURE_LOAD_TILE
#undef RURE_SRC
#undef RURE_STAGE
    if (valid) {
      if (STRIDE > 1 && L_.fast) { L_.s = L_.t / f.P; L_.fast = false; }
      at = L128;
      while (!L_.done && at < L) {
        if (STRIDE == 1) step1<MODE>(L_, f, tab, base[at], at);
        else careful_step<MODE>(L_, f, base[at], at);
        ++at;
      }
      if (!L_.done && f.eof[L_.s]) L_.last = L;
      finish_lane<MODE>(L_, r, base, L, 0, h, out, bt.quit_flag);
    }
  }
}

// ---------------------------------------------------------------- sets
// RegexSet::matches (re_set.rs:184-213 -> exec.rs:998-1038 ->
// dfa.rs:525-570 forward_many).  The reference carries Match instructions
// forward in set states (dfa.rs:984-994) and reads the answer off the last
// state (dfa.rs:1004-1015); our set DFA reports the patterns reached by each
// step instead (now_mask of the state entered, host/dfa_build.cpp), so the
// lane ORs them up: same union, far fewer states.  Only the few states that
// report matches leave the LDS fast path.
__device__ __forceinline__ bool set_careful(uint32_t &s, uint64_t &mask, const SetDfaDev &f, uint32_t b,
                                            bool &quit) {
  s = f.full[(size_t)s * 256 + b];
  if (s >= f.n_normal) {
    if (s < f.n_match_end) {
      mask |= f.now_mask[s];
      return mask == f.all;  // every pattern matched: nothing left to learn
    }
    if (s == f.quit) quit = true;
    return true;  // dead or quit
  }
  return false;
}

__device__ __forceinline__ bool set_step1(uint32_t &s, uint64_t &mask, const SetDfaDev &f, const uint8_t *lds,
                                          uint32_t b, bool &quit) {
  if (s < f.hot) {
    uint32_t t = lds[__umul24(s, kRow) + b];
    if (t != f.hot) { s = t; return false; }
  }
  return set_careful(s, mask, f, b, quit);
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
    uint64_t at = bt.start, mask = 0;
    bool quit = false, done = false;
    uint32_t s;
    if (at > len) { s = f.dead; done = true; }
    else { s = f.start[fwd_flag_index(base, len, at)]; done = s == f.dead; }
    while (!done && at < len && (((uintptr_t)(base + at)) & 15)) {
      done = set_step1(s, mask, f, lds, base[at], quit);
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
      for (int j = 0; j < 16 && !done; ++j)
        done = set_step1(s, mask, f, lds, (words[j >> 2] >> ((j & 3) * 8)) & 0xFF, quit);
      at += 16;
    }
    while (!done && at < len) {
      done = set_step1(s, mask, f, lds, base[at], quit);
      ++at;
    }
    uint64_t m;
    if (quit) note_quit(bt.quit_flag);
    if (quit) m = QUITMARK;
    else if (done) m = mask;  // dead, or every pattern already matched
    else m = mask | f.eof_mask[s];
    out[h] = m;
  }
}

// ------------------------------------------------------- sets, core form
// Large sets (C4: 64 patterns, 6511 states): the states that differ only in
// the matches their entry reports collapse into 1947 "cores", and byte
// columns into K classes, so the table of the ~1000 most reachable cores fits
// in one CU's LDS as u16 entries (next core + output code).  Each byte costs a
// class lookup (independent of the state) and one dependent u16 lookup; the
// output codes of a 16-byte chunk are collected in a 64-bit bag with one
// shift + or per byte and merged after the chunk.  A chunk that leaves the
// hot cores or meets a code that needs the global table is redone from its
// first byte against the global tables (outputs are ORed, so redoing is
// harmless).
__device__ __forceinline__ bool core_careful(uint32_t &c, uint64_t &mask, const SetCoreDev &f, uint32_t k,
                                             bool &quit) {
  const size_t i = (size_t)c * f.K + k;
  mask |= f.gout[i];
  c = f.gcore[i];
  if (c == f.dead) return true;
  if (c == f.quit) { quit = true; return true; }
  return (mask & f.all) == f.all;
}

// One lookup of the hot core table: entry (core t, class k) at LDS byte
// 256 + t * K2 + 2k — one 24-bit multiply-add (v_mad_u32_u24, full rate) and
// a u16 LDS read on the dependent chain.  The address is formed as an LDS
// (address space 3) integer: set_core_kernel has no static LDS, so its dynamic
// window starts at byte 0, and a generic pointer would cost an extra add of
// the window's base per byte.  k2 = 2k comes from the LDS class map, which
// the kernel stores doubled.
typedef __attribute__((address_space(3))) const uint16_t lds_u16_t;
__device__ __forceinline__ uint32_t core_entry(uint32_t t, uint32_t K2, uint32_t k2) {
  return *(lds_u16_t *)(uintptr_t)(256u + __umul24(t, K2) + k2);
}

// Code 63 (a report that is not one pattern < 62) takes its mask from the
// global table: the chain only sets bit 63 of the bag, and a chunk that has it
// walks its bytes again for those loads (no byte waits on a global load).
// The bags of a haystack's chunks are ORed into `codes` and decoded through
// the LDS code table once, at the end of the haystack (the mask is the OR of
// the masks of the codes seen, in any order): a per-chunk decode loop cost
// 11% of C4's time.  (The early exit when every pattern has matched is then
// taken only on the careful path; it never changes a result.)
#define RURE_CORE_CHUNK(ACTIVE)                                                         \
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};                                           \
  const uint32_t KI = 2 * f.K; /* the identity column, doubled */                      \
  uint32_t kc[16];                                                                      \
  _Pragma("unroll") for (int j = 0; j < 16; ++j) kc[j] = cls[(w[j >> 2] >> ((j & 3) * 8)) & 0xFF]; \
  _Pragma("unroll") for (int j = 0; j < 16; ++j) { /* a select, not a branch per byte */ \
    const bool act = ACTIVE;                                                            \
    kc[j] = act ? kc[j] : KI;                                                           \
  }                                                                                     \
  if (c < f.hot) {                                                                      \
    const uint32_t K2 = 2 * (f.K + 1); /* LDS rows: K classes + the identity column */ \
    uint32_t t = c;                                                                     \
    uint64_t bag = 0;                                                                   \
    _Pragma("unroll") for (int j = 0; j < 16; ++j) {                                    \
      const uint32_t e = core_entry(t, K2, kc[j]);                                      \
      bag |= 1ull << (e & 63);                                                          \
      t = e >> 6;                                                                       \
    }                                                                                   \
    if ((bag >> 63) && t != f.hot) {                                                    \
      uint32_t x = c;                                                                   \
      for (int j = 0; j < 16; ++j) {                                                    \
        const uint32_t e = core_entry(x, K2, kc[j]);                                    \
        if ((e & 63) == 63) mask |= f.gout[(size_t)x * f.K + (kc[j] >> 1)];             \
        x = e >> 6;                                                                     \
      }                                                                                 \
    }                                                                                   \
    if (t != f.hot) {                                                                   \
      codes |= bag;                                                                     \
      c = t;                                                                            \
      if (c == f.dead) return true;                                                     \
      if (c == f.quit) { quit = true; return true; }                                    \
      return false;                                                                     \
    }                                                                                   \
  }

__device__ __forceinline__ bool core_chunk16(uint32_t &c, uint64_t &mask, uint64_t &codes, const SetCoreDev &f,
                                             const uint8_t *cls, uint4 v, bool &quit) {
  RURE_CORE_CHUNK(true)
#pragma unroll 1
  for (int j = 0; j < 16; ++j)
    if (core_careful(c, mask, f, kc[j] >> 1, quit)) return true;
  return false;
}

// core_chunk16 over the bytes k in [k0, kend) of an aligned block only: the
// head and the tail of a line (lines start anywhere) cost one pass of the
// same branch-free lookup chain instead of up to 15 single steps each; the
// inactive bytes leave the core and the bag unchanged.
__device__ __forceinline__ bool core_chunk_masked(uint32_t &c, uint64_t &mask, uint64_t &codes, const SetCoreDev &f,
                                                  const uint8_t *cls, uint4 v, uint32_t k0, uint32_t kend,
                                                  bool &quit) {
  RURE_CORE_CHUNK((uint32_t)j >= k0 && (uint32_t)j < kend)
#pragma unroll 1
  for (uint32_t j = k0; j < kend; ++j)
    if (core_careful(c, mask, f, kc[j] >> 1, quit)) return true;
  return false;
}
#undef RURE_CORE_CHUNK

// byte k (0..15) of a block
__device__ __forceinline__ uint32_t block_byte(uint4 v, uint32_t k) {
  const uint32_t q = k >> 2;
  const uint32_t w = q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
  return (w >> ((k & 3) * 8)) & 0xFF;
}

// fwd_flag_index (dfa_device.hpp) from the bytes around `at`: prev = text[at-1]
// (at > 0), cur = text[at] (at < len).
__device__ __forceinline__ uint32_t fwd_flag_index_bytes(uint64_t len, uint64_t at, uint32_t prev, uint32_t cur) {
  const bool start = at == 0, end = len == 0;
  const bool start_line = at == 0 || prev == '\n';
  const bool wl = at > 0 && word_byte((uint8_t)prev);
  const bool wn = at < len && word_byte((uint8_t)cur);
  return (start ? 1u : 0u) | (end ? 2u : 0u) | (start_line ? 4u : 0u) | (end ? 8u : 0u) | (wl != wn ? 16u : 32u) |
         (wl ? 64u : 0u);
}

// One haystack's set scan with the core-form tables (the per-lane body of
// set_core_kernel): head / full / tail 16-byte chunks, the next block's load
// in flight while one is stepped.  The caller has loaded (a line ahead) hb =
// the aligned block holding text[at] and b1 = the block after it (used only
// if the haystack continues past hb); ST = the start cores in LDS.
// diagnostic stamps (set_core_kernel's PROF build, RURE_AMD_CORE_PROF=1)
__device__ __forceinline__ uint64_t core_stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <bool PROF, typename PF>
__device__ __forceinline__ uint64_t core_scan_one(const SetCoreDev &f, const uint8_t *cls, const uint64_t *MT,
                                                  const uint16_t *ST, const uint64_t *HE, const uint8_t *base,
                                                  uint64_t len, uint64_t at, uint4 hb, uint4 b1, uint32_t *qf,
                                                  uint64_t *acc, PF prefetch) {
  uint64_t t0 = 0;
  if (PROF) t0 = core_stamp();
  uint64_t mask = 0, codes = 0;
  bool quit = false, done;
  uint32_t c;
  const uint32_t k0 = (uint32_t)((uintptr_t)(base + at) & 15);
  if (at > len) { c = f.dead; done = true; }
  else {
    const uint32_t prev = at > 0 ? base[at - 1] : 0u;
    const uint32_t cur = at < len ? block_byte(hb, k0) : 0u;
    c = ST[fwd_flag_index_bytes(len, at, prev, cur)];
    done = c == f.dead;
  }
  uint4 cur = hb;
  if (!done && at < len && k0) {  // head: the rest of one aligned block
    const uint32_t kend = len - at < 16 - k0 ? k0 + (uint32_t)(len - at) : 16;
    done = core_chunk_masked(c, mask, codes, f, cls, hb, k0, kend, quit);
    at += kend - k0;
    cur = b1;
  }
  uint64_t t1 = 0;
  if (PROF) { t1 = core_stamp(); acc[0] += t1 - t0; }
  // the next block's load is in flight while this one is stepped (the
  // per-lane streams are latency-bound: one round trip per block otherwise).
  // (Tried: 128-byte windows loaded at once, 8 unrolled chunk steps: 1.21 vs
  // 0.79 ms on C4.)
  // (Tried, round 4: two blocks per round so the blocks alternate between
  // two registers instead of being moved into place: 0.625 vs 0.590 ms on C4,
  // VALU 249 M vs 254 M per launch; the kernel waits on its LDS chain, not
  // on issue. profiles/r04_c4_ab.txt)
  while (!done && at + 16 <= len) {
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (at + 16 < len) nxt = *(const uint4 *)(base + at + 16);
    done = core_chunk16(c, mask, codes, f, cls, cur, quit);
    cur = nxt;
    at += 16;
  }
  uint64_t t2 = 0;
  if (PROF) { t2 = core_stamp(); acc[1] += t2 - t1; }
  // The next lines' prologue loads go out here: vector loads complete in
  // order, so a wait for any later load would wait for them too, and from here
  // to the next line's first wait this line issues no more loads.
  prefetch();
  if (!done && at < len)  // tail: at is 16-byte aligned here
    done = core_chunk_masked(c, mask, codes, f, cls, cur, 0, (uint32_t)(len - at), quit);
  if (quit) note_quit(qf);
  if (quit) return QUITMARK;
  uint64_t t3 = 0;
  if (PROF) { t3 = core_stamp(); acc[2] += t3 - t2; }
  // codes 1..62: the LDS code table, four lookups in flight per round (MT[0]
  // is 0: a lane out of codes reads it)
  uint64_t bb = codes & 0x7FFFFFFFFFFFFFFEull;
  while (bb) {
    uint32_t i[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      i[q] = bb ? (uint32_t)__builtin_ctzll(bb) : 0u;
      bb &= bb - 1;
    }
    mask |= MT[i[0]] | MT[i[1]] | MT[i[2]] | MT[i[3]];
  }
  const uint64_t r = done ? mask : (mask | (c < f.hot ? HE[c] : f.eof[c]));
  if (PROF) { (void)__builtin_amdgcn_readfirstlane((uint32_t)r); acc[3] += core_stamp() - t3; }
  return r;
}

// MODE: 0 = fixed stride, 1 = offsets; one haystack per lane (grid-stride).
// Tried on C4 and dropped: offsets as one byte stream cut into equal units per
// lane, each lane scanning the haystacks that start in its unit (1.22 vs
// 0.79 ms: every load of a wave hits 64 distant regions); two haystacks per
// lane with interleaved chains (0.72 vs 0.68 ms: the shorter one's chain
// idles); each wave sorting 128-512 haystacks by length into rounds of 64
// similar ones (0.73-0.87 vs 0.68 ms although 80-95% instead of 66% of the
// lanes' block steps are then useful: the wave's loads spread over more lines).
// LDS byte offset of the start cores (128 x u16) after the table image; the
// hot cores' EOF masks follow them
__host__ __device__ inline uint32_t core_start_off(uint32_t lds_bytes) { return (lds_bytes + 15) & ~15u; }
__host__ __device__ inline uint32_t core_lds_total(uint32_t lds_bytes, uint32_t hot) {
  return core_start_off(lds_bytes) + 256 + 8 * hot;
}

template <int MODE, bool PROF = false>
__global__ __launch_bounds__(1024) void set_core_kernel(BatchDev bt, SetCoreDev f, uint64_t *out,
                                                        uint64_t *prof = nullptr) {
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint32_t i = threadIdx.x * 16; i < f.lds_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(f.lds_image + i);
  uint16_t *ST = (uint16_t *)(lds + core_start_off(f.lds_bytes));
  uint64_t *HE = (uint64_t *)(lds + core_start_off(f.lds_bytes) + 256);
  if (threadIdx.x < 128) ST[threadIdx.x] = f.start[threadIdx.x];
  for (uint32_t i = threadIdx.x; i < f.hot; i += blockDim.x) HE[i] = f.eof[i];
  __syncthreads();
  if (threadIdx.x < 256) lds[threadIdx.x] = (uint8_t)(2 * lds[threadIdx.x]);  // class map, doubled (K < 128)
  __syncthreads();
  const uint8_t *cls = lds;
  const uint64_t *MT = (const uint64_t *)(lds + f.mt_off);
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t at = bt.start;
  // A line's prologue is a chain of dependent loads (its offsets, then the
  // block holding its first byte): the lane loads the offsets two grid
  // strides ahead and the first two blocks one stride ahead, after the
  // current line's first body block (vector loads complete in order, so a
  // wait for that block does not wait for the prefetches), with clamped
  // addresses and no branches (a load under a branch is waited for at the
  // branch's end).  The start cores are read from LDS.
  // (past the batch: the last line's offsets, never scanned)
  // offsets of line l (MODE 0: stride; l clamped into the batch)
  auto line = [&](uint64_t l, uint64_t &o0, uint64_t &o1) {
    const uint64_t lc = l < bt.count ? l : bt.count - 1;
    if (MODE == 0) { o0 = lc * bt.stride; o1 = o0 + bt.length; return; }
    o0 = bt.offs[lc];
    o1 = bt.offs[lc + 1];
  };
  // the block holding text[at] and the one after it (if the line continues)
  auto blocks = [&](uint64_t o0, uint64_t o1, uint4 &b0, uint4 &b1) {
    const uint8_t *p = bt.hay + o0 + at;
    const uint8_t *a = p - ((uintptr_t)p & 15);
    const bool any = at < o1 - o0, more = any && (uint64_t)(a + 16 - p) < o1 - o0 - at;
    if (MODE == 0) {
      b0 = b1 = make_uint4(0, 0, 0, 0);
      if (at < bt.length) { b0 = *(const uint4 *)a; b1 = *(const uint4 *)(more ? a + 16 : a); }
      return;
    }
    const uint4 *q0 = any ? (const uint4 *)a : (const uint4 *)bt.offs;  // offs: 16 readable bytes
    b0 = *q0;
    b1 = *(more ? (const uint4 *)(a + 16) : q0);
  };
  uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= bt.count) return;
  uint64_t a0, a1, b0, b1;
  uint4 x0, x1;
  line(h, a0, a1);
  line(h + nthreads, b0, b1);
  blocks(a0, a1, x0, x1);
  for (; h < bt.count; h += nthreads) {
    uint64_t c0, c1;
    uint4 y0, y1;
    auto prefetch = [&]() {
      uint64_t tl = 0;
      if (PROF) tl = core_stamp();
      line(h + 2 * nthreads, c0, c1);
      blocks(b0, b1, y0, y1);
      if (PROF) acc[4] += core_stamp() - tl;
    };
    out[h] = core_scan_one<PROF>(f, cls, MT, ST, HE, bt.hay + a0, a1 - a0, at, x0, x1, bt.quit_flag, acc, prefetch);
    a0 = b0; a1 = b1; b0 = c0; b1 = c1; x0 = y0; x1 = y1;
  }
  if (PROF && (threadIdx.x & 63) == 0) {
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    for (int k = 0; k < 5; ++k) prof[w * 5 + k] = acc[k];
  }
}

// Visit counts per core over a sample of the batch (global tables only): the
// host then re-ranks the cores so the LDS table holds the ones this data
// visits — the adaptive counterpart of the reference's lazily filled cache
// (dfa.rs:1154-1244), with identical results whatever the ranking.
__global__ __launch_bounds__(256) void core_profile_kernel(BatchDev bt, SetCoreDev f, uint64_t count,
                                                           unsigned int *visits, unsigned int *mask_counts) {
  const uint8_t *cls = f.lds_image;  // class map = first 256 bytes of the image
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < count; h += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t *base;
    uint64_t len;
    if (bt.offs) { const uint64_t o0 = bt.offs[h], o1 = bt.offs[h + 1]; base = bt.hay + o0; len = o1 - o0; }
    else { base = bt.hay + h * bt.stride; len = bt.length; }
    if (bt.start > len) continue;
    uint32_t c = f.start[fwd_flag_index(base, len, bt.start)];
    const uint64_t end = len < bt.start + 4096 ? len : bt.start + 4096;
    for (uint64_t at = bt.start; at < end && c != f.dead && c != f.quit; ++at) {
      const size_t i = (size_t)c * f.K + cls[base[at]];
      const uint32_t m = f.mid[i];
      if (m) atomicAdd(&mask_counts[m], 1u);
      c = f.gcore[i];
      atomicAdd(&visits[c], 1u);
    }
  }
}

hipError_t launch_core_profile(const BatchDev &b, const SetCoreDev &f, uint64_t count, unsigned int *visits,
                               unsigned int *mask_counts, hipStream_t st, int cus) {
  const uint64_t blocks = (count + 255) / 256;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)cus * 4));
  hipLaunchKernelGGL(core_profile_kernel, dim3(grid), dim3(256), 0, st, b, f, count, visits, mask_counts);
  return hipGetLastError();
}

hipError_t launch_set_cores(const BatchDev &b, const SetCoreDev &f, uint64_t *out, hipStream_t st, int cus) {
  // threads per block (RURE_AMD_CORE_BS overrides, tuning); blocks per CU
  // as the LDS table allows
  int bs = 1024;
  if (knob(Knob::CoreBs) > 0) bs = std::max(64, std::min<int>(1024, (int)knob(Knob::CoreBs)));
  const int per_cu =
      std::max<int>(1, std::min<int>(2048 / bs, (int)((160u * 1024u) / core_lds_total(f.lds_bytes, f.hot))));
  const int mode = b.offs ? 1 : 0;
  const uint64_t items = b.count;
  const uint64_t blocks = (items + bs - 1) / bs;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)cus * per_cu));
  hipError_t e;
  const uint32_t lds = core_lds_total(f.lds_bytes, f.hot);  // + the start cores and hot EOF masks
  auto go = [&](auto kern) -> hipError_t {
    if (lds > 64 * 1024 &&
        (e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) !=
            hipSuccess)
      return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), lds, st, b, f, out, (uint64_t *)nullptr);
    return hipGetLastError();
  };
  if (mode == 1 && knob(Knob::CoreProf) == 1) {  // diagnostic: per-phase clock stamps
    const uint64_t nw = (uint64_t)grid * bs / 64;
    uint64_t *prof = nullptr;
    if ((e = hipMalloc(&prof, nw * 5 * 8)) != hipSuccess) return e;
    std::vector<uint64_t> hp(nw * 5);
    auto kern = set_core_kernel<1, true>;
    auto run = [&]() -> hipError_t {
      hipError_t r;
      if ((r = hipMemsetAsync(prof, 0, nw * 5 * 8, st)) != hipSuccess) return r;
      if ((r = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) !=
          hipSuccess)
        return r;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), lds, st, b, f, out, prof);
      if ((r = hipGetLastError()) != hipSuccess) return r;
      if ((r = hipMemcpyAsync(hp.data(), prof, nw * 5 * 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return r;
      return hipStreamSynchronize(st);
    };
    e = run();
    const hipError_t ef = hipFree(prof);
    if (e != hipSuccess) return e;
    if (ef != hipSuccess) return ef;
    double sum[5] = {0, 0, 0, 0, 0};
    for (uint64_t w = 0; w < nw; ++w)
      for (int k = 0; k < 5; ++k) sum[k] += (double)hp[w * 5 + k];
    fprintf(stderr, "core_prof per wave (memtime ticks): prologue+head %.0f body %.0f tail %.0f finish %.0f prefetch %.0f\n",
            sum[0] / nw, sum[1] / nw, sum[2] / nw, sum[3] / nw, sum[4] / nw);
    return hipSuccess;
  }
  if (mode == 1) note_fwd_path(-17);
  if (mode == 1) return go(set_core_kernel<1>);
  return go(set_core_kernel<0>);
}


// ------------------------------------------------------- ragged line batches
// find / is_match / shortest_match over offset batches (log lines, text
// lines): one lane per line, the line walked in 16-byte blocks as the set
// kernel walks its lines.  The head and tail blocks of a line (lines start
// and end anywhere) run the same branch-free 16-lookup chain with the bytes
// outside the line sent to the identity column kIdCol, instead of single
// steps with one global byte load each; a line's prologue (its offsets, then
// the blocks holding its first bytes) is a chain of dependent loads, so the
// lane loads the offsets two lines ahead and the first two blocks one line
// ahead, issued after the current line's body loop.  Every step is
// dfa.rs:576-764's: a block that leaves the hot states (match, dead, quit or
// cold state) is redone byte by byte against the full table.

// One 16-byte block of a line; the bytes [k0, kend) belong to the line, byte
// j sits at haystack position pos0 + j.
template <int MODE, bool MASKED>
__device__ __forceinline__ void line_block(LaneState &L, const FwdDfaDev &f, const uint8_t *lds, uint4 v,
                                           uint64_t pos0, uint32_t k0, uint32_t kend) {
  if (L.s < f.hot) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t t = L.s;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t b = (w[j >> 2] >> ((j & 3) * 8)) & 0xFF;
      if (MASKED) b = ((uint32_t)j >= k0 && (uint32_t)j < kend) ? b : kIdCol;
      t = lds[__umul24(t, kRow) + b];
    }
    if (t != f.hot) { L.s = t; return; }
  }
#pragma unroll 1
  for (uint32_t j = k0; j < kend && !L.done; ++j) step1<MODE>(L, f, lds, block_byte(v, j), pos0 + j);
}

// LDS layout of dfa_line_kernel: the forward hot table, the start states
// (128 x u16), then for find the reverse DFA's hot table (the reverse scan of
// each match steps in LDS instead of the global u16 table).
__host__ __device__ inline uint32_t line_rev_off(uint32_t f_bytes) { return core_start_off(f_bytes) + 256; }
__host__ __device__ inline uint32_t line_lds_total(int mode, uint32_t f_bytes, uint32_t r_bytes) {
  return line_rev_off(f_bytes) + (mode == MODE_FIND ? ((r_bytes + 15) & ~15u) : 0u);
}

template <int MODE>
__global__ __launch_bounds__(1024) void dfa_line_kernel(BatchDev bt, FwdDfaDev f, RevDfaDev r, void *out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint32_t i = threadIdx.x * 16; i < f.lds_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(f.lds_image + i);
  uint8_t *rlds = lds + line_rev_off(f.lds_bytes);
  if (MODE == MODE_FIND)
    for (uint32_t i = threadIdx.x * 16; i < r.lds_bytes; i += blockDim.x * 16)
      *(uint4 *)(rlds + i) = *(const uint4 *)(r.lds_image + i);
  uint16_t *ST = (uint16_t *)(lds + core_start_off(f.lds_bytes));
  if (threadIdx.x < 128) ST[threadIdx.x] = f.start[threadIdx.x];
  __syncthreads();
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t at0 = bt.start;
  auto line = [&](uint64_t h, uint64_t &o0, uint64_t &o1) {
    const uint64_t hc = h < bt.count ? h : bt.count - 1;  // past the batch: the last line, never scanned
    o0 = bt.offs[hc];
    o1 = bt.offs[hc + 1];
  };
  // the block holding text[at0] and the one after it (if the line continues),
  // clamped addresses, no branches
  auto blocks = [&](uint64_t o0, uint64_t o1, uint4 &b0, uint4 &b1) {
    const uint8_t *p = bt.hay + o0 + at0;
    const uint8_t *a = p - ((uintptr_t)p & 15);
    const bool any = at0 < o1 - o0, more = any && (uint64_t)(a + 16 - p) < o1 - o0 - at0;
    const uint4 *q0 = any ? (const uint4 *)a : (const uint4 *)bt.offs;  // offs: 16 readable bytes
    b0 = *q0;
    b1 = *(more ? (const uint4 *)(a + 16) : q0);
  };
  uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= bt.count) return;
  uint64_t a0, a1, b0, b1;
  uint4 x0, x1;
  line(h, a0, a1);
  line(h + nthreads, b0, b1);
  blocks(a0, a1, x0, x1);
  for (; h < bt.count; h += nthreads) {
    uint64_t c0, c1;
    uint4 y0, y1;
    const uint8_t *base = bt.hay + a0;
    const uint64_t len = a1 - a0;
    uint64_t at = at0;
    LaneState L;
    L.last = NONE;
    L.quit = false;
    L.fast = false;
    L.t = 0;
    L.done = false;
    const uint32_t k0 = (uint32_t)((uintptr_t)(base + at) & 15);
    if (at > len) {
      L.s = f.dead;
      L.done = true;
    } else {
      if (f.ustart1) {
        L.s = f.ustart1 - 1;
      } else {
        const uint32_t prev = at > 0 ? base[at - 1] : 0u;
        const uint32_t cur = at < len ? block_byte(x0, k0) : 0u;
        L.s = ST[fwd_flag_index_bytes(len, at, prev, cur)];
      }
      if (L.s >= f.n_normal) L.done = true;  // dead start state (dfa.rs:484)
    }
    uint4 cur = x0;
    if (!L.done && at < len && k0) {  // head: the rest of one aligned block
      const uint32_t kend = len - at < 16 - k0 ? k0 + (uint32_t)(len - at) : 16;
      line_block<MODE, true>(L, f, lds, x0, at - k0, k0, kend);
      at += kend - k0;
      cur = x1;
    }
    while (!L.done && at + 16 <= len) {  // at is 16-byte aligned here
      uint4 nxt = make_uint4(0, 0, 0, 0);
      if (at + 16 < len) nxt = *(const uint4 *)(base + at + 16);
      line_block<MODE, false>(L, f, lds, cur, at, 0, 16);
      cur = nxt;
      at += 16;
    }
    // the next lines' prologue loads (vector loads complete in order: issued
    // here, no later wait of this line waits for them)
    line(h + 2 * nthreads, c0, c1);
    blocks(b0, b1, y0, y1);
    if (!L.done && at < len) line_block<MODE, true>(L, f, lds, cur, at, 0, (uint32_t)(len - at));
    if (!L.done && f.eof[L.s]) L.last = len;  // dfa.rs:748-763
    finish_lane<MODE>(L, r, base, len, at0, h, out, bt.quit_flag, rlds);
    a0 = b0; a1 = b1; b0 = c0; b1 = c1; x0 = y0; x1 = y1;
  }
}

// whether dfa_line_kernel serves an offsets batch (RURE_AMD_LINES=0: the
// one-lane-per-haystack dfa_fwd_kernel, A/B)
static bool line_path_ok(const BatchDev &b, const FwdDfaDev &f) {
  if (b.offs == nullptr || f.all || b.count == 0) return false;
  return knob(Knob::Lines) != 0;
}

template <int MODE>
static hipError_t launch_lines_m(const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out,
                                 hipStream_t st) {
  const uint32_t lds = line_lds_total(MODE, f.lds_bytes, r.lds_bytes);
  const int bs = 1024;
  const int per_cu = std::max<int>(1, std::min<int>(2, (int)((160u * 1024u) / lds)));
  const uint64_t blocks = (b.count + bs - 1) / bs;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)f.cus * per_cu));
  auto kern = dfa_line_kernel<MODE>;
  hipError_t e;
  if (lds > 64 * 1024 &&
      (e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), lds, st, b, f, r, out);
  return hipGetLastError();
}

// ------------------------------------------------------- anchored reverse
// MatchType::DfaAnchoredReverse (exec.rs:1175-1177): a regex anchored at the
// end and not at the start matches only at the end of the text, so the
// reverse DFA runs from there over text[start..] (find_dfa_anchored_reverse,
// exec.rs:671-688; quit_after_match for is_match / shortest_match, exec.rs:
// 395-406, 442-453) and reads O(match) bytes instead of the haystack.  The
// slice hides the byte before `start` from the reverse DFA's look-behind, as
// in the reference.  One lane per haystack.
template <int MODE, bool STRIDED>
__global__ __launch_bounds__(256) void dfa_anchored_rev_kernel(BatchDev bt, RevDfaDev r, void *out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint32_t i = threadIdx.x * 16; i < r.lds_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(r.lds_image + i);
  __syncthreads();
  const uint8_t *rlds = r.lds_bytes ? lds : nullptr;
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
    const uint64_t rs = bt.start > len ? NONE : rev_scan<MODE != MODE_FIND>(r, rlds, base, len, bt.start, len);
    if (rs == QUITMARK) note_quit(bt.quit_flag);
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = rs == QUITMARK ? 2 : (rs != NONE ? 1 : 0);
    } else if (MODE == MODE_SHORTEST) {
      ((uint64_t *)out)[h] = rs == QUITMARK ? QUITMARK : (rs != NONE ? len : NONE);
    } else {
      ((uint64_t *)out)[2 * h] = rs;
      ((uint64_t *)out)[2 * h + 1] = rs == QUITMARK ? QUITMARK : (rs != NONE ? len : NONE);
    }
  }
}

template <int MODE>
static hipError_t launch_anchored_rev_m(const BatchDev &b, const RevDfaDev &r, void *out, hipStream_t st, int grid) {
  if (b.offs)
    hipLaunchKernelGGL((dfa_anchored_rev_kernel<MODE, false>), dim3(grid), dim3(256), r.lds_bytes, st, b, r, out);
  else
    hipLaunchKernelGGL((dfa_anchored_rev_kernel<MODE, true>), dim3(grid), dim3(256), r.lds_bytes, st, b, r, out);
  return hipGetLastError();
}

hipError_t launch_dfa_anchored_rev(int mode, const BatchDev &b, const RevDfaDev &r, void *out, hipStream_t st,
                                   int grid) {
  g_last_fwd_path.store(-2);
  switch (mode) {
    case MODE_FIND: return launch_anchored_rev_m<MODE_FIND>(b, r, out, st, grid);
    case MODE_ISMATCH: return launch_anchored_rev_m<MODE_ISMATCH>(b, r, out, st, grid);
    default: return launch_anchored_rev_m<MODE_SHORTEST>(b, r, out, st, grid);
  }
}

// ------------------------------------------------------------------ launch
template <int MODE, bool STRIDED>
static hipError_t launch_fwd(const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out,
                             hipStream_t st, int grid) {
  // no start-state prefix skip here: one lane per haystack, and the skip's
  // registers cost more than it saves on every pattern measured
  // (profiles/r03_prefix_ab.jsonl, "lines": 1.33 -> 1.81 ms for >[^\n]*\n)
  hipLaunchKernelGGL((dfa_fwd_kernel<MODE, STRIDED, false>), dim3(grid), dim3(256), f.lds_bytes, st, b, f, r, out);
  return hipGetLastError();
}


template <int MODE, int STRIDE>
static hipError_t launch_tile_s(const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out, hipStream_t st,
                                int grid) {
  const uint32_t bytes = STRIDE == 1 ? f.lds_bytes : f.lds_bytes_s;
  g_last_fwd_path.store(STRIDE);
  // group scatter multiplier: a prime, coprime with the group count
  const uint64_t ngroups = (b.count + 63) / 64;
  uint64_t mul = 40503;
  auto gcd = [](uint64_t a, uint64_t c) { while (c) { uint64_t t = a % c; a = c; c = t; } return a; };
  while (ngroups > 1 && gcd(mul, ngroups) != 1) mul += 2;
  if (ngroups <= 1) mul = 0;
  if (bytes <= (uint32_t)kTileTabSmall)
    hipLaunchKernelGGL((dfa_fwd_tile_kernel<MODE, kTileTabSmall, STRIDE>), dim3(grid), dim3(256), 0, st, b, f, r, out,
                       mul);
  else
    hipLaunchKernelGGL((dfa_fwd_tile_kernel<MODE, kTileTab, STRIDE>), dim3(grid), dim3(256), 0, st, b, f, r, out, mul);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_tile(const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out, hipStream_t st,
                              int grid) {
  // Latency-bound regime (few lanes per CU): fewer dependent LDS lookups per
  // byte win (multi-byte table).  Throughput regime (many lanes): fewer LDS
  // operations per byte win (byte table, one ds_read_u8 per byte).
  // (measured on C2, 1M x 4 KiB: byte table 1.03 ms, stride-4 table 1.09 ms;
  // 64-byte tiles at 7 waves/SIMD 1.18 ms — the lookups' LDS cycles bound it)
  const bool latency_bound = b.count <= (uint64_t)f.cus * 16 * 64 / 2;  // < half the resident lanes
  if (latency_bound && f.stride == 4 && f.lds_bytes_s <= (uint32_t)kTileTab) return launch_tile_s<MODE, 4>(b, f, r, out, st, grid);
  if (latency_bound && f.stride == 2 && f.lds_bytes_s <= (uint32_t)kTileTab) return launch_tile_s<MODE, 2>(b, f, r, out, st, grid);
  return launch_tile_s<MODE, 1>(b, f, r, out, st, grid);
}

bool tile_path_ok(const BatchDev &b, const FwdDfaDev &f) {
  return b.offs == nullptr && b.start == 0 && (b.stride % 16) == 0 && (((uintptr_t)b.hay) & 15) == 0 &&
         b.length <= b.stride && b.length >= 128 &&
         f.lds_bytes <= (uint32_t)kTileTab;
}

hipError_t launch_dfa_fwd(int mode, const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, void *out,
                          hipStream_t st, int grid) {
  const bool strided = b.offs == nullptr;
  if (tile_path_ok(b, f)) {
    int waves = (int)((b.count + 63) / 64);
    // one haystack group per wave (C2: 0.810 ms vs 0.818 with two groups per
    // wave, 0.84 with a persistent 4-blocks-per-CU grid)
    (void)grid;
    int tgrid = (int)std::min<uint64_t>((uint64_t)(waves + 3) / 4, (uint64_t)f.cus * 64);
    if (tgrid < 1) tgrid = 1;
    switch (mode) {
      case MODE_FIND: return launch_tile<MODE_FIND>(b, f, r, out, st, tgrid);
      case MODE_ISMATCH: return launch_tile<MODE_ISMATCH>(b, f, r, out, st, tgrid);
      default: return launch_tile<MODE_SHORTEST>(b, f, r, out, st, tgrid);
    }
  }
  if (line_path_ok(b, f)) {
    g_last_fwd_path.store(-8);
    switch (mode) {
      case MODE_FIND: return launch_lines_m<MODE_FIND>(b, f, r, out, st);
      case MODE_ISMATCH: return launch_lines_m<MODE_ISMATCH>(b, f, r, out, st);
      default: return launch_lines_m<MODE_SHORTEST>(b, f, r, out, st);
    }
  }
  g_last_fwd_path.store(0);
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
