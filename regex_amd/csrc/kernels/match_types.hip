// find / is_match / shortest_match batches under the reference's Literal and
// DfaSuffix match types (MatchDev, match_device.hpp): the searches whose
// results the reference's engine choice makes differ from a forward DFA
// search (exec.rs:601-625 find_literals with an anchored-start or empty
// literal searcher, exec.rs:725-794 the reverse suffix scan).  One lane per
// haystack; DfaSuffix's scans step the global DFA tables.  A search that
// quits (Unicode \b on a non-ASCII byte) leaves the quit marker for the Pike
// VM pass, as the DFA kernels do (exec.rs:507-512: find_nfa from the start).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "match_device.hpp"

namespace rure_amd {

template <int MODE>
__global__ __launch_bounds__(256) void lane_search_kernel(BatchDev bt, MatchDev m, FwdDfaDev fg, RevDfaDev r,
                                                          void *out) {
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < bt.count; h += nthreads) {
    const uint8_t *base;
    uint64_t len;
    if (bt.offs) {
      const uint64_t o0 = bt.offs[h], o1 = bt.offs[h + 1];
      base = bt.hay + o0;
      len = o1 - o0;
    } else {
      base = bt.hay + h * bt.stride;
      len = bt.length;
    }
    uint64_t ms = NONE, me = NONE;
    const int k = mt_search<MODE>(m, fg, r, base, len, bt.start, &ms, &me);
    if (k == 2 && bt.quit_flag) atomicOr(bt.quit_flag, 1u);
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = (uint8_t)k;
    } else if (MODE == MODE_SHORTEST) {
      ((uint64_t *)out)[h] = k == 2 ? QUITMARK : k == 1 ? me : NONE;
    } else {
      ((uint64_t *)out)[2 * h] = k == 2 ? QUITMARK : k == 1 ? ms : NONE;
      ((uint64_t *)out)[2 * h + 1] = k == 2 ? QUITMARK : k == 1 ? me : NONE;
    }
  }
}

// ---------------------------------------------- DfaSuffix over long haystacks
// exec_dfa_reverse_suffix (exec.rs:725-756) walks the suffix occurrences
// left to right: slice i = [end of occurrence i - 1, end of occurrence i)
// (the first from the search start), a reverse DFA over each, and the first
// slice whose scan matches, quits or reaches its slice start (None: the
// forward DFA answers) decides.  When the longest common suffix cannot
// overlap itself, the occurrences it walks are all of its occurrences, so the
// slices are known up front and their scans independent: the haystack is cut
// into units (by occurrence start), pass 1 finds each unit's last occurrence
// end, a max-scan gives each unit the end before it, pass 2 scans each
// unit's slices in order and keeps its first decisive one (atomicMin over the
// occurrence start per haystack), pass 3 answers per haystack.  One lane per
// haystack (lane_search_kernel) would walk a 16 GiB haystack alone.
struct SuffixRec {
  uint64_t q, ms, me;
  int32_t kind;  // 1 match, 2 quit, -1 None
  int32_t pad;
};

__device__ __forceinline__ void unit_of(const BatchDev &b, uint64_t u, uint64_t nk, uint64_t C, uint64_t *h,
                                        const uint8_t **base, uint64_t *c0, uint64_t *c1) {
  *h = u / nk;
  const uint64_t k = u - *h * nk;
  *base = b.hay + *h * b.stride;
  *c0 = b.start + k * C;
  *c1 = k + 1 == nk ? b.length : min(b.length, *c0 + C);
}

__global__ __launch_bounds__(256) void suffix_last_kernel(BatchDev b, MatchDev m, uint64_t nunits, uint64_t nk,
                                                          uint64_t C, uint64_t *enc) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, c0, c1;
    const uint8_t *base;
    unit_of(b, u, nk, C, &h, &base, &c0, &c1);
    uint64_t last = 0;  // end of the unit's last occurrence (0: none)
    // searched backwards, 256-byte windows from the unit's end (occurrences
    // do not overlap, so the last one in a window is the unit's last): a
    // dense suffix costs a window, not the unit
    const uint64_t lim = min(b.length, c1 + m.lcs_len - 1);  // occurrences starting before c1
    for (uint64_t we = c1; we > c0 && !last;) {
      const uint64_t ws = we - c0 > 256 ? we - 256 : c0;
      for (uint64_t q = find_lit(base, ws, min(lim, we + m.lcs_len - 1), m.lcs, m.lcs_len); q != NONE;
           q = find_lit(base, q + m.lcs_len, min(lim, we + m.lcs_len - 1), m.lcs, m.lcs_len))
        last = q + m.lcs_len;
      we = ws;
    }
    enc[u] = (h << 40) | last;
  }
}

__global__ __launch_bounds__(256) void suffix_decide_kernel(BatchDev b, MatchDev m, RevDfaDev r, uint64_t nunits,
                                                            uint64_t nk, uint64_t C, const uint64_t *scan,
                                                            SuffixRec *rec, unsigned long long *best) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, c0, c1;
    const uint8_t *base;
    unit_of(b, u, nk, C, &h, &base, &c0, &c1);
    uint64_t prev = b.start;  // the end of the occurrence before this unit's first (the search start)
    if (u % nk) {
      const uint64_t e = scan[u - 1];
      if ((e >> 40) == h && (e & ((1ull << 40) - 1))) prev = e & ((1ull << 40) - 1);
    }
    const uint64_t lim = min(b.length, c1 + m.lcs_len - 1);
    for (uint64_t q = find_lit(base, c0, lim, m.lcs, m.lcs_len); q != NONE;
         q = find_lit(base, q + m.lcs_len, lim, m.lcs, m.lcs_len)) {
      // an earlier slice already decided this haystack: the rest is moot
      if (__hip_atomic_load(&best[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < q) break;
      const uint64_t end = q + m.lcs_len;
      uint64_t pos;
      const int k = rev_slice(r, base, prev, end, &pos);
      int kind = 0;
      if (k == 2) kind = 2;
      else if (pos == prev) kind = -1;  // Match(0) | NoMatch(0): None
      else if (k == 1) kind = 1;
      if (kind) {
        SuffixRec x;
        x.q = q;
        x.ms = pos;
        x.me = end;
        x.kind = kind;
        x.pad = 0;
        rec[u] = x;
        atomicMin(&best[h], (unsigned long long)q);
        break;
      }
      prev = end;
    }
  }
}

// status per haystack: 0 answered (out written), 3 the forward DFA must answer
template <int MODE>
__global__ __launch_bounds__(256) void suffix_finish_kernel(BatchDev b, FwdDfaDev fg, uint64_t nk, uint64_t C,
                                                            const SuffixRec *rec, const unsigned long long *best,
                                                            void *out, uint8_t *status) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < b.count; h += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q = best[h];
    uint64_t ms = NONE, me = NONE;
    int k = 0;  // 0 no match, 1 match, 2 quit
    uint8_t stt = 0;
    if (q != NONE) {
      const SuffixRec x = rec[h * nk + (q - b.start) / C];
      if (x.kind == 2) {
        k = 2;
      } else if (x.kind < 0) {
        stt = 3;
      } else if (MODE != MODE_FIND) {  // shortest_dfa_reverse_suffix: the suffix end
        k = 1;
        me = x.me;
      } else {  // exec.rs:781-793: the forward DFA from the reverse scan's start
        const uint8_t *base = b.hay + h * b.stride;
        LaneState L;
        lane_start(L, fg, base, b.length, x.ms);
        fwd_run<MODE_FIND>(L, fg, nullptr, base, b.length, x.ms);
        if (L.quit) k = 2;
        else if (L.last != NONE) { k = 1; ms = x.ms; me = L.last; }
      }
    }
    status[h] = stt;
    if (stt) continue;
    if (k == 2 && b.quit_flag) atomicOr(b.quit_flag, 1u);
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = (uint8_t)k;
    } else if (MODE == MODE_SHORTEST) {
      ((uint64_t *)out)[h] = k == 2 ? QUITMARK : k == 1 ? me : NONE;
    } else {
      ((uint64_t *)out)[2 * h] = k == 2 ? QUITMARK : k == 1 ? ms : NONE;
      ((uint64_t *)out)[2 * h + 1] = k == 2 ? QUITMARK : k == 1 ? me : NONE;
    }
  }
}

hipError_t launch_suffix_long(int mode, const BatchDev &b, const MatchDev &m, const FwdDfaDev &f,
                              const RevDfaDev &r, uint64_t chunk, void *out, uint8_t *status, hipStream_t st,
                              int cus) {
  note_fwd_path(-9);
  FwdDfaDev fg = f;  // global-table stepping
  fg.hot = 0;
  fg.all = 0;
  fg.stride = 1;
  const uint64_t span = b.length - b.start;
  const uint64_t nk = (span + chunk - 1) / chunk;
  const uint64_t nunits = nk * b.count;
  uint64_t *enc = nullptr, *scan = nullptr;
  SuffixRec *rec = nullptr;
  unsigned long long *best = nullptr;
  hipError_t e = scratch_malloc((void **)&enc, nunits * 8, st);
  if (e == hipSuccess) e = scratch_malloc((void **)&scan, nunits * 8, st);
  if (e == hipSuccess) e = scratch_malloc((void **)&rec, nunits * sizeof(SuffixRec), st);
  if (e == hipSuccess) e = scratch_malloc((void **)&best, b.count * 8, st);
  if (e == hipSuccess) e = hipMemsetAsync(best, 0xFF, b.count * 8, st);
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((nunits + 255) / 256, (uint64_t)cus * 8));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(suffix_last_kernel, dim3(grid), dim3(256), 0, st, b, m, nunits, nk, chunk, enc);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    size_t tmp = 0;
    e = rocprim::inclusive_scan(nullptr, tmp, enc, scan, (size_t)nunits, rocprim::maximum<uint64_t>(), st);
    void *buf = nullptr;
    if (e == hipSuccess) e = scratch_malloc(&buf, tmp, st);
    if (e == hipSuccess) e = rocprim::inclusive_scan(buf, tmp, enc, scan, (size_t)nunits, rocprim::maximum<uint64_t>(), st);
    if (buf) { hipError_t e2 = scratch_free(buf, st); if (e == hipSuccess) e = e2; }
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(suffix_decide_kernel, dim3(grid), dim3(256), 0, st, b, m, r, nunits, nk, chunk, scan, rec, best);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    const int g2 = (int)std::max<uint64_t>(1, std::min<uint64_t>((b.count + 255) / 256, (uint64_t)cus * 8));
    if (mode == MODE_FIND)
      hipLaunchKernelGGL(suffix_finish_kernel<MODE_FIND>, dim3(g2), dim3(256), 0, st, b, fg, nk, chunk, rec, best, out,
                         status);
    else if (mode == MODE_ISMATCH)
      hipLaunchKernelGGL(suffix_finish_kernel<MODE_ISMATCH>, dim3(g2), dim3(256), 0, st, b, fg, nk, chunk, rec, best,
                         out, status);
    else
      hipLaunchKernelGGL(suffix_finish_kernel<MODE_SHORTEST>, dim3(g2), dim3(256), 0, st, b, fg, nk, chunk, rec, best,
                         out, status);
    e = hipGetLastError();
  }
  for (void *q : {(void *)enc, (void *)scan, (void *)rec, (void *)best})
    if (q) { hipError_t e2 = scratch_free(q, st); if (e == hipSuccess) e = e2; }
  return e;
}

hipError_t launch_lane_search(int mode, const BatchDev &b, const MatchDev &m, const FwdDfaDev &f,
                              const RevDfaDev &r, void *out, hipStream_t st, int cus) {
  note_fwd_path(-5);
  FwdDfaDev fg = f;  // global-table stepping (no LDS image staged)
  fg.hot = 0;
  fg.all = 0;
  fg.stride = 1;
  const uint64_t blocks = (b.count + 255) / 256;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)cus * 8));
  switch (mode) {
    case MODE_FIND:
      hipLaunchKernelGGL(lane_search_kernel<MODE_FIND>, dim3(grid), dim3(256), 0, st, b, m, fg, r, out);
      break;
    case MODE_ISMATCH:
      hipLaunchKernelGGL(lane_search_kernel<MODE_ISMATCH>, dim3(grid), dim3(256), 0, st, b, m, fg, r, out);
      break;
    default:
      hipLaunchKernelGGL(lane_search_kernel<MODE_SHORTEST>, dim3(grid), dim3(256), 0, st, b, m, fg, r, out);
      break;
  }
  return hipGetLastError();
}

}  // namespace rure_amd
