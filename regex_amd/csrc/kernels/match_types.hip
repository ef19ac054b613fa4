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

// ------------------------------------- DfaSuffix find_iter over long haystacks
// find_iter under DfaSuffix is a chain of exec_dfa_reverse_suffix searches
// (exec.rs:725-794), each from the previous match end.  With a longest
// common suffix that cannot overlap itself, every occurrence is walked, and a
// match (it ends with the suffix) ends where an occurrence ends, so the next
// search starts exactly at an occurrence end: search k = the search that
// starts right after occurrence k - 1 (or at the haystack's start), whose
// slices are [end of occurrence i - 1, end of occurrence i) for i >= k — the
// same slices for every search that reaches them.  So: (1) every occurrence
// (units, count, scan, list); (2) every slice's reverse scan, once (NEXT: it
// died inside the slice; DEC(s): a match starts at s, its end from the
// forward DFA at s; FALL: it reached the slice start, the reference's None);
// (3) per k, the first slice >= k that is not NEXT gives search k's match and
// the search after it (DEC: known; FALL: the forward DFA from k's start,
// exec.rs:773); (4) the searches the iteration makes are the path from each
// haystack's first search, marked by pointer doubling; (5) their matches
// written in order.  Work is per occurrence and parallel where the wave path
// had lane 0 walk the haystack.
enum : uint8_t { SUF_NEXT = 0, SUF_DEC = 1, SUF_FALL = 2 };

__global__ __launch_bounds__(256) void suf_count_kernel(BatchDev b, MatchDev m, uint64_t nunits, uint64_t nk,
                                                        uint64_t C, uint64_t *cnt) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, c0, c1;
    const uint8_t *base;
    unit_of(b, u, nk, C, &h, &base, &c0, &c1);
    const uint64_t lim = min(b.length, c1 + m.lcs_len - 1);  // occurrences starting in [c0, c1)
    uint64_t n = 0;
    for (uint64_t q = find_lit(base, c0, lim, m.lcs, m.lcs_len); q != NONE;
         q = find_lit(base, q + m.lcs_len, lim, m.lcs, m.lcs_len))
      ++n;
    cnt[u] = n;
  }
}

__global__ __launch_bounds__(256) void suf_list_kernel(BatchDev b, MatchDev m, uint64_t nunits, uint64_t nk,
                                                       uint64_t C, const uint64_t *off, uint64_t *occ) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, c0, c1;
    const uint8_t *base;
    unit_of(b, u, nk, C, &h, &base, &c0, &c1);
    const uint64_t lim = min(b.length, c1 + m.lcs_len - 1);
    uint64_t o = off[u];
    for (uint64_t q = find_lit(base, c0, lim, m.lcs, m.lcs_len); q != NONE;
         q = find_lit(base, q + m.lcs_len, lim, m.lcs, m.lcs_len))
      occ[o++] = q;
  }
}

// occurrence i's haystack: the last h with hfirst[h] <= i
__device__ __forceinline__ uint64_t suf_hay(const uint64_t *hfirst, uint64_t count, uint64_t i) {
  uint64_t lo = 0, hi = count;  // hfirst[lo] <= i < hfirst[hi]
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (hfirst[mid] <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}

// the index of the occurrence that ends at e in haystack h, or N
__device__ __forceinline__ uint64_t suf_idx(const uint64_t *occ, const uint64_t *hfirst, uint64_t h, uint64_t e,
                                            uint32_t L, uint64_t N) {
  uint64_t lo = hfirst[h], hi = hfirst[h + 1];
  if (e < L) return N;
  const uint64_t q = e - L;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (occ[mid] < q) lo = mid + 1;
    else hi = mid;
  }
  return lo < hfirst[h + 1] && occ[lo] == q ? lo : N;
}

// (2): each slice's reverse scan, and the forward end of a DEC slice's match
__global__ __launch_bounds__(256) void suf_rev_kernel(BatchDev b, MatchDev m, FwdDfaDev fg, RevDfaDev r, uint64_t N,
                                                      const uint64_t *occ, const uint64_t *hfirst, uint8_t *rtype,
                                                      uint64_t *dms, uint64_t *dme, uint32_t *err) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = suf_hay(hfirst, b.count, i);
    const uint8_t *base = b.hay + h * b.stride;
    const uint64_t lo = i == hfirst[h] ? b.start : occ[i - 1] + m.lcs_len, hi = occ[i] + m.lcs_len;
    uint64_t pos;
    const int k = rev_slice(r, base, lo, hi, &pos);
    uint8_t t = SUF_NEXT;
    if (k == 2) {
      atomicOr(err, 1u);  // (quit: the caller keeps the wave path)
    } else if (pos == lo) {
      t = SUF_FALL;
    } else if (k == 1) {
      t = SUF_DEC;
      LaneState L;
      lane_start(L, fg, base, b.length, pos);
      fwd_run<MODE_FIND>(L, fg, nullptr, base, b.length, pos);
      if (L.quit || L.last == NONE) atomicOr(err, 1u);
      dms[i] = pos;
      dme[i] = L.last;
    }
    rtype[i] = t;
  }
}

// suffix minimum of "the first non-NEXT slice at or after i", through a
// minimum scan of the reversed sequence
__global__ void suf_revval_kernel(uint64_t N, const uint8_t *rtype, uint64_t *vr) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < N; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = N - 1 - j;
    vr[j] = rtype[i] != SUF_NEXT ? i : N;
  }
}

// (3): search k's match (ms, me; NONE: none) and the search after it (N: none)
__global__ __launch_bounds__(256) void suf_next_kernel(BatchDev b, MatchDev m, FwdDfaDev fg, RevDfaDev r, uint64_t N,
                                                       const uint64_t *occ, const uint64_t *hfirst,
                                                       const uint8_t *rtype, const uint64_t *dms, const uint64_t *dme,
                                                       const uint64_t *sr, uint32_t *nxt, uint64_t *ms, uint64_t *me,
                                                       uint32_t *err) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < N; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = suf_hay(hfirst, b.count, k);
    const uint64_t i = sr[N - 1 - k];
    uint64_t s = NONE, e = NONE, n = N;
    if (i < hfirst[h + 1]) {  // a slice of this haystack decides
      if (rtype[i] == SUF_DEC) {
        s = dms[i];
        e = dme[i];
      } else {  // None: find_dfa_forward from the search's start (exec.rs:773)
        const uint8_t *base = b.hay + h * b.stride;
        const uint64_t p = k == hfirst[h] ? b.start : occ[k - 1] + m.lcs_len;
        uint64_t fs, fe;
        const int kk = dfa_find(fg, r, nullptr, nullptr, base, b.length, p, &fs, &fe);
        if (kk == 2) atomicOr(err, 1u);
        if (kk == 1) {
          s = fs;
          e = fe;
        }
      }
      if (e != NONE) {
        const uint64_t j = suf_idx(occ, hfirst, h, e, m.lcs_len, N);
        if (j == N) atomicOr(err, 1u);  // a match not ending at an occurrence: cannot happen
        else n = j + 1 < hfirst[h + 1] ? j + 1 : N;
      }
    }
    nxt[k] = (uint32_t)n;
    ms[k] = s;
    me[k] = e;
  }
}

// (4): pointer doubling from each haystack's first search
__global__ void suf_roots_kernel(uint64_t count, const uint64_t *hfirst, uint8_t *mark) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < count; h += (uint64_t)gridDim.x * blockDim.x)
    if (hfirst[h] < hfirst[h + 1]) mark[hfirst[h]] = 1;
}
__global__ void suf_mark_kernel(uint64_t N, const uint32_t *J, uint8_t *mark) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < N; k += (uint64_t)gridDim.x * blockDim.x)
    if (mark[k] && J[k] < N) mark[J[k]] = 1;  // (marks made this round add later path nodes: harmless)
}
__global__ void suf_jump_kernel(uint64_t N, const uint32_t *J, uint32_t *J2) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < N; k += (uint64_t)gridDim.x * blockDim.x)
    J2[k] = J[k] < N ? J[J[k]] : (uint32_t)N;
}

// (5)
__global__ void suf_emit_flag_kernel(uint64_t N, const uint8_t *mark, const uint64_t *me, uint64_t *flag) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < N; k += (uint64_t)gridDim.x * blockDim.x)
    flag[k] = mark[k] && me[k] != NONE ? 1 : 0;
}
__global__ void suf_write_kernel(uint64_t N, const uint64_t *flag, const uint64_t *pos, const uint64_t *ms,
                                 const uint64_t *me, uint64_t *out, uint64_t cap) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < N; k += (uint64_t)gridDim.x * blockDim.x)
    if (flag[k] && pos[k] < cap) {
      out[2 * pos[k]] = ms[k];
      out[2 * pos[k] + 1] = me[k];
    }
}
__global__ void suf_counts_kernel(uint64_t count, const uint64_t *hfirst, const uint64_t *pos, uint64_t *counts,
                                  uint64_t *total) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h <= count; h += (uint64_t)gridDim.x * blockDim.x) {
    if (h < count) counts[h] = pos[hfirst[h + 1]] - pos[hfirst[h]];
    else *total = pos[hfirst[count]];
  }
}

__global__ void suf_hfirst_kernel(uint64_t count, uint64_t nk, const uint64_t *off, uint64_t *hfirst) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h <= count; h += (uint64_t)gridDim.x * blockDim.x)
    hfirst[h] = off[h * nk];
}

namespace {
template <typename T, typename Op>
hipError_t scan_u64(bool inclusive, const T *in, T *out, size_t n, Op op, T init, hipStream_t st) {
  size_t tmp = 0;
  hipError_t e = inclusive ? rocprim::inclusive_scan(nullptr, tmp, in, out, n, op, st)
                           : rocprim::exclusive_scan(nullptr, tmp, in, out, init, n, op, st);
  void *buf = nullptr;
  if (e == hipSuccess) e = scratch_malloc(&buf, std::max<size_t>(tmp, 16), st);
  if (e == hipSuccess)
    e = inclusive ? rocprim::inclusive_scan(buf, tmp, in, out, n, op, st)
                  : rocprim::exclusive_scan(buf, tmp, in, out, init, n, op, st);
  if (buf) { hipError_t e2 = scratch_free(buf, st); if (e == hipSuccess) e = e2; }
  return e;
}
}  // namespace

hipError_t launch_suffix_iter(const BatchDev &b, const MatchDev &m, const FwdDfaDev &f, const RevDfaDev &r,
                              uint64_t chunk, const IterOut &o, hipStream_t st, int cus) {
  FwdDfaDev fg = f;  // global-table stepping
  fg.hot = 0;
  fg.all = 0;
  fg.stride = 1;
  const uint64_t span = b.length - b.start;
  const uint64_t nk = (span + chunk - 1) / chunk, nunits = nk * b.count;
  auto grid = [&](uint64_t n) { return (int)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, (uint64_t)cus * 8)); };
  std::vector<void *> bufs;
  auto alloc = [&](void **p, size_t bytes) {
    hipError_t e = scratch_malloc(p, std::max<size_t>(bytes, 16), st);
    if (e == hipSuccess) bufs.push_back(*p);
    return e;
  };
  auto done = [&](hipError_t e) {
    for (void *p : bufs) { hipError_t e2 = scratch_free(p, st); if (e == hipSuccess) e = e2; }
    return e;
  };
  uint64_t *cnt, *off, *hfirst, *occ, *dms, *dme, *vr, *sr, *ms, *me, *flag, *pos;
  uint8_t *rtype, *mark;
  uint32_t *nxt, *J2, *err;
  hipError_t e;
  if ((e = alloc((void **)&cnt, (nunits + 1) * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&off, (nunits + 1) * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&hfirst, (b.count + 1) * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&err, 16)) != hipSuccess) return done(e);
  if ((e = hipMemsetAsync(cnt + nunits, 0, 8, st)) != hipSuccess) return done(e);
  if ((e = hipMemsetAsync(err, 0, 4, st)) != hipSuccess) return done(e);
  hipLaunchKernelGGL(suf_count_kernel, dim3(grid(nunits)), dim3(256), 0, st, b, m, nunits, nk, chunk, cnt);
  if ((e = hipGetLastError()) != hipSuccess) return done(e);
  if ((e = scan_u64(false, cnt, off, nunits + 1, rocprim::plus<uint64_t>(), (uint64_t)0, st)) != hipSuccess)
    return done(e);
  hipLaunchKernelGGL(suf_hfirst_kernel, dim3(grid(b.count + 1)), dim3(256), 0, st, b.count, nk, off, hfirst);
  if ((e = hipGetLastError()) != hipSuccess) return done(e);
  uint64_t N = 0;
  if ((e = hipMemcpyAsync(&N, off + nunits, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return done(e);
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return done(e);
  if (N >= 0x7FFFFFFFull) return done(hipErrorNotSupported);
  const uint64_t Na = std::max<uint64_t>(N, 1);
  if ((e = alloc((void **)&occ, Na * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&rtype, Na)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&dms, Na * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&dme, Na * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&vr, Na * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&sr, Na * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&nxt, Na * 4)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&J2, Na * 4)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&ms, Na * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&me, Na * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&mark, Na)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&flag, (Na + 1) * 8)) != hipSuccess) return done(e);
  if ((e = alloc((void **)&pos, (Na + 1) * 8)) != hipSuccess) return done(e);
  if (N) {
    hipLaunchKernelGGL(suf_list_kernel, dim3(grid(nunits)), dim3(256), 0, st, b, m, nunits, nk, chunk, off, occ);
    hipLaunchKernelGGL(suf_rev_kernel, dim3(grid(N)), dim3(256), 0, st, b, m, fg, r, N, occ, hfirst, rtype, dms, dme,
                       err);
    hipLaunchKernelGGL(suf_revval_kernel, dim3(grid(N)), dim3(256), 0, st, N, rtype, vr);
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    if ((e = scan_u64(true, vr, sr, N, rocprim::minimum<uint64_t>(), (uint64_t)0, st)) != hipSuccess) return done(e);
    hipLaunchKernelGGL(suf_next_kernel, dim3(grid(N)), dim3(256), 0, st, b, m, fg, r, N, occ, hfirst, rtype, dms, dme,
                       sr, nxt, ms, me, err);
    if ((e = hipMemsetAsync(mark, 0, N, st)) != hipSuccess) return done(e);
    hipLaunchKernelGGL(suf_roots_kernel, dim3(grid(b.count)), dim3(256), 0, st, b.count, hfirst, mark);
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    // paths of at most N searches: ceil(log2 N) + 1 doublings
    uint32_t *J = nxt, *Jn = J2;
    for (uint64_t span2 = 1; span2 <= N; span2 <<= 1) {
      hipLaunchKernelGGL(suf_mark_kernel, dim3(grid(N)), dim3(256), 0, st, N, J, mark);
      hipLaunchKernelGGL(suf_jump_kernel, dim3(grid(N)), dim3(256), 0, st, N, J, Jn);
      std::swap(J, Jn);
    }
    hipLaunchKernelGGL(suf_mark_kernel, dim3(grid(N)), dim3(256), 0, st, N, J, mark);
    hipLaunchKernelGGL(suf_emit_flag_kernel, dim3(grid(N)), dim3(256), 0, st, N, mark, me, flag);
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
  }
  if ((e = hipMemsetAsync(flag + N, 0, 8, st)) != hipSuccess) return done(e);
  if ((e = scan_u64(false, flag, pos, N + 1, rocprim::plus<uint64_t>(), (uint64_t)0, st)) != hipSuccess) return done(e);
  uint32_t herr = 0;
  if ((e = hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return done(e);
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return done(e);
  if (herr) return done(hipErrorNotSupported);  // the caller keeps the wave path
  if (N) hipLaunchKernelGGL(suf_write_kernel, dim3(grid(N)), dim3(256), 0, st, N, flag, pos, ms, me, o.matches, o.cap);
  hipLaunchKernelGGL(suf_counts_kernel, dim3(grid(b.count + 1)), dim3(256), 0, st, b.count, hfirst, pos, o.counts,
                     o.total);
  note_fwd_path(-11);
  return done(hipGetLastError());
}

}  // namespace rure_amd
