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
