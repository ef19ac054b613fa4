// Diagnostic (not part of the library): bank-conflict granularity and
// dependent-chain latency of ds_read_u8 on gfx950, for the DFA lookup
// layout.  Run under rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS to read
// the extra cycles per pattern; the kernel also reports cycles per dependent
// lookup (s_memtime) for one wave per CU and for 16 waves per CU.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lds_probe.hip -o /tmp/lds_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

// pattern: 0 same byte (broadcast), 1 byte lane&3 of dword 0, 2 byte lane
// (4 lanes per dword), 3 dword lane*32 (same bank, 32-way), 4 printable byte
// of a 304-pitch row, state spread lane%S over rows
template <int PAT>
__global__ __launch_bounds__(1024) void probe(uint32_t iters, uint32_t rows, uint64_t *cyc, uint32_t *sink, uint32_t fill) {
  __shared__ uint8_t t[64 * 304 + 4096];
  for (uint32_t i = threadIdx.x; i < sizeof(t); i += blockDim.x) t[i] = (uint8_t)(fill >> (i & 31));
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = lane * 2654435761u + blockIdx.x;
  uint32_t s = 0;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (uint32_t i = 0; i < iters; ++i) {
    x = x * 1664525u + 1013904223u;
    uint32_t a;
    if (PAT == 0) a = 5;
    else if (PAT == 1) a = lane & 3;
    else if (PAT == 2) a = lane;
    else if (PAT == 3) a = (lane & 31) * 128;
    else {
      const uint32_t b = 32 + (x >> 8) % 95;
      const uint32_t row = rows > 1 ? ((x >> 20) % 16 == 0 ? 1 + (x >> 24) % (rows - 1) : 0) : 0;
      a = row * 304 + b;
    }
    s = t[a + s];  // s stays 0: table is zero; keeps the chain dependent
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0 && threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  if (s == 123) sink[0] = s;
}

template <int PAT>
void run(const char *name, int blocks, int threads, uint32_t rows) {
  uint64_t *cyc;
  uint32_t *sink;
  hipMalloc(&cyc, blocks * 8);
  hipMalloc(&sink, 4);
  const uint32_t iters = 1 << 16;
  hipLaunchKernelGGL(probe<PAT>, dim3(blocks), dim3(threads), 0, 0, iters, rows, cyc, sink, 0u);
  if (hipGetLastError() != hipSuccess) printf("launch failed\n");
  hipDeviceSynchronize();
  uint64_t c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-34s blocks %4d threads %4d rows %2u: %.1f cycles per dependent lookup\n", name, blocks, threads, rows,
         (double)c / iters);
  hipFree(cyc);
  hipFree(sink);
}

int main() {
  for (int threads : {64, 1024}) {
    run<0>("same byte (broadcast)", 256, threads, 1);
    run<1>("bytes lane&3 of one dword", 256, threads, 1);
    run<2>("byte lane (4 lanes per dword)", 256, threads, 1);
    run<3>("dword lane*32 (same bank)", 256, threads, 1);
    run<4>("printable byte, row 0", 256, threads, 1);
    run<4>("printable byte, 1/16 lanes rows 1-10", 256, threads, 11);
  }
  return 0;
}
