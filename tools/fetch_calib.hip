// Diagnostic: FETCH_SIZE calibration for C4's access pattern.  Reads the
// same ragged offset batch the set kernel reads (10M lines, 40-160 bytes,
// concatenated), with the set kernel's per-lane pattern (one lane per line,
// aligned 16-byte loads from the block holding the line's first byte to its
// last, plus the two offsets) and as one coalesced stream of the same bytes,
// so `rocprofv3 --pmc FETCH_SIZE` on this binary separates the counter's
// view of the access pattern from the kernel's own extra reads.
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

__global__ __launch_bounds__(1024) void per_line(const uint8_t *hay, const uint64_t *offs, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t h = blockIdx.x * 1024ull + threadIdx.x; h < n; h += (uint64_t)gridDim.x * 1024) {
    const uint64_t o0 = offs[h], o1 = offs[h + 1];
    for (uint64_t a = o0 & ~15ull; a < o1; a += 16) {
      const uint4 v = *(const uint4 *)(hay + a);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

__global__ __launch_bounds__(256) void stream(const uint4 *p, uint64_t nvec, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main() {
  const uint64_t n = 10000000;
  std::vector<uint64_t> offs(n + 1, 0);
  std::mt19937_64 rng(0x5EED0004);
  std::uniform_int_distribution<int> len(40, 160);
  for (uint64_t i = 0; i < n; ++i) offs[i + 1] = offs[i] + len(rng);
  const uint64_t bytes = offs[n];
  uint8_t *hay;
  uint64_t *doffs;
  uint32_t *out;
  if (hipMalloc(&hay, bytes + 64) != hipSuccess || hipMalloc(&doffs, (n + 1) * 8) != hipSuccess ||
      hipMalloc(&out, 4) != hipSuccess)
    return 1;
  (void)hipMemset(hay, 'a', bytes + 64);
  (void)hipMemcpy(doffs, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(per_line, dim3(256 * 2), dim3(1024), 0, 0, hay, doffs, n, out);
    hipLaunchKernelGGL(stream, dim3(256 * 8), dim3(256), 0, 0, (const uint4 *)hay, (bytes + 15) / 16, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("lines %llu text %llu bytes offsets %llu bytes\n", (unsigned long long)n, (unsigned long long)bytes,
         (unsigned long long)((n + 1) * 8));
  return 0;
}
