// Diagnostic: HBM read rate of the scan kernel's access pattern (one lane per
// 4 KiB haystack, 128-byte per-lane bursts) vs a coalesced stream.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__global__ __launch_bounds__(256) void lane_per_hay(const uint8_t *hay, uint64_t n, uint64_t L, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t h = blockIdx.x * 256ull + threadIdx.x; h < n; h += (uint64_t)gridDim.x * 256) {
    const uint4 *p = (const uint4 *)(hay + h * L);
    for (uint64_t at = 0; at < L / 16; at += 8) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = p[at + k];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

__global__ __launch_bounds__(256) void coalesced(const uint4 *p, uint64_t nvec, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}


// coalesced tile load (instruction k: 8 haystacks x 128 B), transposed through
// a per-wave LDS buffer (XOR-swizzled rows), each lane then reads its own row.
__global__ __launch_bounds__(256) void tile_lds(const uint8_t *hay, uint64_t n, uint64_t L, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint4 stage[4][64 * 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  uint32_t acc = 0;
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  for (uint64_t g = blockIdx.x * 4ull + w; g * 64 < n; g += waves) {
    const uint64_t h0 = g * 64;
    for (uint64_t at = 0; at < L; at += 128) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint64_t hh = h0 + 8 * k + (lane >> 3);
        v[k] = *(const uint4 *)(hay + hh * L + at + 16 * (lane & 7));
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int hh = 8 * k + (lane >> 3), seg = lane & 7;
        buf[hh * 8 + (seg ^ ((hh >> 1) & 7))] = v[k];
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        uint4 r = buf[lane * 8 + (m ^ ((lane >> 1) & 7))];
        acc ^= r.x ^ r.y ^ r.z ^ r.w;
      }
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

// tile_lds with the next tile's loads in flight while the current one is
// read back (the scan kernels' pipeline), and a fixed amount of per-lane work
// per 16 bytes (WORK dependent integer ops) standing in for the DFA chain
template <int WORK>
__global__ __launch_bounds__(256) void tile_pipe(const uint8_t *hay, uint64_t n, uint64_t L, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint4 stage[4][64 * 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  uint32_t acc = 0;
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  for (uint64_t g = blockIdx.x * 4ull + w; g * 64 < n; g += waves) {
    const uint64_t h0 = g * 64;
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = *(const uint4 *)(hay + (h0 + 8 * k + (lane >> 3)) * L + 16 * (lane & 7));
    for (uint64_t at = 0; at < L; at += 128) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int hh = 8 * k + (lane >> 3), seg = lane & 7;
        buf[hh * 8 + (seg ^ ((hh >> 1) & 7))] = v[k];
      }
      __builtin_amdgcn_wave_barrier();
      const uint64_t an = at + 128 < L ? at + 128 : at;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = *(const uint4 *)(hay + (h0 + 8 * k + (lane >> 3)) * L + an + 16 * (lane & 7));
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        uint4 r = buf[lane * 8 + (m ^ ((lane >> 1) & 7))];
        uint32_t x = r.x ^ r.y ^ r.z ^ r.w;
#pragma unroll
        for (int q = 0; q < WORK; ++q) x = x * 0x9E3779B1u + (x >> 7);
        acc ^= x;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

template <int WORK>
void run_pipe(const char *name, const uint8_t *hay, uint64_t n, uint64_t L, uint64_t bytes, uint32_t *out, int g) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) tile_pipe<WORK><<<g, 256>>>(hay, n, L, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (rep) printf("%s grid=%d  %.3f ms  %.1f GB/s\n", name, g, ms / 5, bytes / (ms / 5) / 1e6);
  }
}

int main(int argc, char **argv) {
  const uint64_t L = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4096, n = (4ull << 30) / L, bytes = n * L;
  printf("L=%llu n=%llu\n", (unsigned long long)L, (unsigned long long)n);
  uint8_t *hay; uint32_t *out;
  hipMalloc(&hay, bytes); hipMalloc(&out, 4);
  hipMemset(hay, 1, bytes);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  int grids[] = {1024, 2048, 4096};
  for (int g : grids) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < 5; ++i) lane_per_hay<<<g, 256>>>(hay, n, L, out);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep) printf("lane_per_hay grid=%d  %.3f ms  %.1f GB/s\n", g, ms / 5, bytes / (ms / 5) / 1e6);
    }
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < 5; ++i) coalesced<<<g, 256>>>((const uint4 *)hay, bytes / 16, out);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep) printf("coalesced    grid=%d  %.3f ms  %.1f GB/s\n", g, ms / 5, bytes / (ms / 5) / 1e6);
    }
  }
  for (int g : grids) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < 5; ++i) tile_lds<<<g, 256>>>(hay, n, L, out);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep) printf("tile_lds     grid=%d  %.3f ms  %.1f GB/s\n", g, ms / 5, bytes / (ms / 5) / 1e6);
    }
  }
  int grids2[] = {1024, 2048, 4096, 8192};
  for (int g : grids2) {
    run_pipe<0>("tile_pipe0  ", hay, n, L, bytes, out, g);
    run_pipe<8>("tile_pipe8  ", hay, n, L, bytes, out, g);
    run_pipe<32>("tile_pipe32 ", hay, n, L, bytes, out, g);
  }
  return 0;
}
