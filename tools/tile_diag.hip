// Diagnostic (not part of the library): the coalesced-tile scan structure of
// dfa_fwd_tile_kernel with three inner loops, to see what bounds it.
//   V0  tile loads + LDS transpose, per-byte VALU only (no table lookups)
//   V1  + one LDS table lookup per byte, independent of the previous one
//   V2  + dependent lookups s = T[s*304 + b] (the real DFA chain)
// Build: hipcc -O3 --offload-arch=gfx950 tools/tile_diag.hip -o /tmp/tile_diag
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kRow = 304, kRows = 16;

__device__ __noinline__ uint32_t careful16(uint32_t s, uint4 v, const uint8_t *g) {
  // stands in for the product's byte-by-byte redo against the global table
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (int j = 0; j < 16; ++j) s = g[(s * 256 + ((w[j >> 2] >> ((j & 3) * 8)) & 0xFF)) & 4095];
  return s;
}

template <int V>
__device__ __forceinline__ uint32_t step4(uint32_t s, uint32_t w, const uint8_t *tab) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t b = (w >> (8 * k)) & 0xFF;
    if (V == 0) s = (s * 33u) ^ b;
    else if (V == 1) s += tab[(b * 7u) & 1023u];
    else s = tab[s * kRow + b];  // V2, V3
  }
  return s;
}

template <int V, int PERM = 0>
__global__ __launch_bounds__(256) void tile_kernel(const uint8_t *hay, uint64_t n, uint64_t L, uint64_t S,
                                                   const uint8_t *img, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint8_t tab[kRows * kRow + 96];
  __shared__ __attribute__((aligned(16))) uint4 stage[4][64 * 8];
  for (uint32_t i = threadIdx.x * 16; i < kRows * kRow; i += blockDim.x * 16) *(uint4 *)(tab + i) = *(const uint4 *)(img + i);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  const int src_h = lane >> 3, src_seg = lane & 7;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + w; g * 64 < n; g += nwaves) {
    // PERM 1: haystack rows of a wave scattered (odd multiplier mod n); PERM 2:
    // the wave's group index scattered (rows stay consecutive)
    const uint64_t gg = PERM == 2 ? (g * 40503u) & (n / 64 - 1) : g;
    const uint8_t *src0 = hay + (gg * 64 + src_h) * S + 16 * src_seg;
    const uint64_t kstep = 8 * S;
    uint4 n0, n1, n2, n3, n4, n5, n6, n7;
#define LOAD(a)                                                                               \
  n0 = *(const uint4 *)(src0 + (a)); n1 = *(const uint4 *)(src0 + kstep + (a));               \
  n2 = *(const uint4 *)(src0 + 2 * kstep + (a)); n3 = *(const uint4 *)(src0 + 3 * kstep + (a)); \
  n4 = *(const uint4 *)(src0 + 4 * kstep + (a)); n5 = *(const uint4 *)(src0 + 5 * kstep + (a)); \
  n6 = *(const uint4 *)(src0 + 6 * kstep + (a)); n7 = *(const uint4 *)(src0 + 7 * kstep + (a));
#define STG(k, v) buf[(8 * (k) + src_h) * 8 + (src_seg ^ (((8 * (k) + src_h) >> 1) & 7))] = (v);
    LOAD(0)
    uint32_t s = 0;
    bool done = false;
    const int sw = (lane >> 1) & 7;
    for (uint64_t at = 0; at < L; at += 128) {
      if (V == 3 && !__any(!done)) break;
      STG(0, n0) STG(1, n1) STG(2, n2) STG(3, n3) STG(4, n4) STG(5, n5) STG(6, n6) STG(7, n7)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint64_t an = at + 128 < L ? at + 128 : at;
      LOAD(an)
      uint4 cur = buf[lane * 8 + sw];
#pragma unroll 1
      for (int m = 0; m < 8; ++m) {
        uint4 nx = buf[lane * 8 + ((m + 1 < 8 ? m + 1 : 7) ^ sw)];
        if (V == 3) {
          // product-like: skip done lanes, sentinel check, careful redo path
          if (!done) {
            uint32_t t = s;
            if (s < 15u) {
              t = step4<2>(t, cur.x, tab);
              t = step4<2>(t, cur.y, tab);
              t = step4<2>(t, cur.z, tab);
              t = step4<2>(t, cur.w, tab);
            }
            if (t != 15u) s = t;
            else { s = careful16(s, cur, img); done = s == 77; }
          }
        } else {
          s = step4<V>(s, cur.x, tab);
          s = step4<V>(s, cur.y, tab);
          s = step4<V>(s, cur.z, tab);
          s = step4<V>(s, cur.w, tab);
        }
        cur = nx;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    out[g * 64 + lane] = s;
  }
}

// V5: two independent chains per lane (haystacks lane and lane + 64 of a
// 128-haystack group), 64-byte tiles: same 8 KiB of staging per wave, twice
// the chains per CU.
__global__ __launch_bounds__(256) void tile2_kernel(const uint8_t *hay, uint64_t n, uint64_t L, uint64_t S,
                                                   const uint8_t *img, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint8_t tab[kRows * kRow + 96];
  __shared__ __attribute__((aligned(16))) uint4 stage[4][128 * 4];
  for (uint32_t i = threadIdx.x * 16; i < kRows * kRow; i += blockDim.x * 16) *(uint4 *)(tab + i) = *(const uint4 *)(img + i);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  const int src_h = lane >> 2, src_seg = lane & 3;  // 16 rows x 4 segments per instruction
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint64_t ngroups = n / 128;
  for (uint64_t gi = (uint64_t)blockIdx.x * 4 + w; gi < ngroups; gi += nwaves) {
    const uint64_t g = (gi * 40503u) % ngroups;
    const uint8_t *src0 = hay + (g * 128 + src_h) * S + 16 * src_seg;
    const uint64_t kstep = 16 * S;
    uint4 n0, n1, n2, n3, n4, n5, n6, n7;
#define LOAD2(a)                                                                              \
  n0 = *(const uint4 *)(src0 + (a)); n1 = *(const uint4 *)(src0 + kstep + (a));               \
  n2 = *(const uint4 *)(src0 + 2 * kstep + (a)); n3 = *(const uint4 *)(src0 + 3 * kstep + (a)); \
  n4 = *(const uint4 *)(src0 + 4 * kstep + (a)); n5 = *(const uint4 *)(src0 + 5 * kstep + (a)); \
  n6 = *(const uint4 *)(src0 + 6 * kstep + (a)); n7 = *(const uint4 *)(src0 + 7 * kstep + (a));
#define STG2(k, v) buf[(16 * (k) + src_h) * 4 + (src_seg ^ (((16 * (k) + src_h) >> 2) & 3))] = (v);
    LOAD2(0)
    uint32_t sa = 0, sb = 0;
    const int swa = (lane >> 2) & 3, swb = ((lane + 64) >> 2) & 3;
    for (uint64_t at = 0; at < L; at += 64) {
      STG2(0, n0) STG2(1, n1) STG2(2, n2) STG2(3, n3) STG2(4, n4) STG2(5, n5) STG2(6, n6) STG2(7, n7)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint64_t an = at + 64 < L ? at + 64 : at;
      LOAD2(an)
#pragma unroll 1
      for (int m = 0; m < 4; ++m) {
        const uint4 ca = buf[lane * 4 + (m ^ swa)];
        const uint4 cb = buf[(lane + 64) * 4 + (m ^ swb)];
        const uint32_t wa[4] = {ca.x, ca.y, ca.z, ca.w}, wb[4] = {cb.x, cb.y, cb.z, cb.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          sa = tab[sa * kRow + ((wa[j >> 2] >> ((j & 3) * 8)) & 0xFF)];
          sb = tab[sb * kRow + ((wb[j >> 2] >> ((j & 3) * 8)) & 0xFF)];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    out[g * 128 + lane] = sa;
    out[g * 128 + lane + 64] = sb;
  }
}

__global__ void fill(uint8_t *p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    const uint32_t r = (uint32_t)x;
    p[i] = (r % 1000) < 200 ? (uint8_t)('0' + (r >> 10) % 10) : (uint8_t)(32 + (r >> 10) % 95);
  }
}

template <int V, int PERM = 0>
float run(const uint8_t *hay, uint64_t n, uint64_t L, uint64_t S, const uint8_t *img, uint32_t *out, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((tile_kernel<V, PERM>), dim3(grid), dim3(256), 0, 0, hay, n, L, S, img, out);
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((tile_kernel<V, PERM>), dim3(grid), dim3(256), 0, 0, hay, n, L, S, img, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const uint64_t n = 1 << 20, L = 4096;
  uint8_t *hay, *img;
  uint32_t *out;
  hipMalloc(&hay, n * (L + 512));
  hipMalloc(&img, kRows * kRow);
  hipMalloc(&out, n * 4);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, hay, n * (L + 512));
  // synthetic DFA rows: digits advance a counter state, anything else resets to 0
  uint8_t h[kRows * kRow];
  for (int s = 0; s < kRows; ++s)
    for (int b = 0; b < kRow; ++b) h[s * kRow + b] = (b >= '0' && b <= '9') ? (uint8_t)((s + 1) % 11) : 0;
  hipMemcpy(img, h, sizeof(h), hipMemcpyHostToDevice);
  const int grid = 2048;
  const double gb = (double)n * L / 1e9;
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL((tile_kernel<0, 2>), dim3(grid), dim3(256), 0, 0, hay, n, L, L, img, out);
  hipDeviceSynchronize();
  for (uint64_t S : {L, L + 64, L + 128, L + 256, L + 512}) {
    float t0 = run<0>(hay, n, L, S, img, out, grid);
    float t1 = run<1>(hay, n, L, S, img, out, grid);
    float t2 = run<2>(hay, n, L, S, img, out, grid);
    printf("stride %5lu: V0 tiles+VALU %.3f ms %.0f GB/s | V1 +indep LDS %.3f ms %.0f GB/s | V2 +chain %.3f ms %.0f GB/s\n",
           (unsigned long)S, t0, gb / t0 * 1e3, t1, gb / t1 * 1e3, t2, gb / t2 * 1e3);
  }
  {
    float c = run<3, 2>(hay, n, L, L, img, out, grid);
    printf("stride 4096, scattered groups: V3 (product-like control) %.3f ms %.0f GB/s\n", c, gb / c * 1e3);
    float a = run<2, 2>(hay, n, L, L, img, out, grid);
    printf("stride 4096, scattered groups: V2 %.3f ms %.0f GB/s\n", a, gb / a * 1e3);
    float b0 = run<0, 2>(hay, n, L, L, img, out, grid);
    printf("stride 4096, scattered groups: V0 %.3f ms %.0f GB/s\n", b0, gb / b0 * 1e3);
  }
  for (int gr : {1024, 2048}) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(tile2_kernel, dim3(gr), dim3(256), 0, 0, hay, n, L, L, img, out);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(tile2_kernel, dim3(gr), dim3(256), 0, 0, hay, n, L, L, img, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 10;
    printf("V5 two chains/lane, 64-B tiles, grid %d: %.3f ms %.0f GB/s\n", gr, ms, gb / ms * 1e3);
  }
  for (int gr : {1024, 4096, 8192}) {
    float t2 = run<2>(hay, n, L, L, img, out, gr);
    printf("grid %d: V2 %.3f ms %.0f GB/s\n", gr, t2, gb / t2 * 1e3);
  }
  return 0;
}
