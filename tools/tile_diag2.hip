// Diagnostic (not part of the library): the product's dfa_fwd_tile_kernel on
// the synthetic DFA and data of tools/tile_diag.hip (digits advance a counter
// state, anything else resets), to compare the product's control structure
// with the bare tile loop at identical inputs.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/tile_diag2.hip -o /tmp/tile_diag2
#include "../regex_amd/csrc/kernels/dfa_scan.hip"

#include <stdio.h>
#include <vector>

using namespace rure_amd;

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

template <typename T>
T *up(const std::vector<T> &v) {
  T *d;
  hipMalloc(&d, v.size() * sizeof(T) + 256);
  hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  return d;
}

int main() {
  const uint64_t n = 1 << 20, L = 4096;
  uint8_t *hay;
  hipMalloc(&hay, n * L + 64);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, hay, n * L);
  const int NS = 12, HOT = 11, DEAD = 11;
  std::vector<uint16_t> full(NS * 256);
  for (int s = 0; s < NS; ++s)
    for (int b = 0; b < 256; ++b) full[s * 256 + b] = s == DEAD ? DEAD : (b >= '0' && b <= '9') ? (s + 1) % 11 : 0;
  std::vector<uint8_t> img(((HOT + 1) * kRow + 15) & ~15, 0);
  for (int s = 0; s <= HOT; ++s)
    for (int b = 0; b < 256; ++b) img[s * kRow + b] = s == HOT ? HOT : (uint8_t)full[s * 256 + b];
  std::vector<uint8_t> eof(NS, 0);
  std::vector<uint16_t> start(128, 0);
  FwdDfaDev f{};
  f.lds_image = up(img);
  f.lds_bytes = (uint32_t)img.size();
  f.hot = HOT;
  f.stride = 1;
  f.cus = 256;
  f.full = up(full);
  f.eof = up(eof);
  f.start = up(start);
  f.n_normal = 11;
  f.n_match_end = 11;
  f.dead = DEAD;
  f.quit = 0xFFFFFFFFu;
  RevDfaDev r{};
  r.full = f.full;
  r.eof = f.eof;
  r.start = f.start;
  r.n_normal = 11;
  r.n_match_end = 11;
  r.dead = DEAD;
  r.quit = 0xFFFFFFFFu;
  uint64_t *out;
  hipMalloc(&out, n * 16);
  BatchDev b{hay, nullptr, L, L, n, 0};
  const int grid = 2048;
  for (int mode : {MODE_FIND, MODE_ISMATCH, MODE_FIND, MODE_ISMATCH, MODE_FIND}) {
    launch_dfa_fwd(mode, b, f, r, out, 0, grid);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) launch_dfa_fwd(mode, b, f, r, out, 0, grid);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("product tile kernel, mode %d, synthetic DFA: %.3f ms %.0f GB/s\n", mode, ms, n * L / 1e6 / ms);
  }
  return 0;
}
