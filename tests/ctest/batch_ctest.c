/* The batched device entry points of include/rure_amd.h used from plain C
 * (the way a C caller of regex-capi would add the GPU path): device buffers
 * from the HIP runtime, rure_amd_find_batch / _find_iter_batch /
 * _find_iter_span, each checked against the single-haystack rure_find /
 * rure_iter_next of the same library (rure.h:197-330 semantics). */
#define _POSIX_C_SOURCE 199309L
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rure_amd.h"

static int failures = 0;
#define CHECK(cond, ...)                     \
  do {                                       \
    if (!(cond)) {                           \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);          \
      fprintf(stderr, "\n");                 \
      ++failures;                            \
    }                                        \
  } while (0)
#define HIP(x) CHECK((x) == hipSuccess, "%s", #x)

/* deterministic text: words, dates and newlines */
static void make_text(uint8_t *t, size_t n, uint32_t seed) {
  static const char *words[] = {"foo ", "bar ", "2017-12-30 ", "aaaa ", "\n", "Holmes ", "x1 ", "2018-01-02\n"};
  size_t i = 0;
  while (i < n) {
    seed = seed * 1103515245u + 12345u;
    const char *w = words[(seed >> 16) % 8];
    for (size_t j = 0; w[j] && i < n; ++j) t[i++] = (uint8_t)w[j];
  }
}

int main(void) {
  const size_t L = 4096, N = 64, TOT = L * N;
  uint8_t *host = malloc(TOT);
  make_text(host, TOT, 7u);
  uint8_t *dev = NULL;
  HIP(hipMalloc((void **)&dev, TOT + 16));
  HIP(hipMemcpy(dev, host, TOT, hipMemcpyHostToDevice));
  rure *re = rure_compile_must("\\d{4}-\\d{2}-\\d{2}");

  /* batched find: one leftmost-first match per haystack */
  rure_amd_batch b = {dev, NULL, L, L, N, 0};
  rure_match *dm = NULL, hm[64];
  HIP(hipMalloc((void **)&dm, N * sizeof(rure_match)));
  CHECK(rure_amd_find_batch(re, &b, dm, NULL) == RURE_AMD_OK, "find_batch");
  HIP(hipMemcpy(hm, dm, N * sizeof(rure_match), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < N; ++i) {
    rure_match m;
    const bool ok = rure_find(re, host + i * L, L, 0, &m);
    CHECK(ok ? (hm[i].start == m.start && hm[i].end == m.end) : hm[i].start == SIZE_MAX, "find_batch[%zu]", i);
  }

  /* find_iter over the whole text: matches vs rure_iter_next */
  const size_t cap = 1 << 16;
  rure_match *di = NULL, *hi = malloc(cap * sizeof(rure_match));
  uint64_t *dcount = NULL, *dtotal = NULL, total = 0;
  HIP(hipMalloc((void **)&di, cap * sizeof(rure_match)));
  HIP(hipMalloc((void **)&dcount, 8));
  HIP(hipMalloc((void **)&dtotal, 8));
  rure_amd_batch one = {dev, NULL, TOT, TOT, 1, 0};
  CHECK(rure_amd_find_iter_batch(re, &one, dcount, di, cap, dtotal, NULL) == RURE_AMD_OK, "find_iter_batch");
  HIP(hipMemcpy(&total, dtotal, 8, hipMemcpyDeviceToHost));
  HIP(hipMemcpy(hi, di, total * sizeof(rure_match), hipMemcpyDeviceToHost));
  rure_iter *it = rure_iter_new(re);
  rure_match m;
  size_t k = 0;
  while (rure_iter_next(it, host, TOT, &m)) {
    CHECK(k < total && hi[k].start == m.start && hi[k].end == m.end, "find_iter[%zu]", k);
    ++k;
  }
  rure_iter_free(it);
  CHECK(k == total, "find_iter count %zu vs %llu", k, (unsigned long long)total);

  /* the same iteration as three chained spans (sharded / streamed) */
  const size_t cuts[4] = {0, TOT / 3 + 5, 2 * TOT / 3 + 1, TOT};
  rure_amd_iter_state *dexit = NULL, hexit;
  HIP(hipMalloc((void **)&dexit, 2 * sizeof(rure_amd_iter_state)));
  size_t got = 0;
  for (int s = 0; s < 3; ++s) {
    const rure_amd_iter_state *entry = s ? &dexit[(s - 1) & 1] : NULL;
    uint64_t cnt = 0;
    CHECK(rure_amd_find_iter_span(re, dev, TOT, cuts[s], cuts[s + 1], entry, dcount, di, cap, &dexit[s & 1],
                                  NULL) == RURE_AMD_OK, "find_iter_span %d", s);
    HIP(hipMemcpy(&cnt, dcount, 8, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(hi, di, cnt * sizeof(rure_match), hipMemcpyDeviceToHost));
    HIP(hipMemcpy(&hexit, &dexit[s & 1], sizeof hexit, hipMemcpyDeviceToHost));
    for (uint64_t j = 0; j < cnt; ++j) CHECK(hi[j].start >= cuts[s] && hi[j].start < cuts[s + 1], "span owner");
    got += cnt;
  }
  CHECK(got == total, "spans %zu vs %llu", got, (unsigned long long)total);

  /* Stream order: with ~10 ms of finds queued ahead on a
   * stream, find_iter returns while that work is still running (it only
   * enqueues): [a-z]+, \w+ (the run engine reads UTF-8 itself) and
   * \w+@\w+\.\w+ (Unicode classes: the ASCII shadow's quit stays a device
   * flag that gates the full automaton's pass, enqueued behind it). */
  {
    const size_t BIGL = 4096, BIGN = 65536;
    uint8_t *big = NULL;
    rure_match *bm = NULL;
    hipStream_t st;
    HIP(hipStreamCreate(&st));
    HIP(hipMalloc((void **)&big, BIGL * BIGN + 16));
    HIP(hipMemset(big, 'a', BIGL * BIGN + 16));
    HIP(hipMalloc((void **)&bm, BIGN * sizeof(rure_match)));
    rure_amd_batch bb = {big, NULL, BIGL, BIGL, BIGN, 0};
    rure *lower = rure_compile_must("[a-z]+");
    rure *word = rure_compile_must("\\w+");
    rure *mail = rure_compile_must("\\w+@\\w+\\.\\w+");
    for (int pass = 0; pass < 3; ++pass) {
      rure *r = pass == 0 ? lower : pass == 1 ? word : mail;
      /* warm: first calls build and upload tables */
      CHECK(rure_amd_find_iter_batch(r, &one, dcount, di, cap, dtotal, st) == RURE_AMD_OK, "warm iter");
      HIP(hipStreamSynchronize(st));
      for (int i = 0; i < 200; ++i) CHECK(rure_amd_find_batch(re, &bb, bm, st) == RURE_AMD_OK, "queued find");
      struct timespec t0, t1;
      clock_gettime(CLOCK_MONOTONIC, &t0);
      CHECK(rure_amd_find_iter_batch(r, &one, dcount, di, cap, dtotal, st) == RURE_AMD_OK, "iter after queue");
      clock_gettime(CLOCK_MONOTONIC, &t1);
      const hipError_t q = hipStreamQuery(st);
      const double ms = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6;
      CHECK(q == hipErrorNotReady, "find_iter (pass %d) waited for the stream (query %d, %.2f ms)", pass, (int)q, ms);
      HIP(hipStreamSynchronize(st));
    }
    rure_free(lower);
    rure_free(word);
    rure_free(mail);
    hipFree(big);
    hipFree(bm);
    HIP(hipStreamDestroy(st));
  }

  rure_free(re);
  hipFree(dev);
  hipFree(dm);
  hipFree(di);
  hipFree(dcount);
  hipFree(dtotal);
  hipFree(dexit);
  free(host);
  free(hi);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("all checks passed\n");
  return 0;
}
