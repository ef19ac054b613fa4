// Device scratch cache (dfa_scan.hpp scratch_malloc / scratch_free).
#include "runtime.hpp"

namespace rt {

// ---------------------------------------------------------- scratch cache
// See dfa_scan.hpp scratch_malloc.  Blocks are rounded up (4 KiB, then
// 64 KiB multiples) and come from hipMalloc.  A freed block is cached per
// device with an event recorded on the freeing stream; an allocation of at
// most half its size on any stream of that device waits for that event
// (hipStreamWaitEvent) and reuses it, so reuse is ordered after the previous
// user's kernels whatever stream either used (a destroyed and recreated
// stream handle, the per-thread default stream).  The cache holds at most
// max(kScratchMinCap, 2 x the peak of live scratch bytes), at most
// kScratchMaxCap (RURE_AMD_SCRATCH_CAP overrides, bytes); a block freed
// beyond that is returned to the driver once its event has completed.
// Cached blocks go back to the driver on rure_amd_release_scratch(), when the
// last rure / rure_set is freed, and before a retry when an allocation fails.
// (The stream-ordered pool of hipMallocAsync kept freed memory mapped even
// after hipMemPoolTrimTo on this ROCm, measured in round 3.)
constexpr size_t kScratchMinCap = 256ull << 20, kScratchMaxCap = 8ull << 30;
struct ScratchBlock {
  size_t n;
  int dev;
  hipEvent_t ev;   // recorded at the last free (nullptr: never freed yet)
  hipStream_t st;  // the stream of the last free
};
struct ScratchCache {
  std::mutex mu;
  std::map<int, std::multimap<size_t, std::pair<void *, ScratchBlock>>> free_blocks;
  std::unordered_map<void *, ScratchBlock> live;
  size_t cached = 0, live_bytes = 0, peak_live = 0;
};
ScratchCache &scratch_cache() {
  static ScratchCache *c = new ScratchCache();  // never destroyed: frees may run at exit
  return *c;
}
size_t scratch_round(size_t n) { return n <= 4096 ? 4096 : (n + 65535) & ~(size_t)65535; }
size_t scratch_cap(const ScratchCache &c) {
  if (knob(Knob::ScratchCap) >= 0) return (size_t)knob(Knob::ScratchCap);
  return std::min(kScratchMaxCap, std::max(kScratchMinCap, 2 * c.peak_live));
}
// Returns a block to the driver after its last use.
void scratch_release_block(void *p, const ScratchBlock &b) {
  if (b.ev) {
    (void)hipEventSynchronize(b.ev);
    (void)hipEventDestroy(b.ev);
  }
  (void)hipFree(p);
}
// Returns every cached block (caller holds c.mu).
void scratch_drop_all(ScratchCache &c) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto &kv : c.free_blocks) {
    if (kv.second.empty()) continue;
    (void)hipSetDevice(kv.first);
    for (auto &blk : kv.second) scratch_release_block(blk.second.first, blk.second.second);
    kv.second.clear();
  }
  (void)hipSetDevice(cur);
  c.cached = 0;
}
std::atomic<long> g_live_handles{0};   // rure + rure_set objects alive

void scratch_release() {
  ScratchCache &c = scratch_cache();
  std::lock_guard<std::mutex> g(c.mu);
  scratch_drop_all(c);
}

void handle_created() { g_live_handles.fetch_add(1); }
void handle_freed() {
  if (g_live_handles.fetch_sub(1) == 1) scratch_release();
}

}  // namespace rt

hipError_t rure_amd::scratch_malloc(void **p, size_t bytes, hipStream_t st) {
  if (!p) return hipErrorInvalidValue;
  int d = 0;
  hipError_t e = hipGetDevice(&d);
  if (e != hipSuccess) return e;
  const size_t n = scratch_round(bytes);
  ScratchCache &c = scratch_cache();
  {
    std::lock_guard<std::mutex> g(c.mu);
    auto &fb = c.free_blocks[d];
    auto b = fb.lower_bound(n);
    if (b != fb.end() && b->first <= 2 * n) {
      void *q = b->second.first;
      ScratchBlock blk = b->second.second;
      fb.erase(b);
      c.cached -= blk.n;
      c.live[q] = blk;
      c.live_bytes += blk.n;
      c.peak_live = std::max(c.peak_live, c.live_bytes);
      *p = q;
      // Reuse on the stream that freed it is ordered by the stream itself
      // (hipStreamDestroy completes a stream's work before its handle can be
      // handed out again); the wait is a barrier packet that cost the
      // latency-bound C1 step ~5 us.  hipStreamPerThread names a different
      // stream on every thread, so it always waits.
      if (!blk.ev || (st == blk.st && st != hipStreamPerThread)) return hipSuccess;
      return hipStreamWaitEvent(st, blk.ev, 0);
    }
  }
  void *q = nullptr;
  e = hipMalloc(&q, n);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> g(c.mu);
      scratch_drop_all(c);
    }
    e = hipMalloc(&q, n);
  }
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(c.mu);
  c.live[q] = ScratchBlock{n, d, nullptr, nullptr};
  c.live_bytes += n;
  c.peak_live = std::max(c.peak_live, c.live_bytes);
  *p = q;
  return hipSuccess;
}

hipError_t rure_amd::scratch_free(void *p, hipStream_t st) {
  if (!p) return hipSuccess;
  ScratchCache &c = scratch_cache();
  ScratchBlock blk{0, 0, nullptr, nullptr};
  {
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return hipErrorInvalidValue;  // not a scratch block
    blk = it->second;
    c.live.erase(it);
    c.live_bytes -= blk.n;
    hipError_t e = hipSuccess;
    if (!blk.ev) e = hipEventCreateWithFlags(&blk.ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(blk.ev, st);
    blk.st = st;
    if (e == hipSuccess && c.cached + blk.n <= scratch_cap(c)) {
      c.free_blocks[blk.dev].emplace(blk.n, std::make_pair(p, blk));
      c.cached += blk.n;
      return hipSuccess;
    }
  }
  scratch_release_block(p, blk);
  return hipSuccess;
}

// C ABI: the cache's state (tests, bench)
void rure_amd_scratch_stats(size_t *cached, size_t *live, long *handles) {
  ScratchCache &c = scratch_cache();
  std::lock_guard<std::mutex> g(c.mu);
  if (cached) *cached = c.cached;
  if (live) *live = c.live_bytes;
  if (handles) *handles = g_live_handles.load();
}
