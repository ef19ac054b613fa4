// Batched find_iter (re_trait.rs:197-221 over ExecNoSync::find_at,
// exec.rs:473-514) for gfx950.
//
// The iteration is sequential by nature: each search starts where the
// previous match ended.  Long haystacks are cut into chunks ("units"); one
// lane iterates each unit *speculatively* from a fresh start at the unit's
// first byte, owning the matches that start inside it.  For patterns without
// look-around assertions, a unit's speculative result is exact unless the
// true sequence enters it in a different state: a match of the previous unit
// that runs past the cut ("dirty" exit).  Those units are repaired by running
// the true iteration and the speculative one in lockstep until they emit the
// same match (from there on they coincide); a repair that does not converge
// inside its unit changes that unit's exit and is propagated by a sequential
// walker (rare).  Counts are prefix-summed on the device and a final pass
// writes every unit's matches in order (copied from the unit's slot buffer
// when the speculation held and the unit had few matches).
//
// Patterns whose DFA can quit (Unicode word boundary) or that have no DFA, and
// patterns with assertions, are iterated one haystack per wavefront without
// chunking (per search: DFA on one lane, the Pike VM on the wave when the DFA
// quits or is absent) — the reference's per-search engine dispatch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <vector>
#include <stdint.h>

#include "dfa_device.hpp"
#include "match_device.hpp"
#include "nfa_device.hpp"

namespace rure_amd {

namespace {

// A launch gated on a device word (BatchDev::gate): it returns at once
// unless (*gate != 0) == gate_set (every block alike).
__device__ __forceinline__ bool gated_off(const BatchDev &b) {
  return b.gate && ((__atomic_load_n(b.gate, __ATOMIC_RELAXED) != 0) != (b.gate_set != 0));
}

// Speculative matches kept per unit: enough for one match per 32 bytes of
// the unit (the emit pass copies them instead of re-running the unit).
__host__ __device__ inline uint32_t unit_slots(uint64_t chunk) {
  uint64_t s = chunk / 32;
  return (uint32_t)(s < 4 ? 4 : s > 1024 ? 1024 : s);
}

enum : uint32_t {
  U_SPEC_CLEAN = 1,   // speculative exit is equivalent to a fresh start at the next unit
  U_CLEAN = 2,        // final exit clean
  U_FIXED = 4,        // final entry differs from the speculative one
  U_QUIT = 8,         // a search quit (sticky: the batch then goes to the wave path; f.can_quit only)
  U_COPY = 16,        // fixed, and its matches are slots[skip, skip + count)
  U_LEX_TAIL = 32,    // iter_spec_lex_tile_kernel: exit = the lexer's iteration state, the tail pass finishes
  U_COMPACT = 64,     // the lexer's slots: its pad (= its count) records as u32 start - c0 | end - c0 << 16,
                      // then the tail pass's as absolute ulonglong2 from the back (lex_rec32 / lex_row16)
  U_UNSURE = 128,     // look-around: the speculation's first reverse scan reached c0, so the true
                      // iteration entering earlier may differ even after a clean exit (repaired always)
  U_PEND = 256,       // the wave-served iteration: the lane stopped at a search that quit (exit = the
                      // state before it, U.pad = it is the unit's first); a wave answers it
  U_RESUME = 512,     // ... answered: the lanes go on from the exit (iter_spec_burst_kernel mode 2)
};

// Look-around (FwdDfaDev::looks).  A search from p runs its reverse scan over
// text[p..e] (exec.rs:651-661), whose EOF step reads p as the start of the
// text: the start it reports may depend on p, not only on the match.  So
//  - a unit's speculation (a fresh search at c0) equals the true iteration
//    entering earlier only when its first reverse scan died before reaching
//    c0 (U_UNSURE otherwise: repaired from the true entry like a dirty one);
//  - two exits are interchangeable ahead of an U_UNSURE unit only when they
//    are the same state (exit_equiv strict), and the join shortcut
//    (join_speculation) is off;
//  - a reverse NoMatch (dfa_find_cut 3) ends the reference's iteration: the
//    exit is kIterStop and every later unit of the haystack yields nothing.
// tests/iter_sim.py models this; tests/test_iter_chunks.py checks it against
// the oracle with one-byte units.
static constexpr uint64_t kIterStop = ~0ull - 1;

struct IterSt {
  uint64_t p, lm;  // next search start; end of the last match (NONE if none)
};

struct Unit {
  IterSt entry, exit, spec_exit;
  uint32_t spec_count, flags;
  uint32_t skip, pad;  // U_COPY: speculative matches dropped at the front; pad: U_COMPACT's lexer count
};

static_assert(sizeof(Unit) == 64, "iter_copy_group_kernel reads a unit's last 16 bytes");

struct Geo {  // unit -> (haystack, chunk) for fixed-stride batches
  uint64_t nk;      // units per haystack
  uint64_t chunk;   // bytes per unit
  uint64_t end;     // cut of the last unit (~0: the haystack end; a span's hi)
  uint32_t slots;   // speculative matches stored per unit
};

// U_COMPACT slots are interleaved over the 64 units of a lexer wave (their
// slot areas together, g.slots rows of 64 x 16 bytes): row k holds lexer
// records 4k..4k+3 of every unit, lane by lane, so the lexer's per-tile row
// stores write a few whole 1 KiB rows instead of 64 scattered partial lines
// (the scattered layout left ~33 MB of partly written lines in flight,
// more than L2).  The tail pass's records take rows from the back.
// lex_rec32: u32 index of lexer record i of unit u; lex_row16: ulonglong2
// index of unit u's 16 bytes in row k.
__device__ __forceinline__ uint64_t lex_rec32(const Geo &g, uint64_t u, uint32_t i) {
  return (u >> 6) * 256 * (uint64_t)g.slots + (uint64_t)(i >> 2) * 256 + (u & 63) * 4 + (i & 3);
}
__device__ __forceinline__ uint64_t lex_row16(const Geo &g, uint64_t u, uint32_t k) {
  return (u >> 6) * 64 * (uint64_t)g.slots + (uint64_t)k * 64 + (u & 63);
}

// Speculative record i of unit u (U_COMPACT: the first nlex as u16 pairs
// relative to c0, the rest absolute from the back rows).
__device__ __forceinline__ ulonglong2 slot_rec(const uint64_t *slots, const Geo &g, uint64_t u, uint32_t i,
                                               bool compact, uint64_t c0, uint32_t nlex) {
  if (compact) {
    if (i < nlex) {
      const uint32_t v = ((const uint32_t *)slots)[lex_rec32(g, u, i)];
      return make_ulonglong2(c0 + (v & 0xFFFFu), c0 + (v >> 16));
    }
    return ((const ulonglong2 *)slots)[lex_row16(g, u, g.slots - 1 - (i - nlex))];
  }
  return ((const ulonglong2 *)(slots + u * g.slots * 2))[i];
}

__device__ __forceinline__ void unit_bounds(const BatchDev &b, const Geo &g, uint64_t u, uint64_t *h,
                                            const uint8_t **base, uint64_t *len, uint64_t *c0, uint64_t *c1) {
  *h = u / g.nk;
  const uint64_t k = u % g.nk;
  if (b.offs) {
    const uint64_t o0 = b.offs[*h], o1 = b.offs[*h + 1];
    *base = b.hay + o0;
    *len = o1 - o0;
  } else {
    *base = b.hay + *h * b.stride;
    *len = b.length;
  }
  *c0 = b.start + k * g.chunk;
  *c1 = (k + 1 == g.nk) ? g.end : b.start + (k + 1) * g.chunk;
}

// The wave's Pike VM for searches whose DFA quits (the wave-served chunked
// iteration: every lane of the wave runs the same search, wave-uniform).
struct WaveCtx {
  const NfaDev *nf;
  pike::Lists *W;
  pike::TagGen *tg;
};

// One step of re_trait.rs:197-221 (empty-match rule: next search at e + 1,
// an empty match at the previous match end is skipped).
// reached: the first search's dfa_find_cut reach flag (look-around).
// wc: a search whose DFA quits runs on the Pike VM instead (exec.rs:485-487:
// the reference's fallback for that one search), bounded by the cut the same
// way (pike_one's cut); its answer does not depend on the search start.
__device__ int iter_next(const FwdDfaDev &f, const RevDfaDev &r, const uint8_t *lds, const uint8_t *rlds,
                         const uint8_t *base, uint64_t len, uint64_t cut, IterSt &st, uint64_t *s, uint64_t *e,
                         bool *reached = nullptr, const WaveCtx *wc = nullptr, bool *piked = nullptr) {
  while (true) {
    if (st.p > len) return 0;
    int k = dfa_find_cut(f, r, lds, rlds, base, len, st.p, cut, s, e, reached);
    if (k == 0 && f.can_quit == 2 && st.p > 0 && st.p < cut && base[st.p - 1] >= 0x80) {
      // No match before the cut, from a start whose previous byte is >= 0x80:
      // the DFA's start flags read it as a non-word byte (dfa.rs:1423), and
      // the reference's unbounded scan goes on past the cut -- if it quits
      // on a byte >= 0x80 its NFA answers for this search, which may start
      // before the cut.  The lanes hand such a search over as a quit; the
      // wave runs the unbounded scan to see.
      if (!wc) {
        k = 2;
      } else {
        uint64_t s2, e2;
        if (dfa_find(f, r, lds, rlds, base, len, st.p, &s2, &e2) == 2) k = 2;
      }
    }
    if (k == 2 && wc) {
      if (piked) *piked = true;
      uint64_t r0, r1;
      pike::pike_one<MODE_FIND>(*wc->nf, *wc->W, *wc->tg, base, len, st.p, &r0, &r1, st.p < cut ? cut : ~0ull);
      if (reached) *reached = false;
      k = r1 == NONE ? 0 : 1;
      *s = r0;
      *e = r1;
    }
    reached = nullptr;
    if (k != 1) return k;
    if (*s == *e) {
      st.p = *e + 1;
      if (st.lm == *e) continue;
    } else {
      st.p = *e;
    }
    st.lm = *e;
    return 1;
  }
}

// The matches a unit owns: those whose start is < c1, iterating from `st`.
struct UnitIter {
  IterSt st;
  uint64_t c1;
  uint64_t from;  // the first search may scan from here: no match starts in [st.p, from)
  bool ended, clean, quit;
  bool first, unsure;  // look-around: the first search's reverse scan reached its start
  bool waved;          // a search ran on the wave's Pike VM (wc)
  IterSt exit;

  __device__ void init(IterSt s0, uint64_t cut) {
    st = s0;
    c1 = cut;
    from = 0;
    ended = clean = quit = unsure = waved = false;
    first = true;
  }
  // Returns true with the next owned match, false when the unit is finished.
  __device__ bool next(const FwdDfaDev &f, const RevDfaDev &r, const uint8_t *lds, const uint8_t *rlds,
                       const uint8_t *base, uint64_t len, uint64_t *s, uint64_t *e, const WaveCtx *wc = nullptr) {
    if (ended) return false;
    if (st.p == kIterStop) {  // the iteration ended (look-around: a reverse NoMatch)
      ended = true;
      exit = st;
      return false;
    }
    if (st.p >= c1) {  // the previous match ran up to / past the cut
      ended = true;
      exit = st;
      clean = st.p == c1 && (st.lm != c1 || f.nonempty);
      return false;
    }
    const IterSt snap = st;
    // the search from st.p finds what a search from `from` finds when no
    // match starts in between (the regexes of the lexer path have no
    // look-around and never match empty); its state stays st's
    IterSt q = st;
    if (q.p < from) q.p = from;
    bool reached = false;
    bool pk = false;
    const int k = iter_next(f, r, lds, rlds, base, len, c1, q, s, e, first ? &reached : nullptr, wc, &pk);
    waved |= pk;
    if (first) unsure = reached;
    first = false;
    if (k == 1 && *s < c1) { st = q; return true; }
    if (k == 3) {  // look-around: this search's NoMatch ends the iteration
      ended = true;
      exit = {kIterStop, NONE};
      return false;
    }
    // no match starts before the cut (the search is cut-bounded, see
    // dfa_find_cut): a fresh search at the cut finds what the unrestricted
    // one would (no assertions on this path)
    ended = true;
    exit = snap;
    clean = k != 2;
    quit = k == 2;
    return false;
  }
};

// strict: the next unit is U_UNSURE (only the same state enters it alike)
__device__ __forceinline__ bool exit_equiv(bool ca, const IterSt &a, bool cb, const IterSt &b, bool strict = false) {
  if (strict) return a.p == b.p && a.lm == b.lm;
  if (ca || cb) return ca && cb;
  return a.p == b.p && a.lm == b.lm;
}

// Dynamic LDS of the DFA kernels here: forward hot table, then the reverse
// one (offset rev_lds_offset).
__host__ __device__ inline uint32_t rev_lds_offset(uint32_t fwd_bytes) { return (fwd_bytes + 15) & ~15u; }
inline size_t iter_lds_bytes(const FwdDfaDev &f, const RevDfaDev &r) { return rev_lds_offset(f.lds_bytes) + r.lds_bytes; }

__device__ __forceinline__ const uint8_t *stage_tables(const FwdDfaDev &f, const RevDfaDev &r, uint8_t *lds) {
  for (uint32_t i = threadIdx.x * 16; i < f.lds_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(f.lds_image + i);
  uint8_t *rl = lds + rev_lds_offset(f.lds_bytes);
  for (uint32_t i = threadIdx.x * 16; i < r.lds_bytes; i += blockDim.x * 16)
    *(uint4 *)(rl + i) = *(const uint4 *)(r.lds_image + i);
  __syncthreads();
  return r.lds_bytes ? rl : nullptr;
}

// Branch-free exact steps for small automata (FwdDfaDev::all /
// RevDfaDev::all: every state's row in LDS; dead and quit absorb).  Bytes
// k in [k0, kend) of the 16 in `w` are stepped from `s`; lastk = the last k
// whose step entered a match-flag state [nn, nme).  No per-byte branches:
// a match, the dead state or a quit mid-chunk costs the same instructions as
// any other byte, so the rare-event path of find_iter is not a serial
// byte loop run by one lane while the rest of its wave waits.
__device__ __forceinline__ uint32_t steps16(uint32_t s, const uint32_t w[4], uint32_t k0, uint32_t kend,
                                            const uint8_t *tab, uint32_t nn, uint32_t nme, int &lastk) {
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t t = tab[__umul24(s, kRow) + ((w[k >> 2] >> ((k & 3) * 8)) & 0xFF)];
    const bool act = k >= k0 && k < kend;
    s = act ? t : s;
    lastk = (act && t - nn < nme - nn) ? (int)k : lastk;
  }
  return s;
}

// Forward scan of text[at..end) (end - at <= 128 + 15, all-mode tables,
// MODE_FIND: dfa.rs:576-764 up to the dead state): the window's blocks are
// loaded first, then each goes through the exact4 fast chain and, if that
// entered a match / dead / quit state, the branch-free steps16.
__device__ __forceinline__ void fwd_window_all(LaneState &L, const FwdDfaDev &f, const uint8_t *lds,
                                               const uint8_t *base, uint64_t at, uint64_t end) {
  const uintptr_t a0 = (uintptr_t)(base + at) & ~(uintptr_t)15;
  const uintptr_t ae = (uintptr_t)(base + end);
  uint4 v[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
    if (a0 + 16 * k < ae) v[k] = *(const uint4 *)(a0 + 16 * k);
  // position of the window's first byte (negative when the haystack starts
  // mid-block)
  const int64_t p0 = (int64_t)at - (int64_t)((uintptr_t)(base + at) & 15);
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int64_t bp = p0 + 16 * k;
    if (L.done || bp >= (int64_t)end) break;
    const uint32_t k0 = bp < (int64_t)at ? (uint32_t)((int64_t)at - bp) : 0;
    const uint32_t kend = (int64_t)end - bp < 16 ? (uint32_t)((int64_t)end - bp) : 16;
    const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
    if (k0 == 0 && kend == 16) {
      uint32_t t = L.s, mx = 0;
      t = exact4(t, w[0], lds, mx);
      t = exact4(t, w[1], lds, mx);
      t = exact4(t, w[2], lds, mx);
      t = exact4(t, w[3], lds, mx);
      if (mx < f.n_normal) { L.s = t; continue; }
    }
    int lastk = -1;
    L.s = steps16(L.s, w, k0, kend, lds, f.n_normal, f.n_match_end, lastk);
    if (lastk >= 0) L.last = (uint64_t)(bp + lastk);  // Match(at - 1): the byte's position
    if (L.s >= f.n_match_end) {
      L.done = true;
      L.quit = L.s != f.dead;
    }
  }
}

// rev_scan (exec.rs:651-661, dfa.rs:768-866) for all-mode reverse tables:
// blocks walked backwards, bytes reversed in registers, branch-free steps.
// reached: as rev_scan's.
__device__ __forceinline__ uint64_t rev_scan_all(const RevDfaDev &r, const uint8_t *rlds, const uint8_t *base,
                                                 uint64_t len, uint64_t lo, uint64_t me, bool *reached = nullptr) {
  uint32_t s = r.ustart1 ? r.ustart1 - 1 : r.start[rev_flag_index(base, lo, len, me)];
  if (s == r.dead) return NONE;
  uint64_t rs = NONE, a = me;
  while (a > lo) {
    // up to 8 blocks below `a` loaded at once (their latencies overlap)
    const uintptr_t top = (uintptr_t)(base + a - 1) & ~(uintptr_t)15;
    const uintptr_t bot = (uintptr_t)(base + lo);
    uint4 vb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (top - 16 * k + 15 >= bot) vb[k] = *(const uint4 *)(top - 16 * k);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (a <= lo) break;
      const uintptr_t p = (uintptr_t)(base + a - 1);
      const uint4 v = vb[k];
      const uint32_t w[4] = {__builtin_bswap32(v.w), __builtin_bswap32(v.z), __builtin_bswap32(v.y),
                             __builtin_bswap32(v.x)};
      const uint32_t k0 = 15 - (uint32_t)(p & 15);  // reversed index of the byte at a - 1
      const uint32_t kend = a - lo < 16 - k0 ? k0 + (uint32_t)(a - lo) : 16;
      int lastk = -1;
      s = steps16(s, w, k0, kend, rlds, r.n_normal, r.n_match_end, lastk);
      if (lastk >= 0) rs = a - (uint32_t)(lastk - k0);  // the reverse match flag: start = byte position + 1
      a -= kend - k0;
      if (s >= r.n_match_end) return s == r.dead ? rs : QUITMARK;
    }
  }
  if (reached) *reached = true;
  if (r.eof[s]) rs = lo;
  return rs;
}

// Pass 1, burst-interleaved.  Written as a nest of loops per lane (forward
// scan to the dead state, reverse scan, restart; the round-1 kernel, deleted
// in round 5 after losing every A/B), a lane whose search ends early waits,
// masked off, until every other lane of its wave has finished its own
// forward loop — usually its whole unit — and then scans the rest of its
// unit alone.  Here the wave loop is over bursts: in
// each iteration every searching lane advances its current forward scan by
// at most one aligned 128-byte burst (the same LDS fast path, fwd_range); a
// lane whose scan ended does its reverse scan, applies the iteration rule
// (re_trait.rs:197-221) and sets up its next search (exec.rs:632-662) in
// the same iteration.
// abortf (a caller that re-runs the batch when a search quits): the first
// quit sets it, and every wave polls it every 16 bursts and stops (its unit
// records are then meaningless; the call reports the quit).
__global__ __launch_bounds__(1024) void iter_spec_burst_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f,
                                                              RevDfaDev r, Unit *units, uint64_t *slots,
                                                              uint32_t *counts, uint32_t *dirty, uint32_t *abortf,
                                                              uint32_t mode) {
  // mode bit 0: the wave-served iteration (a quit leaves the unit U_PEND);
  // bit 1: resume the U_RESUME units from their records, skip the others
  // (none when no unit was left pending: dirty bit 1)
  if (gated_off(b) || ((mode & 2) && !(__atomic_load_n(dirty, __ATOMIC_RELAXED) & 2u))) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint8_t *rlds = stage_tables(f, r, lds);
  for (uint64_t u0 = (uint64_t)blockIdx.x * blockDim.x; u0 < nunits; u0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = u0 + threadIdx.x;
    uint64_t h = 0, len = 0, c0 = 0, c1 = 0;
    const uint8_t *base = b.hay;
    uint64_t p = 0, lm = NONE, sp = 0, slm = NONE;  // iteration state and UnitIter's snapshot
    uint64_t at = 0, at0 = 0, cutpos = NONE;        // the current forward scan
    uint64_t ex_p = 0, ex_lm = NONE;
    bool clean = true, quit = false, searching = false;
    bool first = true, unsure = false;  // look-around: UnitIter's
    bool qfirst = false;                // the search that quit was the unit's first
    uint32_t n = 0;
    LaneState L;
    L.done = true;

    auto finish = [&](uint64_t ep, uint64_t elm, bool cl) {
      searching = false;
      ex_p = ep;
      ex_lm = elm;
      clean = cl;
    };
    auto begin_search = [&]() {  // iter_next's loop top
      if (p > len) { finish(sp, slm, true); return; }
      lane_start(L, f, base, len, p);
      at0 = at = p;
      cutpos = (c1 > p && c1 - 1 <= len) ? c1 - 1 : NONE;
      searching = true;
    };
    auto unit_next = [&]() {  // UnitIter::next's entry
      if (p >= c1) { finish(p, lm, p == c1 && (lm != c1 || f.nonempty)); return; }
      sp = p;
      slm = lm;
      begin_search();
    };
    bool active = u < nunits;
    if (active && (mode & 2)) {
      const Unit R0 = units[u];
      active = (R0.flags & U_RESUME) != 0;
      if (active) {
        p = R0.exit.p;
        lm = R0.exit.lm;
        n = R0.spec_count;
        first = R0.pad != 0;
        unsure = (R0.flags & U_UNSURE) != 0;
      }
    }
    if (active) {
      unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
      if (!(mode & 2)) p = c0;
      unit_next();
    }
    uint32_t polls = 0;
    while (__ballot(searching)) {
      if (abortf && (++polls & 15) == 0 &&
          __ballot(__hip_atomic_load(abortf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0))
        break;
      if (!searching) continue;
      if (at == cutpos) {  // dfa_find_cut: no new match may start at or after the cut
        L.s = f.strip[L.s];
        if (L.s == f.dead) L.done = true;
        cutpos = NONE;
      }
      if (!L.done && at < len) {
        uint64_t lim = (((uintptr_t)(base + at) & ~(uintptr_t)15) + 128) - (uintptr_t)base;
        lim = min(lim, len);
        if (cutpos != NONE) lim = min(lim, cutpos);
        if (f.all) fwd_window_all(L, f, lds, base, at, lim);
        else fwd_range<MODE_FIND>(L, f, lds, base, at, lim);
        at = lim;
      }
      if (!L.done && (at < len || cutpos == len)) continue;  // the scan goes on next burst
      // the forward scan ended: EOF step, reverse scan, iteration rule
      if (!L.done && f.eof[L.s]) L.last = len;
      if (L.quit) {
        quit = true;
        qfirst = first;
        if (abortf) atomicOr(abortf, 1u);
        finish(sp, slm, false);
        continue;
      }
      if (L.last == NONE) {
        // (iter_next: a start after a byte >= 0x80 with no match before the
        // cut is handed over as a quit)
        if (f.can_quit == 2 && at0 > 0 && at0 < c1 && base[at0 - 1] >= 0x80) {
          quit = true;
          qfirst = first;
          if (abortf) atomicOr(abortf, 1u);
          finish(sp, slm, false);
        } else {
          finish(sp, slm, true);
        }
        continue;
      }
      const uint64_t me = L.last;
      uint64_t ms = at0;
      bool reached = me == at0;
      if (me != at0) {  // exec.rs:647
        const uint64_t rs = r.all ? rev_scan_all(r, rlds, base, len, at0, me, &reached)
                                  : rev_scan(r, rlds, base, len, at0, me, &reached);
        const bool was_first = first;
        if (first) unsure = reached;
        first = false;
        if (rs == QUITMARK) {
          quit = true;
          qfirst = was_first;
          if (abortf) atomicOr(abortf, 1u);
          finish(sp, slm, false);
          continue;
        }
        if (rs == NONE) {  // look-around: the search's NoMatch ends the iteration
          if (f.looks) finish(kIterStop, NONE, false);
          else finish(sp, slm, true);
          continue;
        }
        ms = rs;
      }
      if (first) unsure = reached;
      first = false;
      if (ms == me) {
        p = me + 1;
        if (lm == me) { begin_search(); continue; }  // empty match at the previous match end: skipped
      } else {
        p = me;
      }
      lm = me;
      if (ms >= c1) { finish(sp, slm, true); continue; }  // owned by the next unit
      if (n < g.slots) {  // streaming stores: dense units write GBs of slots (5-7 % on \b\w+\b, [a-z]+)
        __builtin_nontemporal_store(ms, &slots[(u * g.slots + n) * 2]);
        __builtin_nontemporal_store(me, &slots[(u * g.slots + n) * 2 + 1]);
      }
      ++n;
      unit_next();
    }
    if (active) {
      Unit U;
      U.entry = {c0, NONE};
      U.exit = {ex_p, ex_lm};
      U.spec_exit = U.exit;
      U.spec_count = n;
      // (a unit after a byte >= 0x80 is unsure too when the DFA can quit: a
      // search from before its start reads that byte and quits, the fresh
      // one at c0 reads it as a non-word byte, dfa.rs:1423)
      const bool pre = f.can_quit == 2 && c0 > 0 && base[c0 - 1] >= 0x80;
      // (a resumed unit stays U_QUIT: one of its searches ran on the Pike VM)
      U.flags = (clean ? (U_SPEC_CLEAN | U_CLEAN) : 0) | (quit ? U_QUIT : 0) | (quit && (mode & 1) ? U_PEND : 0) |
                ((mode & 2) ? U_QUIT : 0) | (((f.looks && unsure) || pre) && u % g.nk != 0 ? U_UNSURE : 0);
      U.skip = 0;
      U.pad = quit && qfirst ? 1 : 0;  // (a quit unit: its exit is the state before the search that quit)
      units[u] = U;
      counts[u] = n;
      // (the fix pass has work; bit 1: some unit is pending, the wave rounds have work)
      if ((U.flags & (U_SPEC_CLEAN | U_UNSURE)) != U_SPEC_CLEAN) atomicOr(dirty, (U.flags & U_PEND) ? 3u : 1u);
    }
  }
}

// Pass 1 with the literal engine, for regexes that are a finite set of
// strings (host/literals.hpp; the reference runs its complete-prefix Literal
// engine for them, exec.rs:1148-1166, literals.rs:28-250).  A unit's
// speculative iteration needs no automaton: every start position is tested
// on its own — a hash of its first lit_k bytes against a 64 Kibit LDS bitmap
// of the literals' prefixes, the counterpart of Teddy's fingerprint filter
// (simd_accel/teddy128.rs) — so the 64 positions of a step are independent
// (no dependent chain per byte).  Hits are verified in priority order (the
// first literal that matches is the leftmost-first match) and the greedy
// iteration of re_trait.rs:197-221 keeps those starting at or after the
// previous match end (literals are non-empty).  The unit records are the
// same as iter_spec_burst_kernel's; repairs and the walker use the DFA.
// (lit_verify: dfa_device.hpp)
template <bool K4, bool K8>
__global__ __launch_bounds__(1024) void iter_spec_lit_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f,
                                                            Unit *units, uint64_t *slots, uint32_t *counts, uint32_t *dirty) {
  if (gated_off(b)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint32_t i = threadIdx.x * 16; i < f.lit_bytes; i += blockDim.x * 16)
    *(uint4 *)(lds + i) = *(const uint4 *)(f.lit_image + i);
  __syncthreads();
  const uint32_t *bitmap = (const uint32_t *)lds;
  const uint32_t *bitmap2 = (const uint32_t *)(lds + kLitBitmap2);
  const uint32_t kmask = K4 ? 0xFFFFFFFFu : ((1u << (8 * f.lit_k)) - 1);
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, len, c0, c1;
    const uint8_t *base;
    unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
    uint64_t p = c0, lm = NONE;
    uint32_t n = 0;
    // candidate starts: [c0, iend) — before the cut, room for the shortest literal
    const uint64_t iend = min(c1, len + 1 >= f.lit_minlen ? len + 1 - f.lit_minlen : 0);
    if (iend > c0) {
      const uintptr_t hi_blk = (uintptr_t)(base + len);
      const uintptr_t aend = (uintptr_t)(base + iend);
      for (uintptr_t a = (uintptr_t)(base + c0) & ~(uintptr_t)15; a < aend; a += 64) {
        uint64_t cand = lit_cands64<K4, K8>(a, hi_blk, bitmap, bitmap2, kmask);
        const int64_t p0 = (int64_t)(a - (uintptr_t)base);
        while (cand) {
          const int j = __builtin_ctzll(cand);
          cand &= cand - 1;
          const int64_t i = p0 + j;
          if (i < (int64_t)c0 || i < (int64_t)p || (uint64_t)i >= iend) continue;
          const int x = lit_verify(f, lds, base, len, (uint64_t)i);
          if (x < 0) continue;
          const uint64_t e = (uint64_t)i + lds[kLitLens + x];
          if (n < g.slots) *(ulonglong2 *)&slots[(u * g.slots + n) * 2] = make_ulonglong2((uint64_t)i, e);
          ++n;
          p = lm = e;
        }
      }
    }
    // UnitIter's exit: the state before the search that finds no owned match
    // (clean), or the end of a match running up to / past the cut
    Unit U;
    U.entry = {c0, NONE};
    U.exit = {p, lm};
    U.spec_exit = U.exit;
    U.spec_count = n;
    const bool clean = p < c1 || (p == c1 && (lm != c1 || f.nonempty));
    U.flags = clean ? (U_SPEC_CLEAN | U_CLEAN) : 0;
    U.skip = U.pad = 0;
    units[u] = U;
    counts[u] = n;
    if (!(U.flags & U_SPEC_CLEAN)) atomicOr(dirty, 1u);  // the fix pass has work
  }
}

// Pass 1 with the Shift-And engine, for string sets whose strings all have
// the same length L (host: sa_* fields; the regex-dna variants).  The set is
// a bit-parallel NFA (class sequences, one bit per position): per byte
// D = ((D << 1) | init) & mask[b] — the mask read does not depend on D, so a
// lane's dependent chain is two VALU operations per byte instead of an LDS
// round trip.  A sequence's last bit set after byte q is a string ending at
// q, i.e. the match [q - L + 1, q + 1); equal lengths make the leftmost-first
// match at a start unique and the iteration greedy on ends (re_trait.rs:
// 197-221).  A unit scans from c0 with D = 0 (starts < c0 are not its own)
// to c1 + L - 1, so it sees every string starting before its cut; blocks whose
// OR of final bits is zero (almost all) take no per-byte branch.  Same unit
// records as iter_spec_lit_kernel.
template <typename W>
__global__ __launch_bounds__(256) void iter_spec_sa_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f,
                                                           Unit *units, uint64_t *slots, uint32_t *counts,
                                                           uint32_t *dirty) {
  if (gated_off(b)) return;
  __shared__ W B[256];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) B[i] = (W)f.sa_image[i];
  __syncthreads();
  const W I = (W)f.sa_init, F = (W)f.sa_final;
  const uint64_t L = f.sa_len;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, len, c0, c1;
    const uint8_t *base;
    unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
    uint64_t p = c0, lm = NONE;
    uint32_t n = 0;
    const uint64_t qend = c1 >= len ? len : min(len, c1 + L - 1);  // last bytes q < qend
    W D = 0;
    if (qend > c0) {
      // 128-byte windows of 8 aligned blocks; the next window's loads are in
      // flight while this one is stepped
      const uintptr_t ae = (uintptr_t)(base + qend);
      uintptr_t a = (uintptr_t)(base + c0) & ~(uintptr_t)15;
      uint4 cur[8], nxt[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (a + 16 * k < ae) cur[k] = *(const uint4 *)(a + 16 * k);
      while (a < ae) {
        const uintptr_t an = a + 128;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (an + 16 * k < ae) nxt[k] = *(const uint4 *)(an + 16 * k);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uintptr_t ab = a + 16 * k;
          if (ab >= ae) break;
          const uint4 v = cur[k];
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          const int64_t bp = (int64_t)(ab - (uintptr_t)base);
          const uint32_t k0 = bp < (int64_t)c0 ? (uint32_t)((int64_t)c0 - bp) : 0;
          const uint32_t kend = (int64_t)qend - bp < 16 ? (uint32_t)((int64_t)qend - bp) : 16;
          const W D0 = D;
          W acc = 0;
          if (k0 == 0 && kend == 16) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              D = ((D << 1) | I) & B[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
              acc |= D & F;
            }
          } else {
#pragma unroll
            for (uint32_t j = 0; j < 16; ++j) {
              const W Dn = ((D << 1) | I) & B[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
              const bool act = j >= k0 && j < kend;
              D = act ? Dn : D;
              acc |= act ? (Dn & F) : (W)0;
            }
          }
          if (acc) {  // rare: the block holds string ends; walk it byte by byte
            W E = D0;
#pragma unroll 1
            for (uint32_t j = k0; j < kend; ++j) {
              E = ((E << 1) | I) & B[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
              if (E & F) {
                const uint64_t e = (uint64_t)bp + j + 1, st = e - L;
                if (st >= p && st < c1) {
                  if (n < g.slots) *(ulonglong2 *)&slots[(u * g.slots + n) * 2] = make_ulonglong2(st, e);
                  ++n;
                  p = lm = e;
                }
              }
            }
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        a = an;
      }
    }
    Unit U;
    U.entry = {c0, NONE};
    U.exit = {p, lm};
    U.spec_exit = U.exit;
    U.spec_count = n;
    const bool clean = p < c1 || (p == c1 && (lm != c1 || f.nonempty));
    U.flags = clean ? (U_SPEC_CLEAN | U_CLEAN) : 0;
    U.skip = U.pad = 0;
    units[u] = U;
    counts[u] = n;
    if (!(U.flags & U_SPEC_CLEAN)) atomicOr(dirty, 1u);  // the fix pass has work
  }
}

// iter_spec_sa_kernel with coalesced loads, for fixed-stride batches whose
// units are whole 128-byte lines at 16-byte aligned starts: one wave owns 64
// consecutive units and each load covers 8 units x one 128-byte line,
// transposed through a per-wave XOR-swizzled LDS stage (dfa_scan.hip's tile
// layout), so the scan reads HBM at the tile kernel's rate instead of the
// lane-per-unit rate.  The L - 1 bytes past a unit's cut (strings starting
// before it) come from the next unit's first 16 bytes, held by the next lane,
// or from memory for the wave's last lane.  The last unit of each haystack
// (ragged) runs the per-lane loop of iter_spec_sa_kernel.
template <typename W>
__device__ __forceinline__ void sa_block(W &D, const W *B, W I, W F, const uint32_t w[4], uint32_t k0, uint32_t kend,
                                         int64_t bp, uint64_t L, uint64_t c1, uint64_t &p, uint64_t &lm,
                                         uint32_t &n, uint64_t *myslots, uint32_t nslots) {
  const W D0 = D;
  W acc = 0;
  if (k0 == 0 && kend == 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      D = ((D << 1) | I) & B[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
      acc |= D & F;
    }
  } else {
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const W Dn = ((D << 1) | I) & B[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
      const bool act = j >= k0 && j < kend;
      D = act ? Dn : D;
      acc |= act ? (Dn & F) : (W)0;
    }
  }
  if (acc) {  // rare: the block holds string ends; walk it byte by byte
    W E = D0;
#pragma unroll 1
    for (uint32_t j = k0; j < kend; ++j) {
      E = ((E << 1) | I) & B[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
      if (E & F) {
        const uint64_t e = (uint64_t)bp + j + 1, st = e - L;
        if (st >= p && st < c1) {
          if (n < nslots) *(ulonglong2 *)&myslots[2 * n] = make_ulonglong2(st, e);
          ++n;
          p = lm = e;
        }
      }
    }
  }
}

template <typename W>
__device__ __forceinline__ void sa_unit_record(const FwdDfaDev &f, uint64_t u, uint64_t c0, uint64_t c1, uint64_t p,
                                               uint64_t lm, uint32_t n, Unit *units, uint32_t *counts,
                                               uint32_t *dirty) {
  Unit U;
  U.entry = {c0, NONE};
  U.exit = {p, lm};
  U.spec_exit = U.exit;
  U.spec_count = n;
  const bool clean = p < c1 || (p == c1 && (lm != c1 || f.nonempty));
  U.flags = clean ? (U_SPEC_CLEAN | U_CLEAN) : 0;
  U.skip = U.pad = 0;
  units[u] = U;
  counts[u] = n;
  if (!clean) atomicOr(dirty, 1u);  // the fix pass has work
}

template <typename W>
__global__ __launch_bounds__(256) void iter_spec_sa_tile_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f,
                                                                Unit *units, uint64_t *slots, uint32_t *counts,
                                                                uint32_t *dirty) {
  if (gated_off(b)) return;
  __shared__ W B[256];
  __shared__ __attribute__((aligned(16))) uint4 stage[4][64 * 8];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) B[i] = (W)f.sa_image[i];
  __syncthreads();
  const W I = (W)f.sa_init, F = (W)f.sa_final;
  const uint64_t L = f.sa_len, C = g.chunk, nk = g.nk;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  const int src_h = lane >> 3, src_seg = lane & 7, sw = (lane >> 1) & 7;
  const uint64_t ngroups = (nunits + 63) / 64, nwaves = (uint64_t)gridDim.x * 4;
  const bool single = b.count == 1;
  auto hk = [&](uint64_t uu, uint64_t &h, uint64_t &k) {
    if (single) { h = 0; k = uu; } else { h = uu / nk; k = uu - h * nk; }
  };
  for (uint64_t gi = (uint64_t)blockIdx.x * 4 + w; gi < ngroups; gi += nwaves) {
    const uint64_t u = gi * 64 + lane;
    uint64_t h, k;
    hk(u, h, k);
    const bool valid = u < nunits;
    const bool full = valid && k + 1 < nk;
    const uint8_t *src[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t us = gi * 64 + 8 * j + src_h, hs, ks;
      hk(us, hs, ks);
      if (us >= nunits || ks + 1 >= nk) hs = ks = 0;  // absent / ragged units re-read unit 0 (full)
      src[j] = b.hay + hs * b.stride + b.start + ks * C + 16 * src_seg;
    }
    const uint8_t *base = b.hay + h * b.stride;
    const uint64_t len = b.length, c0 = b.start + k * C;
    const uint64_t c1 = k + 1 == nk ? g.end : c0 + C;
    uint64_t *myslots = slots + u * g.slots * 2;
    uint64_t p = c0, lm = NONE;
    uint32_t n = 0;
    W D = 0;
    uint4 first = make_uint4(0, 0, 0, 0);
    uint4 n0, n1, n2, n3, n4, n5, n6, n7;
#define RURE_LOAD_TILE(a)                                                                                     \
  n0 = *(const uint4 *)(src[0] + (a)); n1 = *(const uint4 *)(src[1] + (a));                                  \
  n2 = *(const uint4 *)(src[2] + (a)); n3 = *(const uint4 *)(src[3] + (a));                                  \
  n4 = *(const uint4 *)(src[4] + (a)); n5 = *(const uint4 *)(src[5] + (a));                                  \
  n6 = *(const uint4 *)(src[6] + (a)); n7 = *(const uint4 *)(src[7] + (a));
#define RURE_STAGE(kk, v) buf[(8 * (kk) + src_h) * 8 + (src_seg ^ (((8 * (kk) + src_h) >> 1) & 7))] = (v);
    RURE_LOAD_TILE(0)
    for (uint64_t at = 0; at < C; at += 128) {
      RURE_STAGE(0, n0) RURE_STAGE(1, n1) RURE_STAGE(2, n2) RURE_STAGE(3, n3)
      RURE_STAGE(4, n4) RURE_STAGE(5, n5) RURE_STAGE(6, n6) RURE_STAGE(7, n7)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint64_t an = at + 128 < C ? at + 128 : at;
      RURE_LOAD_TILE(an)
      if (full) {
        uint4 cur = buf[lane * 8 + sw];
        if (at == 0) first = cur;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const uint4 nx = buf[lane * 8 + ((m + 1 < 8 ? m + 1 : 7) ^ sw)];
          const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
          sa_block<W>(D, B, I, F, wd, 0, 16, (int64_t)(c0 + at + 16 * m), L, c1, p, lm, n, myslots, g.slots);
          cur = nx;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#undef RURE_LOAD_TILE
#undef RURE_STAGE
    // the next unit's first 16 bytes from the next lane (its unit follows
    // this one in memory when this one is full)
    uint4 nxt;
    nxt.x = __shfl_down(first.x, 1);
    nxt.y = __shfl_down(first.y, 1);
    nxt.z = __shfl_down(first.z, 1);
    nxt.w = __shfl_down(first.w, 1);
    if (!valid) continue;
    if (full) {
      // strings starting before the cut end in [c1, c1 + L - 1)
      const uint64_t qend = min(len, c1 + L - 1);
      uint64_t q = c1;
      if (q < qend && lane < 63 && k + 2 < nk) {  // the next unit is full: lane + 1 holds its first block
        const uint32_t wd[4] = {nxt.x, nxt.y, nxt.z, nxt.w};
        const uint32_t kend = qend - q < 16 ? (uint32_t)(qend - q) : 16;
        sa_block<W>(D, B, I, F, wd, 0, kend, (int64_t)q, L, c1, p, lm, n, myslots, g.slots);
        q += 16;
      }
      for (; q < qend; q += 16) {  // from memory (aligned: c1 is)
        const uint4 v = *(const uint4 *)(base + q);
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        const uint32_t kend = qend - q < 16 ? (uint32_t)(qend - q) : 16;
        sa_block<W>(D, B, I, F, wd, 0, kend, (int64_t)q, L, c1, p, lm, n, myslots, g.slots);
      }
    } else {
      // ragged last unit of its haystack: the per-lane loop
      const uint64_t qend = c1 >= len ? len : min(len, c1 + L - 1);
      for (uintptr_t a = (uintptr_t)(base + c0) & ~(uintptr_t)15; c0 < qend && a < (uintptr_t)(base + qend); a += 16) {
        const uint4 v = *(const uint4 *)a;
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        const int64_t bp = (int64_t)(a - (uintptr_t)base);
        const uint32_t k0 = bp < (int64_t)c0 ? (uint32_t)((int64_t)c0 - bp) : 0;
        const uint32_t kend = (int64_t)qend - bp < 16 ? (uint32_t)((int64_t)qend - bp) : 16;
        sa_block<W>(D, B, I, F, wd, k0, kend, bp, L, c1, p, lm, n, myslots, g.slots);
      }
    }
    sa_unit_record<W>(f, u, c0, c1, p, lm, n, units, counts, dirty);
  }
}

// ------------------------------------------------------------------------
// Several Shift-And regexes over one text in one pass (rure_amd_find_iter_
// span_multi; regex-dna's 9 variants read the stripped stream once instead of
// 9 times).  Every regex keeps its own bits (packed into NW 32-bit words: a
// word's sequences step together, the init bits re-arm each sequence's first
// bit whatever the previous one shifted in), its own greedy iteration state
// and its own unit records, so the per-regex passes after this one (fix,
// walk, emit) are unchanged and each regex's matches are exactly its own
// find_iter's.  All regexes share one string length L and the unit geometry.
constexpr int kSaMultiMax = 12, kSaMultiWords = 8;
// Regexes of at most 32 bits each, packed into 32-bit words (a regex never
// straddles two words, so a byte's step is one v_lshl_or + one v_and per
// word, with no carries between words).
struct SaMulti {
  uint32_t *image;                    // [256][NW] combined masks (device, built by sa_multi_image_kernel)
  uint32_t init[kSaMultiWords], facc[kSaMultiWords];  // per word: init bits, final bits of its regexes
  uint32_t fany;                      // the OR of facc
  uint64_t len;                       // the common string length L
  uint32_t nre;
  uint32_t word[kSaMultiMax];         // word of regex x
  uint32_t shift[kSaMultiMax];        // bit offset of regex x in its word
  uint32_t fin[kSaMultiMax];          // final bits of regex x (in its word)
  uint32_t nonempty[kSaMultiMax];
  const uint64_t *sa_image[kSaMultiMax];  // each regex's own 256 masks
  Unit *units[kSaMultiMax];
  uint64_t *slots[kSaMultiMax];
  uint32_t *counts[kSaMultiMax];
  uint32_t *dirty[kSaMultiMax];
  KmerDev km;                         // k-mer probe engine (km.bitmap != nullptr)
  uint32_t pbits;                     // per-regex state: search position bits (multi_record)
};

// LDS rows of NWP = 4 or 8 words (16-byte reads)
template <int NW> struct SamPitch { static constexpr int v = NW <= 4 ? 4 : 8; };

template <int NW>
__global__ void sa_multi_image_kernel(SaMulti m) {
  const uint32_t c = threadIdx.x;  // 256 threads: one byte value each
  uint32_t wv[NW];
#pragma unroll
  for (int x = 0; x < NW; ++x) wv[x] = 0;
  for (uint32_t q = 0; q < m.nre; ++q) {
    const uint32_t v = (uint32_t)m.sa_image[q][c] << m.shift[q];
#pragma unroll
    for (int x = 0; x < NW; ++x)
      if (m.word[q] == (uint32_t)x) wv[x] |= v;
  }
#pragma unroll
  for (int x = 0; x < SamPitch<NW>::v; ++x) m.image[c * SamPitch<NW>::v + x] = x < NW ? wv[x] : 0u;
}

// Each regex's greedy iteration state in the fused pass, one u32 per regex
// and lane (registers bound the kernel's occupancy): the end of its last
// match relative to the unit start (its next search starts there) in the low
// m.pbits bits, its match count above (the host checks both fit).  The last
// match end equals the search position once a match was seen (nonempty
// strings), so it needs no register of its own.
template <int MQ>
__device__ __forceinline__ void multi_record(const SaMulti &m, uint32_t (&pn)[MQ], int q, uint64_t st, uint64_t e,
                                             uint64_t c0, uint64_t c1, uint64_t u, uint32_t nslots) {
  const uint32_t pmask = (1u << m.pbits) - 1u;
  const uint32_t pq = pn[q] & pmask, nq = pn[q] >> m.pbits;
  if (st >= c0 + pq && st < c1) {
    if (nq < nslots) *(ulonglong2 *)&m.slots[q][(u * nslots + nq) * 2] = make_ulonglong2(st, e);
    pn[q] = (uint32_t)(e - c0) | ((nq + 1) << m.pbits);
  }
}

// sam_block for every regex of the pass: the bits of 16 bytes (k0..kend) and,
// in the rare block holding string ends, each regex's greedy iteration.
template <int NW>
__device__ __forceinline__ void sam_row(const uint32_t *B, uint32_t c, uint32_t (&row)[NW]) {
  const uint4 *r = (const uint4 *)(B + c * SamPitch<NW>::v);
  const uint4 a = r[0];
  const uint32_t t[8] = {a.x, a.y, a.z, a.w, 0, 0, 0, 0};
  uint32_t u[8] = {t[0], t[1], t[2], t[3], 0, 0, 0, 0};
  if (NW > 4) { const uint4 b2 = r[1]; u[4] = b2.x; u[5] = b2.y; u[6] = b2.z; u[7] = b2.w; }
#pragma unroll
  for (int x = 0; x < NW; ++x) row[x] = u[x];
}

template <int NW, int MQ>
__device__ __forceinline__ void sam_block(uint32_t (&D)[NW], const uint32_t *B, const SaMulti &m, const uint32_t w[4],
                                          uint32_t k0, uint32_t kend, int64_t bp, uint64_t c0, uint64_t c1,
                                          uint32_t (&pn)[MQ], uint64_t u, uint32_t nslots) {
  uint32_t D0[NW];
#pragma unroll
  for (int x = 0; x < NW; ++x) D0[x] = D[x];
  if (k0 == 0 && kend == 16) {
    // Whole block: fm = the bytes after which some word holds a final bit
    // (with 9 variants ~57% of wave-blocks hold one somewhere), and Dm = the
    // words after the last such byte, so a block with one such byte (almost
    // all of them) settles its matches without a second walk.
    uint32_t fm = 0, Dm[NW];
#pragma unroll
    for (int x = 0; x < NW; ++x) Dm[x] = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t row[NW];
      sam_row<NW>(B, (w[j >> 2] >> (8 * (j & 3))) & 0xFF, row);
      uint32_t t = 0;
#pragma unroll
      for (int x = 0; x < NW; ++x) {
        D[x] = ((D[x] << 1) | m.init[x]) & row[x];
        t |= D[x];
      }
      const bool hit = (t & m.fany) != 0;
      fm |= hit ? (1u << j) : 0u;
#pragma unroll
      for (int x = 0; x < NW; ++x) {
        Dm[x] = hit ? D[x] : Dm[x];
        asm volatile("" : "+v"(Dm[x]));  // per byte: no copies of D kept for later selects
      }
      asm volatile("" : "+v"(fm));
    }
    if (!fm) return;
    if (__builtin_popcount(fm) == 1) {
      const uint32_t j = __builtin_ctz(fm);
      const uint64_t e = (uint64_t)bp + j + 1, st = e - m.len;
#pragma unroll
      for (int q = 0; q < MQ; ++q) {
        if ((uint32_t)q >= m.nre) break;
        uint32_t ew = Dm[0];
#pragma unroll
        for (int x = 1; x < NW; ++x) ew = m.word[q] == (uint32_t)x ? Dm[x] : ew;
        if (ew & m.fin[q]) multi_record<MQ>(m, pn, q, st, e, c0, c1, u, nslots);
      }
      return;
    }
  } else {
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      uint32_t row[NW];
      sam_row<NW>(B, (w[j >> 2] >> (8 * (j & 3))) & 0xFF, row);
      const bool act = j >= k0 && j < kend;
#pragma unroll
      for (int x = 0; x < NW; ++x) {
        const uint32_t Dn = ((D[x] << 1) | m.init[x]) & row[x];
        D[x] = act ? Dn : D[x];
        acc |= act ? Dn : 0u;
      }
    }
    if (!(acc & m.fany)) return;
  }
  // rare: the block holds string ends; walk it byte by byte
  uint32_t E[NW];
#pragma unroll
  for (int x = 0; x < NW; ++x) E[x] = D0[x];
#pragma unroll 1
  for (uint32_t j = k0; j < kend; ++j) {
    uint32_t row[NW];
    sam_row<NW>(B, (w[j >> 2] >> (8 * (j & 3))) & 0xFF, row);
    uint32_t any = 0;
#pragma unroll
    for (int x = 0; x < NW; ++x) {
      E[x] = ((E[x] << 1) | m.init[x]) & row[x];
      any |= E[x] & m.facc[x];
    }
    if (!any) continue;
    const uint64_t e = (uint64_t)bp + j + 1, st = e - m.len;
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      if ((uint32_t)q >= m.nre) break;
      uint32_t ew = E[0];
#pragma unroll
      for (int x = 1; x < NW; ++x) ew = m.word[q] == (uint32_t)x ? E[x] : ew;
      if (ew & m.fin[q]) multi_record<MQ>(m, pn, q, st, e, c0, c1, u, nslots);
    }
  }
}

// The k-mer probe engine (KmerDev): the 2-bit codes of a block's 16 bytes
// (code(b) = (b >> shift) & 3, four bytes per VALU op) join the previous
// block's in a 64-bit window register; the L-mer ending at each byte is one
// independent probe of the LDS bitmap of the strings' codes (no dependent
// chain).  The probes' random dwords cost ~4.6 bank-conflict cycles per LDS
// read (C3: 171M conflict cycles, 37.5M LDS instructions); a conflict-free
// 32-dword prefilter (1.4% of the 10-bit prefixes hit on regex-dna) with
// the exact bitmap read for its hits cut them to 15M but added a dependent
// LDS round trip and ~45 VALU per block: 0.78-0.86 ms against 0.69
// (round 5, profiles/r05_c3_ab.txt), so the direct probe stays.
// Returns the probe hits (bit j: the L-mer ending at byte j).  Rp:
// the previous block's codes (garbage before a unit's first block: the
// windows reaching into it start before the unit and are dropped by
// kmer_hit).
template <int KL>
__device__ __forceinline__ uint32_t kmer_probe(uint32_t &Rp, const uint32_t *B, const KmerDev &km,
                                               const uint32_t w[4]) {
  // four codes per word packed by one v_dot4_u32_u8 (byte weights 1, 4,
  // 16, 64 on the codes left in place at bit `shift` of each byte)
  const uint32_t M = 0x03030303u << km.shift;
  uint32_t d[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) d[x] = __builtin_amdgcn_udot4(w[x] & M, 0x40100401u, 0u, false);
  uint32_t cw = d[0] >> km.shift;
#pragma unroll
  for (int x = 1; x < 4; ++x) cw |= d[x] << (8 * x - km.shift);
  // The window of the KL-mer ending at byte j starts at bit sh = 2 (17 + j -
  // KL) of cw:Rp.  Its bitmap dword is bits [sh + 5, sh + 2 KL) (address:
  // shifted to bit 2), its bit within the dword bits [sh, sh + 5) (v_bfe_u32
  // reads only the low 5 bits of the offset).
  constexpr uint32_t amask = ((1u << (2 * KL)) - 1u) >> 5 << 2;
  const uint8_t *Bb = (const uint8_t *)B;
  uint32_t cm = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    constexpr int base_sh = 2 * (17 - KL);
    const int sh = base_sh + 2 * j;
    const uint32_t lo = sh >= 32 ? (cw >> (sh - 32)) : __builtin_amdgcn_alignbit(cw, Rp, sh);
    const uint32_t hi = sh + 3 >= 32 ? (cw >> (sh + 3 - 32)) : __builtin_amdgcn_alignbit(cw, Rp, sh + 3);
    const uint32_t word = *(const uint32_t *)(Bb + (hi & amask));
    cm |= __builtin_amdgcn_ubfe(word, lo, 1) << j;
  }
  Rp = cw;
  return cm;
}

// One probe hit: the KL-mer ending before e.  Verified on the text bytes
// (exact whatever the input: a byte outside the alphabet fails; the eight
// loads issue together), then its code's regex mask drives each regex's
// greedy iteration exactly as sam_block does.
template <int MQ, int KL>
__device__ __forceinline__ void kmer_hit(const SaMulti &m, uint64_t e, uint64_t c0, uint64_t c1,
                                         uint32_t (&pn)[MQ], uint64_t u, uint32_t nslots, const uint8_t *base) {
  const KmerDev &km = m.km;
  if (e < (uint64_t)KL || e - KL < c0) return;  // starts before the unit: not its match
  const uint64_t st = e - KL;
  uint32_t code = 0, bad = 0;
#pragma unroll
  for (int i = 0; i < KL; ++i) {
    const uint32_t bb = base[st + i], c = (bb >> km.shift) & 3u;
    bad |= (((km.lut >> (8 * c)) & 0xFFu) ^ bb) | (~(km.present >> c) & 1u);
    code |= c << (2 * i);
  }
  if (bad) return;
  const uint32_t mask = km.mask[code];
#pragma unroll
  for (int q = 0; q < MQ; ++q) {
    if ((uint32_t)q >= m.nre) break;
    if ((mask >> q) & 1u) multi_record<MQ>(m, pn, q, st, e, c0, c1, u, nslots);
  }
}

// kmer_hit for the tile loop, from LDS only: the 8-mer ending at byte p of
// the staged line (bytes before the line: the previous line's last 8, pz:pw)
// is read back from the wave's stage buffer, checked against the alphabet
// (four bytes per v_perm: the byte each code stands for, KmerDev::vlut) and
// its regex mask read from the LDS perfect hash HT (KmerDev::hmul).  kmer_hit
// takes two dependent global round trips (the bytes, then mask[code]), which
// the wave waited for once per line.
template <int MQ>
__device__ __forceinline__ void kmer_hit_lds(const SaMulti &m, const uint16_t *HT, const uint4 *buf, int lane, int sw,
                                             uint32_t p, uint32_t pz, uint32_t pw, uint64_t ls, uint64_t c0,
                                             uint64_t c1, uint32_t (&pn)[MQ], uint64_t u, uint32_t nslots) {
  const KmerDev &km = m.km;
  const uint64_t e = ls + p + 1;
  if (e < 8 || e - 8 < c0) return;  // starts before the unit: not its match
  // virtual dwords: 0, 1 = pz, pw; 2 + 4 b + r = dword r of the line's block b
  const uint32_t v0 = p + 1, d0 = v0 >> 2, sh = 8 * (v0 & 3);
  const uint32_t *bw = (const uint32_t *)(buf + lane * 8);
  uint32_t dw[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint32_t d = d0 + i, ld = d >= 2 ? min(d - 2, 31u) : 0u;
    const uint32_t x = bw[(((ld >> 2) ^ (uint32_t)sw) << 2) | (ld & 3)];
    dw[i] = d == 0 ? pz : d == 1 ? pw : x;
  }
  const uint32_t lo = __builtin_amdgcn_alignbit(dw[1], dw[0], sh), hi = __builtin_amdgcn_alignbit(dw[2], dw[1], sh);
  const uint32_t M = 0x03030303u << km.shift;
  const uint32_t cl = (lo & M) >> km.shift, ch = (hi & M) >> km.shift;  // one code per byte
  if ((__builtin_amdgcn_perm(0u, km.vlut, cl) ^ lo) | (__builtin_amdgcn_perm(0u, km.vlut, ch) ^ hi)) return;
  const uint32_t code =
      __builtin_amdgcn_udot4(cl, 0x40100401u, 0u, false) | (__builtin_amdgcn_udot4(ch, 0x40100401u, 0u, false) << 8);
  // (a set with no injective 10-bit hash: the global table, one round trip)
  const uint32_t mask = km.hglobal ? km.mask[code] : HT[(code * km.hmul) >> 22];
  const uint64_t st = e - 8;
#pragma unroll
  for (int q = 0; q < MQ; ++q) {
    if ((uint32_t)q >= m.nre) break;
    if ((mask >> q) & 1u) multi_record<MQ>(m, pn, q, st, e, c0, c1, u, nslots);
  }
}

// The k-mer engine's step of one block with its hits settled at once (the
// tail paths; the tile loop defers a line's hits to its end, see
// multi_tile_body): bytes k0..kend of the block at bp.
template <int MQ, int KL>
__device__ __forceinline__ void kmer_block(uint32_t &Rp, const uint32_t *B, const SaMulti &m, const uint32_t w[4],
                                           uint32_t k0, uint32_t kend, int64_t bp, uint64_t c0, uint64_t c1,
                                           uint32_t (&pn)[MQ], uint64_t u, uint32_t nslots, const uint8_t *base) {
  uint32_t cm = kmer_probe<KL>(Rp, B, m.km, w);
  cm &= ((kend >= 32 ? 0u : (1u << kend)) - 1u) & ~((1u << k0) - 1u);
#pragma unroll 1
  while (cm) {
    const uint32_t j = __builtin_ctz(cm);
    cm &= cm - 1;
    kmer_hit<MQ, KL>(m, (uint64_t)bp + j + 1, c0, c1, pn, u, nslots, base);
  }
}

// One regex-set step of a block for the tile kernel below: the Shift-And
// words (KMER = false) or the k-mer probes (KMER = true; D[0] holds Rp).
template <int NW, bool KMER, int MQ>
__device__ __forceinline__ void multi_block(uint32_t (&D)[NW], const uint32_t *B, const SaMulti &m,
                                            const uint32_t w[4], uint32_t k0, uint32_t kend, int64_t bp, uint64_t c0,
                                            uint64_t c1, uint32_t (&pn)[MQ], uint64_t u, uint32_t nslots,
                                            const uint8_t *base) {
  if (KMER) kmer_block<MQ, 8>(D[0], B, m, w, k0, kend, bp, c0, c1, pn, u, nslots, base);
  else sam_block<NW, MQ>(D, B, m, w, k0, kend, bp, c0, c1, pn, u, nslots);
}

// The fused speculative pass over ONE haystack span (b.count == 1): the
// coalesced tile layout of iter_spec_sa_tile_kernel (a wave owns 64
// consecutive units; each load covers 8 units x one 128-byte line, staged
// through a swizzled LDS buffer), each lane running every regex of the pass
// over its unit.  MQ >= m.nre bounds the per-regex state arrays.
template <int NW, bool KMER, int MQ, int WPB = 4>
__device__ __forceinline__ void multi_tile_body(const BatchDev &b, const Geo &g, uint64_t nunits, const SaMulti &m) {
  // one LDS object, the table first: its probes' addresses need no base
  // (the compiler placed a separate stage array first and added its size to
  // every probe address: one VALU per byte); k-mer: the bitmap, then the
  // regex masks' perfect hash of kmer_hit_lds
  struct __attribute__((aligned(16))) Lds {
    uint32_t B[KMER ? 2048 : 256 * SamPitch<NW>::v];
    uint16_t HT[KMER ? 1024 : 2];
    uint4 stage[WPB][64 * 8];
  };
  __shared__ Lds lds_;
  uint32_t *const B = lds_.B;
  uint4 (*const stage)[64 * 8] = lds_.stage;
  if (KMER) {
    for (uint32_t i = threadIdx.x; i < 2048; i += blockDim.x) B[i] = m.km.bitmap[i];
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) lds_.HT[i] = m.km.hmask[i];
  } else {
    for (uint32_t i = threadIdx.x; i < 256 * SamPitch<NW>::v; i += blockDim.x) B[i] = m.image[i];
  }
  __syncthreads();
  const uint64_t L = m.len, C = g.chunk, nk = g.nk;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  const int src_h = lane >> 3, src_seg = lane & 7, sw = (lane >> 1) & 7;
  const uint64_t ngroups = (nunits + 63) / 64, nwaves = (uint64_t)gridDim.x * WPB;
  const uint8_t *const base = b.hay;  // one haystack
  const uint64_t len = b.length;
  for (uint64_t gi = (uint64_t)blockIdx.x * WPB + w; gi < ngroups; gi += nwaves) {
    const uint64_t u = gi * 64 + lane, k = u;
    const bool valid = u < nunits;
    const bool full = valid && k + 1 < nk;
    // tile sources: load j covers units gi*64 + 8 j + src_h (absent / ragged
    // units re-read unit 0, which is full), addresses formed per load
    const uint64_t us0 = gi * 64 + src_h;
    const uint8_t *const src0 = base + b.start + 16 * src_seg;
    const uint64_t c0 = b.start + k * C;
    const uint64_t c1 = k + 1 == nk ? g.end : c0 + C;
    uint32_t pn[MQ];
#pragma unroll
    for (int q = 0; q < MQ; ++q) pn[q] = 0;
    uint32_t D[NW];
#pragma unroll
    for (int x = 0; x < NW; ++x) D[x] = 0;
    uint4 n0, n1, n2, n3, n4, n5, n6, n7;
    uint32_t pz = 0, pw = 0;  // k-mer: the previous line's last 8 bytes (kmer_hit_lds)
#define RURE_SRC(j, a) (src0 + ((us0 + 8 * (j) + 1 < nk) ? (us0 + 8 * (j)) * C : 0) + (a))
#define RURE_LOAD_TILE(a)                                                                                     \
  n0 = *(const uint4 *)RURE_SRC(0, a); n1 = *(const uint4 *)RURE_SRC(1, a);                                  \
  n2 = *(const uint4 *)RURE_SRC(2, a); n3 = *(const uint4 *)RURE_SRC(3, a);                                  \
  n4 = *(const uint4 *)RURE_SRC(4, a); n5 = *(const uint4 *)RURE_SRC(5, a);                                  \
  n6 = *(const uint4 *)RURE_SRC(6, a); n7 = *(const uint4 *)RURE_SRC(7, a);
#define RURE_STAGE(kk, v) buf[(8 * (kk) + src_h) * 8 + (src_seg ^ (((8 * (kk) + src_h) >> 1) & 7))] = (v);
    RURE_LOAD_TILE(0)
    for (uint64_t at = 0; at < C; at += 128) {
      RURE_STAGE(0, n0) RURE_STAGE(1, n1) RURE_STAGE(2, n2) RURE_STAGE(3, n3)
      RURE_STAGE(4, n4) RURE_STAGE(5, n5) RURE_STAGE(6, n6) RURE_STAGE(7, n7)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint64_t an = at + 128 < C ? at + 128 : at;
      RURE_LOAD_TILE(an)
      if constexpr (KMER) {
        // The line's probe hits collect in a 128-bit shift register (block
        // mm at bits 16 mm) and are settled after the line: the block loop
        // issues no global load, so nothing in it waits on the next line's
        // tile loads in flight (one vmcnt counter, in order).  Every lane
        // runs the block loop (a lane without a full unit probes staged
        // bytes of unit 0 and drops its hits): the probes' exec mask stays
        // whole.
        uint4 cur = buf[lane * 8 + sw];
        // (two blocks per iteration: a pair's hits are one word of the
        // register, shifted in by moves; after the loop cur is block 7)
        uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
#pragma unroll 1
        for (int mm = 0; mm < 8; mm += 2) {
          uint32_t pair = 0;
#pragma unroll
          for (int x = 0; x < 2; ++x) {
            const uint4 nx = buf[lane * 8 + ((mm + x + 1 < 8 ? mm + x + 1 : 7) ^ sw)];
            const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
            const uint32_t cm = kmer_probe<8>(D[0], B, m.km, wd);
            pair |= cm << (16 * x);
            cur = nx;
          }
          h0 = h1;
          h1 = h2;
          h2 = h3;
          h3 = pair;
        }
        if (full) {
          // one loop over the line's 128 hit bits: the wave iterates as
          // often as its lane with the most hits (mostly once), not once per
          // word holding a hit in some lane
#pragma unroll 1
          while (h0 | h1 | h2 | h3) {
            const uint32_t x = h0 ? 0u : h1 ? 1u : h2 ? 2u : 3u;
            const uint32_t hm = x == 0 ? h0 : x == 1 ? h1 : x == 2 ? h2 : h3;
            const uint32_t j = __builtin_ctz(hm), rest = hm & (hm - 1);
            h0 = x == 0 ? rest : h0;
            h1 = x == 1 ? rest : h1;
            h2 = x == 2 ? rest : h2;
            h3 = x == 3 ? rest : h3;
            kmer_hit_lds<MQ>(m, lds_.HT, buf, lane, sw, 32 * x + j, pz, pw, c0 + at, c0, c1, pn, u, g.slots);
          }
        }
        pz = cur.z;
        pw = cur.w;
      } else if (full) {
        uint4 cur = buf[lane * 8 + sw];
#pragma unroll 1
        for (int mm = 0; mm < 8; ++mm) {
          const uint4 nx = buf[lane * 8 + ((mm + 1 < 8 ? mm + 1 : 7) ^ sw)];
          const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
          multi_block<NW, KMER, MQ>(D, B, m, wd, 0, 16, (int64_t)(c0 + at + 16 * mm), c0, c1, pn, u, g.slots,
                                    base);
          cur = nx;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#undef RURE_LOAD_TILE
#undef RURE_STAGE
#undef RURE_SRC
    if (!valid) continue;
    if (full) {
      // strings starting before the cut end in [c1, c1 + L - 1): the next
      // unit's first bytes, from memory (aligned: c1 is; keeping the tile's
      // first block for a shuffle held 4 more VGPRs over the whole loop)
      const uint64_t qend = min(len, c1 + L - 1);
      for (uint64_t q = c1; q < qend; q += 16) {
        const uint4 v = *(const uint4 *)(base + q);
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        const uint32_t kend = qend - q < 16 ? (uint32_t)(qend - q) : 16;
        multi_block<NW, KMER, MQ>(D, B, m, wd, 0, kend, (int64_t)q, c0, c1, pn, u, g.slots, base);
      }
    } else {
      // ragged last unit of its haystack: the per-lane loop
      const uint64_t qend = c1 >= len ? len : min(len, c1 + L - 1);
      for (uintptr_t a = (uintptr_t)(base + c0) & ~(uintptr_t)15; c0 < qend && a < (uintptr_t)(base + qend); a += 16) {
        const uint4 v = *(const uint4 *)a;
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        const int64_t bp = (int64_t)(a - (uintptr_t)base);
        const uint32_t k0 = bp < (int64_t)c0 ? (uint32_t)((int64_t)c0 - bp) : 0;
        const uint32_t kend = (int64_t)qend - bp < 16 ? (uint32_t)((int64_t)qend - bp) : 16;
        multi_block<NW, KMER, MQ>(D, B, m, wd, k0, kend, bp, c0, c1, pn, u, g.slots, base);
      }
    }
    const uint32_t pmask = (1u << m.pbits) - 1u;
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      if ((uint32_t)q >= m.nre) break;
      const uint32_t nq = pn[q] >> m.pbits;
      const uint64_t pq = c0 + (pn[q] & pmask), lq = nq ? pq : NONE;
      Unit U;
      U.entry = {c0, NONE};
      U.exit = {pq, lq};
      U.spec_exit = U.exit;
      U.spec_count = nq;
      const bool clean = pq < c1 || (pq == c1 && (lq != c1 || m.nonempty[q]));
      U.flags = clean ? (U_SPEC_CLEAN | U_CLEAN) : 0;
      U.skip = U.pad = 0;
      m.units[q][u] = U;
      m.counts[q][u] = nq;
      if (!clean) atomicOr(m.dirty[q], 1u);  // the fix pass has work
    }
  }
}

// Pass 1 with the lexer table (FwdDfaDev::lex_image, host build_lex), for
// patterns whose matches all end in terminal states and start at the first
// byte of F (the regex-dna strip pattern `>[^\n]*\n|\n`): the iteration is a
// DFA walk with no reverse scans and no restarts — a byte whose transition
// would enter a match state instead enters the start state's successor on
// that byte, flagged kLexEmit.  Per byte the chain is a mask, an add and one
// LDS u16 read; the entry's two flag bits go into a 32-bit word per 16-byte
// block (EMIT = a match [start, x) ended at byte x; Z = the next state is the
// start state).  A match's start is the last position before it where the
// state before the byte was the start state or a match had just ended
// (first-byte rule), read off those words.  Coalesced tiles as in
// iter_spec_sa_tile_kernel.  The lexer covers [c0, c1 - 1); from there
// iter_lex_tail_kernel's generic cut-bounded iteration (UnitIter) finishes
// the search in progress at the cut or at the end of the text, and a unit's
// rest from its last match before a block holding a byte >= 0x80 (the
// first-byte rule is proven for ASCII); a separate pass keeps this kernel's
// registers to its byte loop.  Ragged last units run in the tile loop with
// their loads clamped to the batch.  Together: the unit records of
// iter_spec_burst_kernel.
// 16 lexer steps; FULL = false: only bytes [0, kend) (kend < 16), the rest
// leave s unchanged and add no flags.  The chain per byte is one 24-bit
// multiply-add and one LDS u8 read (as the tile kernel's); the flags are the
// entry's low two bits (FwdDfaDev::lex_image), two bits per byte of the
// returned word.
template <bool FULL>
__device__ __forceinline__ uint32_t lex16(uint32_t &s, const uint32_t w[4], const uint8_t *tab, uint32_t kend) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t t = tab[__umul24(s, kLexUnit) + ((w[k >> 2] >> (8 * (k & 3))) & 0xFF)];
    if (FULL || k < kend) {
      m |= (t & 3u) << (2 * k);
      s = t;
    }
  }
  return m;
}

// lex16 four bytes per step (FwdDfaDev::lex4_image, host build_lex4): per
// 4-byte word four independent class lookups (off the chain), then one
// dependent LDS read for the next row and one for the four bytes' flags.
// The chain is a quarter as long and the VALU per byte halves (the byte
// lexer: byte extract, 24-bit multiply-add, flag shift and mask per byte).
// s is a row number here.  FULL = false: bytes from kend on take class 3
// (no byte: state kept, no flags).
template <bool FULL>
__device__ __forceinline__ uint32_t lex16x4(uint32_t &s, const uint32_t w[4], const uint8_t *tab, uint32_t kend) {
  uint32_t c[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t x = w[j];
    c[j] = tab[kLex4Cls + (x & 0xFF)] | tab[kLex4Cls + 256 + ((x >> 8) & 0xFF)] |
           tab[kLex4Cls + 512 + ((x >> 16) & 0xFF)] | tab[kLex4Cls + 768 + (x >> 24)];
    if (!FULL) {
      const uint32_t k0 = 4 * j;  // bytes [max(kend, k0), k0 + 4) of this word are absent
      c[j] |= kend <= k0 ? 0xFFu : kend >= k0 + 4 ? 0u : (0xFFu << (2 * (kend - k0))) & 0xFFu;
    }
  }
  uint32_t m = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t a = (s << 8) | c[j];
    s = tab[a];
    m |= (uint32_t)tab[kLex4Flags + a] << (8 * j);
  }
  return m;
}

// The lexer's matches go to the unit's slots as u32 (start - c0 | end - c0 <<
// 16) records (U_COMPACT, interleaved rows: lex_rec32) through a ring of
// eight records per lane in LDS: the wave's stage buffer, free between the
// tile's chain and the next tile's staging (ring position x of lane l at u32
// 64 x + l: conflict-free), so a push is one LDS write (an eight-register
// queue cost 16 VALU selects per match).  Once per tile one 16-byte store
// writes the row being filled whatever it holds (LexRing::flush), carried in
// four registers across the next staging: no store in the block loop
// depends on the data, so the wait for the next tile's loads counts a fixed
// number of younger stores.  A store whose count depends on the data (one
// per match) made the compiler drain every store before each tile's loads
// could be used (s_waitcnt vmcnt(0)): the kernel ran 0.96 ms with them
// against 0.61 ms without (tools/lex_time.py A/B).  A ninth pending match
// stores its full row early, then waits for its stores.
struct LexRing {
  uint32_t *ring;            // the wave's stage buffer as u32, + lane
  uint32_t c0, c1, c2, c3;   // the row being filled (start | end << 16, units of at most 64 KiB)
  uint32_t n, row;           // records pushed; the row being filled
  __device__ __forceinline__ void restore() {
    const uint32_t h = 256 * (row & 1);
    ring[h] = c0;
    ring[h + 64] = c1;
    ring[h + 128] = c2;
    ring[h + 192] = c3;
  }
  __device__ __forceinline__ void spill(uint32_t *dst, uint32_t rows) {  // the full row, out of turn
    const uint32_t h = 256 * (row & 1);
    *(uint4 *)(dst + 256 * min(row, rows - 1)) = make_uint4(ring[h], ring[h + 64], ring[h + 128], ring[h + 192]);
    ++row;
  }
  __device__ __forceinline__ void push(uint32_t r, uint32_t *dst, uint32_t rows) {
    if (n - 4 * row == 8) {
      spill(dst, rows);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the tile's store count stays fixed
    }
    ring[64 * (n & 7)] = r;
    ++n;
  }
  __device__ __forceinline__ void flush(uint32_t *dst, uint32_t rows) {
    uint32_t h = 256 * (row & 1);
    c0 = ring[h];
    c1 = ring[h + 64];
    c2 = ring[h + 128];
    c3 = ring[h + 192];
    // past the slots: a re-run unit, slots unread
    *(uint4 *)(dst + 256 * min(row, rows - 1)) = make_uint4(c0, c1, c2, c3);
    if (n >= 4 * (row + 1)) {
      ++row;
      h = 256 * (row & 1);
      c0 = ring[h];
      c1 = ring[h + 64];
      c2 = ring[h + 128];
      c3 = ring[h + 192];
    }
  }
};

// The block's matches from its flag word: EMIT at byte j = a match ended at
// bp + j; its start is the last earlier position where the search may have
// begun its match (the state before the byte was the start state — Z of the
// byte before — or a match ended there).  Positions are relative to the unit
// start c0 (fc: the last such position before the block; last: the end of
// the last match).  For a partial block (kend < 16, the walk's last) the
// candidate at bp + kend enters fc harmlessly.
// Over two blocks at once (bytes bp..bp+31, m1: the second block's flags,
// 0 when it was not lexed).
__device__ __forceinline__ void lex_events(uint32_t m0, uint32_t m1, uint32_t bp, uint32_t &cz, uint32_t &fc,
                                            uint32_t &last, uint32_t &n, LexRing &Q, uint32_t *dst, uint32_t cap4) {
  const uint64_t M = ((uint64_t)m1 << 32) | m0;
  uint64_t E = (M >> 1) & 0x5555555555555555ull;
  const uint64_t Z = (M ^ (M >> 1)) & 0x5555555555555555ull;
  const uint64_t A = E | (Z << 2) | cz;
  while (E) {
    const uint32_t j = (uint32_t)__builtin_ctzll(E);
    E &= E - 1;
    const uint64_t below = A & ((1ull << j) - 1ull);
    const uint32_t st = below ? bp + ((63 - (uint32_t)__builtin_clzll(below)) >> 1) : fc;
    const uint32_t x = bp + (j >> 1);
    Q.push(st | (x << 16), dst, cap4);
    ++n;
    last = x;
  }
  if (A) fc = bp + ((63 - (uint32_t)__builtin_clzll(A)) >> 1);
  cz = (uint32_t)(Z >> 62) & 1u;
}

// X4: the four-bytes-per-step table (lex16x4); else one byte per step.
// SINGLE: one haystack (the tile's eight source lines are one base plus
// multiples of 8 chunks: two registers instead of eight 64-bit pointers,
// which keeps X4 within the 128 VGPRs of 4 waves per SIMD).
template <bool X4, bool SINGLE>
__global__ __launch_bounds__(256, 4) void iter_spec_lex_tile_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f,
                                                                 Unit *units, uint64_t *slots, uint32_t *counts) {
  if (gated_off(b)) return;
  // the byte chain's address is one 24-bit multiply-add; 24 rows + the tile
  // stage = 39.5 KB (X4: 5 KB + the stage), 4 blocks (16 waves) per CU
  __shared__ __attribute__((aligned(16))) uint8_t tab[X4 ? kLex4Bytes : kLexBytes];
  __shared__ __attribute__((aligned(16))) uint4 stage[4][64 * 8];
  {
    const uint8_t *img = X4 ? f.lex4_image : f.lex_image;
    const uint32_t nb = X4 ? kLex4Bytes : f.lex_bytes;
    for (uint32_t i = threadIdx.x * 16; i < nb; i += blockDim.x * 16) *(uint4 *)(tab + i) = *(const uint4 *)(img + i);
  }
  __syncthreads();
  const uint64_t C = g.chunk, nk = g.nk;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 *buf = stage[w];
  const int src_h = lane >> 3, src_seg = lane & 7, sw = (lane >> 1) & 7;
  const uint64_t ngroups = (nunits + 63) / 64, nwaves = (uint64_t)gridDim.x * 4;
  const bool single = SINGLE;
  // the last readable 16-byte block of the batch (ragged last units' tiles
  // are clamped to it; their bytes past the haystack are ignored)
  const uint8_t *last_blk = b.hay + (b.count - 1) * b.stride + ((b.length + 15) & ~(uint64_t)15) - 16;
  auto hk = [&](uint64_t uu, uint64_t &h, uint64_t &k) {
    if (single) { h = 0; k = uu; } else { h = uu / nk; k = uu - h * nk; }
  };
  for (uint64_t gi = (uint64_t)blockIdx.x * 4 + w; gi < ngroups; gi += nwaves) {
    const uint64_t u = gi * 64 + lane;
    uint64_t h, k;
    hk(u, h, k);
    const bool valid = u < nunits;
    const uint8_t *src[SINGLE ? 1 : 8];
    if (SINGLE) {
      src[0] = b.hay + b.start + (gi * 64 + src_h) * C + 16 * src_seg;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint64_t us = gi * 64 + 8 * j + src_h, hs, ks;
        hk(us, hs, ks);
        if (us >= nunits) hs = ks = 0;  // absent units re-read unit 0
        src[j] = b.hay + hs * b.stride + b.start + ks * C + 16 * src_seg;
      }
    }
    const uint64_t len = b.length, c0 = b.start + k * C;
    const uint64_t c1 = k + 1 == nk ? g.end : c0 + C;
    // the lexer covers [c0, lim): the byte at c1 - 1 (where the search is cut)
    // and the end of the text are left to the tail pass
    const uint64_t lim = valid ? min(c1 - 1, len) : c0;
    // compact records: four per row (lex_rec32; the queue's row stores
    // write whole rows)
    uint32_t *const dst = (uint32_t *)slots + lex_rec32(g, u, 0);
    const uint32_t cap4 = g.slots;  // rows
    LexRing Q;
    Q.ring = (uint32_t *)buf + lane;
    Q.c0 = Q.c1 = Q.c2 = Q.c3 = 0;
    Q.n = Q.row = 0;
    uint32_t fc = 0, last = 0;  // relative to c0 (lex_events)
    uint32_t n = 0, s = X4 ? f.lex4_s0 : f.lex_s0, cz = 1;
    bool frozen = false;  // a byte >= 0x80 was seen: the rest is the tail pass's
    uint4 n0, n1, n2, n3, n4, n5, n6, n7;
#define RURE_LD(j, a) (*(const uint4 *)min((SINGLE ? src[0] + (j) * 8 * C : src[j]) + (a), last_blk))
#define RURE_LOAD_TILE(a)                                                                                     \
  n0 = RURE_LD(0, a); n1 = RURE_LD(1, a); n2 = RURE_LD(2, a); n3 = RURE_LD(3, a);                            \
  n4 = RURE_LD(4, a); n5 = RURE_LD(5, a); n6 = RURE_LD(6, a); n7 = RURE_LD(7, a);
#define RURE_STAGE(kk, v) buf[(8 * (kk) + src_h) * 8 + (src_seg ^ (((8 * (kk) + src_h) >> 1) & 7))] = (v);
    RURE_LOAD_TILE(0)
    // an empty row store: the loop is entered, as it loops back, with a
    // store younger than the tile loads (the wait for the loads then leaves
    // it in flight, not vmcnt(0))
    *(uint4 *)dst = make_uint4(0, 0, 0, 0);
    for (uint64_t at = 0; at < C; at += 128) {
      RURE_STAGE(0, n0) RURE_STAGE(1, n1) RURE_STAGE(2, n2) RURE_STAGE(3, n3)
      RURE_STAGE(4, n4) RURE_STAGE(5, n5) RURE_STAGE(6, n6) RURE_STAGE(7, n7)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint64_t an = at + 128 < C ? at + 128 : at;
      RURE_LOAD_TILE(an)
      // the tile's 8 blocks through the chain first (flag words kept), then
      // their matches: the event bookkeeping stays off the dependent chain.
      // Active bytes: [c0 + at, lim) up to the first block with a byte >= 0x80.
      const uint64_t t0 = c0 + at;
      const uint64_t rest = lim > t0 ? lim - t0 : 0;
      const uint32_t span = frozen ? 0u : rest < 128 ? (uint32_t)rest : 128u;
      uint32_t mw[8];
      uint32_t act = 0;  // bytes of the tile the lexer took
      if (__builtin_expect(__all(span == 128), 1)) {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const uint4 cur = buf[lane * 8 + (m ^ sw)];
          const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
          const bool hi8 = ((cur.x | cur.y | cur.z | cur.w) & 0x80808080u) != 0;
          frozen = frozen || hi8;
          mw[m] = 0;
          if (!frozen) {
            mw[m] = X4 ? lex16x4<true>(s, wd, tab, 16) : lex16<true>(s, wd, tab, 16);
            act += 16;
          }
        }
      } else {
#pragma unroll 1
        for (int m = 0; m < 8; ++m) {
          const uint4 cur = buf[lane * 8 + (m ^ sw)];
          const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
          const uint32_t kend = span > 16u * m ? min(span - 16u * m, 16u) : 0u;
          uint32_t hi8 = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            hi8 |= wd[q] & (kend >= 4u * q + 4 ? 0xFFFFFFFFu : kend <= 4u * q ? 0u : (1u << (8 * (kend - 4 * q))) - 1u);
          frozen = frozen || (hi8 & 0x80808080u);
          mw[m] = 0;
          if (!frozen && kend) {
            if (X4) mw[m] = kend == 16 ? lex16x4<true>(s, wd, tab, 16) : lex16x4<false>(s, wd, tab, kend);
            else mw[m] = kend == 16 ? lex16<true>(s, wd, tab, 16) : lex16<false>(s, wd, tab, kend);
            act += kend;
          }
        }
      }
      // unrolled: a loop over m indexes mw[] dynamically (a select chain
      // of 7 per block)
      Q.restore();  // the chain has read the stage: the ring may use it
      // two blocks per event loop: the loop runs whenever any lane of the
      // wave has a match in its bytes, i.e. per block nearly always (one
      // match per ~61 bytes per lane); per 32 bytes it runs half as often
      // (0.633 -> 0.619 ms, tools/lex_time.py)
#pragma unroll
      for (int m = 0; m < 8; m += 2)
        if (16u * m < act) lex_events(mw[m], mw[m + 1], (uint32_t)at + 16 * m, cz, fc, last, n, Q, dst, cap4);
      Q.flush(dst, cap4);  // every lane, every tile (slots are padded to whole groups)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#undef RURE_LD
#undef RURE_LOAD_TILE
#undef RURE_STAGE
    if (Q.n > 4 * Q.row) *(uint4 *)(dst + 256 * min(Q.row, cap4 - 1)) = make_uint4(Q.c0, Q.c1, Q.c2, Q.c3);
    if (!valid) continue;
    // (clean flags and counts only matter when the tail pass is skipped,
    // RURE_AMD_LEX_TAIL=0: a diagnostic that leaves the lexer's matches alone)
    Unit U;
    U.entry = {c0, NONE};
    U.exit = n ? IterSt{c0 + last, c0 + last} : IterSt{c0, NONE};
    // spec_exit.p hands the tail pass where its first search may begin
    // scanning: no match is pending before c0 + fc (the last position where
    // the state was the start state or a match ended; on the ASCII text the
    // lexer covered an attempt never dies before it matches, first_byte_rule).
    // Scanning from c0 + last instead re-read the rest of every unit without
    // a late match (the IUB substitutions' tail pass: 0.52 ms per 2.1 GB).
    U.spec_exit = IterSt{max(U.exit.p, c0 + fc), U.exit.lm};
    U.spec_count = n;
    U.flags = U_LEX_TAIL | U_COMPACT | U_SPEC_CLEAN | U_CLEAN;
    U.skip = 0;
    U.pad = n;  // the lexer's records (u16 pairs); the tail pass's go to the back
    units[u] = U;
    counts[u] = n;
  }
}

// The lexer pass's tail: per unit, the generic cut-bounded iteration from the
// state the lexer left at c1 - 1 (or from c0 for U_LEX_REDO units), appending
// to the unit's slots; writes the final speculative record.
__global__ __launch_bounds__(256) void iter_lex_tail_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f,
                                                            RevDfaDev r, Unit *units, uint64_t *slots,
                                                            uint32_t *counts, uint32_t *dirty) {
  if (gated_off(b)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint8_t *rlds = stage_tables(f, r, lds);
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, len, c0, c1;
    const uint8_t *base;
    unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
    Unit U = units[u];
    uint32_t n = U.spec_count;
    UnitIter it;
    it.init(U.exit, c1);
    it.from = U.spec_exit.p;  // the lexer's scan-from hint (iter_spec_lex_tile_kernel)
    uint64_t ms, me;
    const bool compact = (U.flags & U_COMPACT) != 0;
    while (it.next(f, r, lds, rlds, base, len, &ms, &me)) {
      if (n < g.slots) {
        // compact units: absolute records from the back rows (slot_rec)
        const uint64_t k = compact ? lex_row16(g, u, g.slots - 1 - (n - U.pad)) : u * g.slots + n;
        ((ulonglong2 *)slots)[k] = make_ulonglong2(ms, me);
      }
      ++n;
    }
    U.exit = it.exit;
    U.spec_exit = it.exit;
    U.spec_count = n;
    U.flags = (it.clean ? (U_SPEC_CLEAN | U_CLEAN) : 0) | (it.quit ? U_QUIT : 0) | (U.flags & U_COMPACT);
    units[u] = U;
    counts[u] = n;
    if (!(U.flags & U_SPEC_CLEAN)) atomicOr(dirty, 1u);  // the fix pass has work
  }
}

// Where the true iteration of unit j, entered with E, joins the speculative
// one S (started fresh at c0), read off S's recorded matches: S's state
// before it yielded match i is (p_i, lm_i) (p_0 = c0, lm_0 = none; then the
// end of match i-1, plus one after an empty match).  For the last i with
// p_i <= E.p: if E.p > p_i (or the states are equal), no match starts in
// [E.p, s_i) except what S saw, so the search from E.p yields S's match i
// unless it is an empty match at E's last match end (skipped); with E.p ==
// p_i the two searches are the same one.  Returns i
// (i == spec_count: no owned match at all), or -1 = undecided.
__device__ int64_t join_speculation(const Unit &U, uint64_t c0, IterSt E, const uint64_t *slots, const Geo &g,
                                    uint64_t j) {
  const uint32_t n = U.spec_count;
  if (n > g.slots || E.p < c0) return -1;
  const bool cp = (U.flags & U_COMPACT) != 0;
  auto rec = [&](uint32_t i) { return slot_rec(slots, g, j, i, cp, c0, U.pad); };
  uint32_t lo = 0, hi = n;  // last i in [0, n] with p_i <= E.p (p_i strictly increasing)
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    const ulonglong2 r = rec(mid - 1);
    const uint64_t s = r.x, e = r.y;
    if ((s == e ? e + 1 : e) <= E.p) lo = mid;
    else hi = mid - 1;
  }
  const uint32_t i = lo;
  uint64_t pi = c0, lmi = NONE;
  if (i > 0) {
    const ulonglong2 r = rec(i - 1);
    const uint64_t s = r.x, e = r.y;
    pi = s == e ? e + 1 : e;
    lmi = e;
  }
  if (E.p == pi && E.lm != lmi) {
    // same search start, different last match: S's search from p_i yielded
    // its match i directly (no empty match skipped) when S had no last match
    // (i == 0) or match i starts at p_i
    if (!(i == 0 || (i < n && rec(i).x == pi))) return -1;
  }
  if (i < n) {
    const ulonglong2 r = rec(i);
    const uint64_t s = r.x, e = r.y;
    if (s < E.p || (s == e && e == E.lm)) return -1;
    return i;
  }
  return (U.flags & U_SPEC_CLEAN) ? (int64_t)i : -1;
}

// Repairs unit j given its true entry `E`.  Usually decided from the
// speculative slots (join_speculation); otherwise the true and the
// speculative iterations run in lockstep until both emit the same match.
// Updates the unit's record and count; returns true if its exit changed.
__device__ bool repair_unit(const BatchDev &b, const Geo &g, const FwdDfaDev &f, const RevDfaDev &r,
                            const uint8_t *lds, const uint8_t *rlds, uint64_t j, IterSt E, Unit *units,
                            uint32_t *counts, const uint64_t *slots, const WaveCtx *wc = nullptr) {
  uint64_t h, len, c0, c1;
  const uint8_t *base;
  unit_bounds(b, g, j, &h, &base, &len, &c0, &c1);
  Unit U = units[j];
  const bool spec_clean = (U.flags & U_SPEC_CLEAN) != 0;
  // the next unit's speculation is unsure: exits compare as states
  const bool strict = f.looks && (j + 1) % g.nk != 0 && (units[j + 1].flags & U_UNSURE);
  U.entry = E;
  U.flags = (U.flags & ~(U_COPY | U_CLEAN)) | U_FIXED;
  U.skip = 0;
  bool changed;
  if (E.p >= c1) {  // the true iteration passes over the whole unit
    const bool cl = E.p == c1 && (E.lm != c1 || f.nonempty);
    counts[j] = 0;
    changed = !exit_equiv(cl, E, spec_clean, U.spec_exit, strict);
    U.exit = E;
    U.flags |= cl ? U_CLEAN : 0;
    units[j] = U;
    return changed;
  }
  const int64_t i = f.looks ? -1 : join_speculation(U, c0, E, slots, g, j);
  if (i >= 0) {
    if (i < (int64_t)U.spec_count) {
      counts[j] = U.spec_count - (uint32_t)i;
      U.skip = (uint32_t)i;
      U.flags |= U_COPY | (spec_clean ? U_CLEAN : 0);
      U.exit = U.spec_exit;
      changed = false;
    } else {
      counts[j] = 0;
      U.exit = E;
      U.flags |= U_CLEAN;
      changed = !spec_clean;
    }
    units[j] = U;
    return changed;
  }
  UnitIter F, S;
  F.init(E, c1);
  S.init({c0, NONE}, c1);
  uint64_t fs, fe, ss, se;
  bool fm = F.next(f, r, lds, rlds, base, len, &fs, &fe, wc);
  bool sm = S.next(f, r, lds, rlds, base, len, &ss, &se, wc);
  uint32_t fcnt = 0, scnt = 0;
  bool synced = false;
  while (fm) {
    if (sm && fs == ss && fe == se) { synced = true; break; }
    if (!sm || fs < ss || (fs == ss && fe < se)) {
      ++fcnt;
      fm = F.next(f, r, lds, rlds, base, len, &fs, &fe, wc);
    } else {
      ++scnt;
      sm = S.next(f, r, lds, rlds, base, len, &ss, &se, wc);
    }
  }
  if (synced) {
    counts[j] = fcnt + (U.spec_count - scnt);
    U.exit = U.spec_exit;
    U.flags |= spec_clean ? U_CLEAN : 0;
    if (fcnt == 0 && U.spec_count <= g.slots) {
      U.skip = scnt;
      U.flags |= U_COPY;
    }
    changed = false;
  } else {
    counts[j] = fcnt;
    changed = !exit_equiv(F.clean, F.exit, spec_clean, U.spec_exit, strict);
    U.exit = F.exit;
    U.flags |= (F.clean ? U_CLEAN : 0);
  }
  // (U_QUIT: a search quit -- or, served by the wave, ran on the Pike VM:
  // the unit stays the wave kernels' to re-run)
  U.flags |= (F.quit || S.quit || F.waved || S.waved) ? U_QUIT : 0;
  units[j] = U;
  return changed;
}

// Pass 2: units entered through a dirty speculative exit are repaired in
// parallel; repairs that change their own exit are queued for the walker.
// Dirty exits are rare, so a block stages the hot tables into LDS only when
// one of its units needs a repair.
__device__ __forceinline__ void fix_body(const BatchDev &b, const Geo &g, uint64_t nunits, const FwdDfaDev &f,
                                         const RevDfaDev &r, Unit *units, uint32_t *counts, const uint64_t *slots,
                                         uint64_t *queue, unsigned long long *qlen, const uint32_t *dirty,
                                         uint8_t *lds) {
  if (*dirty == 0) return;  // every speculative exit was clean
  const uint8_t *rlds = nullptr;
  bool staged = false;
  for (uint64_t u0 = (uint64_t)blockIdx.x * blockDim.x; u0 + 1 < nunits; u0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = u0 + threadIdx.x;
    const bool need = u + 1 < nunits && (u + 1) % g.nk != 0 &&
                      (!(units[u].flags & U_SPEC_CLEAN) || (units[u + 1].flags & U_UNSURE));
    if (!__syncthreads_or(need)) continue;
    if (!staged) {
      rlds = stage_tables(f, r, lds);
      staged = true;
    }
    // (a unit with U_QUIT is the wave pass's, iter_wfix_kernel: also one
    // whose lane repair quits here)
    const bool lane_ok = need && !(units[u + 1].flags & U_QUIT);
    if (lane_ok && repair_unit(b, g, f, r, lds, rlds, u + 1, units[u].spec_exit, units, counts, slots) &&
        !(units[u + 1].flags & U_QUIT)) {
      const unsigned long long q = atomicAdd(qlen, 1ull);
      queue[q] = u + 1;
    }
  }
}

__global__ __launch_bounds__(1024) void iter_fix_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r,
                                                       Unit *units, uint32_t *counts, const uint64_t *slots,
                                                       uint64_t *queue, unsigned long long *qlen,
                                                       const uint32_t *dirty) {
  if (gated_off(b)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  fix_body(b, g, nunits, f, r, units, counts, slots, queue, qlen, dirty, lds);
}

// Pass 3 (one thread): propagate exits that changed, in unit order.
// wc: the whole wave runs it (wave-uniform; every lane stores the same
// values) and a search whose DFA quits runs on the Pike VM.
__device__ __forceinline__ void walk_body(const BatchDev &b, const Geo &g, uint64_t nunits, const FwdDfaDev &f,
                                          const RevDfaDev &r, Unit *units, uint32_t *counts, const uint64_t *slots,
                                          uint64_t *queue, unsigned long long *qlen, const WaveCtx *wc = nullptr) {
  const uint64_t n = *qlen;
  if (n == 0) return;
  if (threadIdx.x == 0) {
    for (uint64_t i = 1; i < n; ++i) {  // insertion sort (the queue is short)
      uint64_t v = queue[i], k = i;
      while (k > 0 && queue[k - 1] > v) { queue[k] = queue[k - 1]; --k; }
      queue[k] = v;
    }
  }
  if (wc) __syncthreads();
  uint64_t walked = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t j = queue[i];
    if (j + 1 <= walked) continue;
    uint64_t u = j + 1;
    Unit X = units[j];
    while (u < nunits && u % g.nk != 0) {
      const Unit V = units[u];
      // entry the parallel passes assumed for unit u
      const Unit P = units[u - 1];
      const bool assumed_clean = (P.flags & U_SPEC_CLEAN) != 0;
      const bool unsure = (V.flags & U_UNSURE) != 0;
      if (exit_equiv((X.flags & U_CLEAN) != 0, X.exit, assumed_clean, P.spec_exit, unsure)) break;
      Unit W = V;
      if ((X.flags & U_CLEAN) && !unsure) {  // back to the speculative entry
        uint64_t h, len, c0, c1;
        const uint8_t *base;
        unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
        W.entry = {c0, NONE};
        W.exit = W.spec_exit;
        W.flags = (W.flags & ~(U_FIXED | U_CLEAN | U_COPY)) | ((W.flags & U_SPEC_CLEAN) ? U_CLEAN : 0);
        W.skip = 0;
        units[u] = W;
        counts[u] = W.spec_count;
      } else {
        repair_unit(b, g, f, r, f.lds_image /* unused: hot = 0 */, nullptr, u, X.exit, units, counts, slots, wc);
      }
      if (wc) __syncthreads();
      X = units[u];
      ++u;
    }
    walked = u;
  }
}

// Whether a search of the chunked iteration quit (U_QUIT is sticky).
__global__ void iter_quit_kernel(const Unit *units, uint64_t nunits, uint32_t *quit) {
  bool any = false;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x)
    any |= (units[u].flags & U_QUIT) != 0;
  if (any) atomicOr(quit, 1u);
}

__global__ void iter_walk_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r, Unit *units,
                                 uint32_t *counts, const uint64_t *slots, uint64_t *queue, unsigned long long *qlen) {
  if (gated_off(b)) return;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  walk_body(b, g, nunits, f, r, units, counts, slots, queue, qlen);
}

// ------------------------------------- the wave-served chunked iteration
// A regex whose DFA can quit (a Unicode \b over non-ASCII bytes,
// dfa.rs:1491-1496) keeps the chunked iteration: the lane passes above run
// as usual, and a unit where a search quit (U_QUIT) is taken over by one
// wave, which runs that search -- and any later one whose DFA quits -- on
// the Pike VM (exec.rs:485-487: the reference's NFA fallback for that
// search), bounded by the unit's cut like the DFA's.  U_QUIT then marks the
// unit as the wave kernels': its speculation (iter_wspec_kernel), its repair
// (iter_wfix_kernel), the walker (iter_wwalk_kernel, wave-uniform) and its
// re-emission (iter_wemit_kernel).  Tables: global (the LDS holds the Pike
// VM's lists, pike::Lists, nfa_wave_bytes per wave): f.hot = r.hot = 0, and
// an all-rows table is read from its global image (as the walker does).

// Rounds of (a wave answers each pending unit's quitting search, the lanes
// resume) before the waves finish the rest of the pending units themselves.
constexpr int kWaveRounds = 3;

// Where a wave keeps the Pike VM's working set (iter_post picks):
//  kWaveLds    one wave per block, stamps and thread lists in the LDS;
//  kWaveSplit  one wave per block, the stamps -- read and written at random
//              by append_closure -- in the LDS, the thread lists (written and
//              read in order) in the wave's scratch;
//  kWaveTables several waves per block sharing the NFA's tables (leaves,
//              closure offsets and entries, the Unicode word ranges) staged
//              in the LDS, each with its stamps there and its lists in
//              scratch: every step of the Pike VM reads those tables.
enum : uint32_t { kWaveLds = 0, kWaveSplit = 1, kWaveScratch = 2, kWaveTables = 3 };

__host__ __device__ inline size_t wave_table_bytes(const NfaDev &nf) {
  return (((size_t)nf.nentries * 8 + (size_t)nf.nleaves * 12 + (size_t)nf.ncl_off * 4 + (size_t)nf.perlw_n * 8) + 255) &
         ~(size_t)255;
}
__host__ __device__ inline size_t wave_stamp_bytes(const NfaDev &nf) { return ((size_t)nf.nleaves * 4 + 255) & ~(size_t)255; }

struct WaveSetup {
  NfaDev nf;  // kWaveTables: its table pointers into the LDS
  pike::Lists W;
  uint64_t wave, nwaves;
};

__device__ __forceinline__ void wave_setup(const NfaDev &nf0, uint8_t *lds_mem, uint8_t *scratch, uint32_t mode,
                                           WaveSetup &S) {
  const uint32_t wpb = blockDim.x >> 6, wib = threadIdx.x >> 6;
  S.wave = (uint64_t)blockIdx.x * wpb + wib;
  S.nwaves = (uint64_t)gridDim.x * wpb;
  S.nf = nf0;
  const uint32_t N = nf0.nleaves;
  uint8_t *stamps = lds_mem;
  if (mode == kWaveTables) {
    uint32_t *d = (uint32_t *)lds_mem;
    auto stage = [&](const void *src, uint32_t words) {
      const uint32_t *q = (const uint32_t *)src;
      for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) d[i] = q[i];
      uint32_t *at = d;
      d += words;
      return (const void *)at;
    };
    S.nf.entries = (const uint2 *)stage(nf0.entries, 2 * nf0.nentries);
    S.nf.leaves = (const uint32_t *)stage(nf0.leaves, 3 * N);
    S.nf.cl_off = (const uint32_t *)stage(nf0.cl_off, nf0.ncl_off);
    S.nf.perlw = (const uint32_t *)stage(nf0.perlw, 2 * nf0.perlw_n);
    __syncthreads();
    stamps = lds_mem + wave_table_bytes(nf0) + (size_t)wib * wave_stamp_bytes(nf0);
  }
  uint8_t *mem = scratch ? scratch + (size_t)S.wave * nfa_wave_bytes(N) : lds_mem;
  S.W.st[0] = (uint64_t *)mem;
  S.W.st[1] = S.W.st[0] + N;
  S.W.stamp = mode == kWaveLds || mode == kWaveScratch ? (uint32_t *)(S.W.st[1] + N) : (uint32_t *)stamps;
  S.W.leaf[0] = (uint32_t *)(S.W.st[1] + N) + N;
  S.W.leaf[1] = S.W.leaf[0] + N;
  for (uint32_t i = pike::lane_id(); i < N; i += 64) S.W.stamp[i] = 0xFFFFFFFFu;
  pike::wave_sync();
}

// The speculation of every U_PEND unit, resumed at the search that quit
// (the lane pass left the state before it as the unit's exit, its matches so
// far in the slots, U.pad = that search was the unit's first).  STEP: only
// that search, then the unit goes back to the lanes (U_RESUME) unless it
// ended; else the rest of the unit on the wave.
template <bool STEP>
__global__ __launch_bounds__(512) void iter_wspec_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f,
                                                        RevDfaDev r, NfaDev nf, Unit *units, uint64_t *slots,
                                                        uint32_t *counts, uint32_t *dirty, uint8_t *scratch, uint32_t wmode) {  // wmode: kWave*
  if (gated_off(b) || !(__atomic_load_n(dirty, __ATOMIC_RELAXED) & 2u)) return;  // nothing pending
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_mem[];
  WaveSetup S;
  wave_setup(nf, lds_mem, scratch, wmode, S);
  pike::TagGen tg;
  const WaveCtx wc{&S.nf, &S.W, &tg};
  const uint32_t lane = pike::lane_id();
  for (uint64_t u = S.wave; u < nunits; u += S.nwaves) {
    const Unit U = units[u];
    if (!(U.flags & U_PEND)) continue;
    uint64_t h, len, c0, c1;
    const uint8_t *base;
    unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
    UnitIter it;
    it.init(U.exit, c1);
    it.first = U.pad != 0;
    uint32_t n = U.spec_count;
    uint64_t s, e;
    bool more = true;
    while ((more = it.next(f, r, f.lds_image, nullptr, base, len, &s, &e, &wc))) {
      if (n < g.slots && lane == 0) {
        slots[(u * g.slots + n) * 2] = s;
        slots[(u * g.slots + n) * 2 + 1] = e;
      }
      ++n;
      if (STEP) break;  // the search that quit is answered: the lanes go on
    }
    if (STEP && more) {
      Unit V = U;
      V.exit = it.st;
      V.spec_count = n;
      V.pad = 0;
      V.flags = (U.flags & ~(U_PEND | U_UNSURE)) | U_RESUME | U_QUIT |
                ((U.pad != 0 ? f.looks && it.unsure : (U.flags & U_UNSURE) != 0) ? U_UNSURE : 0);
      if (lane == 0) units[u] = V;
      continue;
    }
    const bool pre = f.can_quit == 2 && c0 > 0 && base[c0 - 1] >= 0x80;  // (as iter_spec_burst_kernel)
    const bool unsure = (U.pad != 0 ? f.looks && it.unsure : (U.flags & U_UNSURE) != 0) || pre;
    Unit V;
    V.entry = {c0, NONE};
    V.exit = it.exit;
    V.spec_exit = it.exit;
    V.spec_count = n;
    V.flags = (it.clean ? (U_SPEC_CLEAN | U_CLEAN) : 0) | U_QUIT | (unsure && u % g.nk != 0 ? U_UNSURE : 0);
    V.skip = V.pad = 0;
    if (lane == 0) {
      units[u] = V;
      counts[u] = n;
      if ((V.flags & (U_SPEC_CLEAN | U_UNSURE)) != U_SPEC_CLEAN) atomicOr(dirty, 1u);
    }
  }
}

// fix_body's repairs of the units the lane pass left (U_QUIT: a quit in the
// speculation or in the lane repair); a changed exit is queued for the walker.
__global__ __launch_bounds__(512) void iter_wfix_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r,
                                                       NfaDev nf, Unit *units, uint32_t *counts, const uint64_t *slots,
                                                       uint64_t *queue, unsigned long long *qlen, const uint32_t *dirty,
                                                       uint8_t *scratch, uint32_t wmode) {  // wmode: kWave*
  if (gated_off(b) || *dirty == 0) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_mem[];
  WaveSetup S;
  wave_setup(nf, lds_mem, scratch, wmode, S);
  pike::TagGen tg;
  const WaveCtx wc{&S.nf, &S.W, &tg};
  for (uint64_t u = S.wave; u + 1 < nunits; u += S.nwaves) {
    const uint32_t fn = units[u + 1].flags;
    const bool need = (u + 1) % g.nk != 0 && (fn & U_QUIT) &&
                      (!(units[u].flags & U_SPEC_CLEAN) || (fn & U_UNSURE));
    if (!need) continue;
    const bool ch = repair_unit(b, g, f, r, f.lds_image, nullptr, u + 1, units[u].spec_exit, units, counts, slots, &wc);
    if (ch && pike::lane_id() == 0) {
      const unsigned long long q = atomicAdd(qlen, 1ull);
      queue[q] = u + 1;
    }
  }
}

// The walker with the whole wave (one block of 64).
__global__ __launch_bounds__(64) void iter_wwalk_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r,
                                                        NfaDev nf, Unit *units, uint32_t *counts, const uint64_t *slots,
                                                        uint64_t *queue, unsigned long long *qlen, uint8_t *scratch, uint32_t wmode) {  // wmode: kWave*
  if (gated_off(b) || blockIdx.x != 0) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_mem[];
  WaveSetup S;
  wave_setup(nf, lds_mem, scratch, wmode, S);
  pike::TagGen tg;
  const WaveCtx wc{&S.nf, &S.W, &tg};
  walk_body(b, g, nunits, f, r, units, counts, slots, queue, qlen, &wc);
}

// emit_body's re-runs of U_QUIT units (from the unit's entry, cnt matches).
__global__ __launch_bounds__(512) void iter_wemit_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r,
                                                        NfaDev nf, const Unit *units, const uint64_t *off,
                                                        uint64_t *out, uint64_t cap, uint8_t *scratch, uint32_t wmode) {  // wmode: kWave*
  if (gated_off(b)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_mem[];
  WaveSetup S;
  wave_setup(nf, lds_mem, scratch, wmode, S);
  pike::TagGen tg;
  const WaveCtx wc{&S.nf, &S.W, &tg};
  const uint64_t obase = off[0];
  for (uint64_t u = S.wave; u < nunits; u += S.nwaves) {
    const uint32_t fl = units[u].flags;
    if (!(fl & U_QUIT)) continue;
    const uint64_t o0 = off[u] - obase, cnt = off[u + 1] - off[u];
    if (!cnt || o0 >= cap || !(((fl & U_FIXED) && !(fl & U_COPY)) || cnt > g.slots)) continue;
    uint64_t h, len, c0, c1;
    const uint8_t *base;
    unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
    UnitIter it;
    it.init(units[u].entry, c1);
    uint64_t s, e, i = 0;
    while (i < cnt && it.next(f, r, f.lds_image, nullptr, base, len, &s, &e, &wc)) {
      if (o0 + i < cap && pike::lane_id() == 0) {
        out[2 * (o0 + i)] = s;
        out[2 * (o0 + i) + 1] = e;
      }
      ++i;
    }
  }
}

// Span entry (sharded / streamed find_iter): the first unit is entered with
// the iteration state the previous span left.  Runs after the speculative
// pass and before the parallel repairs, which read only the speculative
// fields of unit 0; a changed exit is queued for the walker.
__global__ void iter_entry_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r, Unit *units,
                                  uint32_t *counts, const uint64_t *slots, const uint64_t *entry, uint64_t *queue,
                                  unsigned long long *qlen) {
  if (gated_off(b)) return;
  if (threadIdx.x != 0 || blockIdx.x != 0 || entry[2]) return;
  if (repair_unit(b, g, f, r, f.lds_image /* unused: hot = 0 */, nullptr, 0, IterSt{entry[0], entry[1]}, units,
                  counts, slots) &&
      g.nk > 1) {
    const unsigned long long q = atomicAdd(qlen, 1ull);
    queue[q] = 0;
  }
}

// The state the iteration leaves at the span end: (next, last_match, fresh).
// A span that runs to the end of the text (`tail` = its length) iterated
// without a cut; "fresh" then means equivalent to a fresh start at the text
// end, where only an empty match at the end could differ.
__device__ __forceinline__ void exit_body(const Unit *units, uint64_t nunits, uint64_t *exit, uint64_t tail,
                                          uint32_t nonempty) {
  const Unit U = units[nunits - 1];
  bool fresh = (U.flags & U_CLEAN) != 0;
  if (tail != ~0ull && U.exit.p >= tail) fresh = U.exit.p == tail && (U.exit.lm != tail || nonempty);
  exit[0] = U.exit.p;
  exit[1] = U.exit.lm;
  exit[2] = fresh ? 1 : 0;
}
__global__ void iter_exit_kernel(const Unit *units, uint64_t nunits, uint64_t *exit, uint64_t tail,
                                 uint32_t nonempty) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  exit_body(units, nunits, exit, tail, nonempty);
}

// Pass 4: write every unit's matches at its offset.  Units whose speculation
// held copy their slot buffer: each lane its own unit's when it holds at most
// 4 records, else the wave's larger units eight at a time.  Units that were repaired, or had more matches
// than slots, re-run their iteration (the block stages the hot tables only
// then).
// LEX: compact (lexer) units may occur (iter_emit_kernel; the multi-regex
// passes never produce them, and the extra paths cost their kernel spills)
template <bool LEX>
__device__ __forceinline__ void emit_body(const BatchDev &b, const Geo &g, uint64_t nunits, const FwdDfaDev &f,
                                          const RevDfaDev &r, const Unit *units, const uint64_t *slots,
                                          const uint64_t *off, uint64_t *out, uint64_t cap, uint8_t *lds,
                                          bool copies = true) {
  const uint8_t *rlds = nullptr;
  bool staged = false;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t obase = off[0];  // off may be a segment of several regexes' shared scan
  for (uint64_t u0 = (uint64_t)blockIdx.x * blockDim.x; u0 < nunits; u0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = u0 + threadIdx.x;
    uint64_t o0 = 0, cnt = 0, cbase = 0;
    uint32_t skip = 0, nlex = 0;
    bool rerun = false, copy = false, compact = false;
    if (u < nunits) {
      o0 = off[u] - obase;
      cnt = off[u + 1] - off[u];
      if (cnt && o0 < cap) {
        const uint32_t fl = units[u].flags;
        rerun = ((fl & U_FIXED) && !(fl & U_COPY)) || cnt > g.slots;
        copy = !rerun && copies;  // copies = false: iter_copy_group_kernel wrote them
        if (fl & U_QUIT) rerun = false;  // the wave's (iter_wemit_kernel)
        skip = (fl & U_COPY) ? units[u].skip : 0;  // loaded by every lane at once, not per copied unit
        compact = LEX && (fl & U_COMPACT) != 0;
        if (compact) {
          uint64_t hh, ll, c1;
          const uint8_t *bb;
          unit_bounds(b, g, u, &hh, &bb, &ll, &cbase, &c1);
          nlex = units[u].pad;
        }
      }
    }
    // A unit with at most 4 records (almost every unit: the copy loop below
    // is a chain of dependent load -> store rounds, one unit per round) copies
    // its own records, every lane at once; larger ones go one at a time with
    // the whole wave.
    const bool own = copy && cnt <= 4;
    if (own) {
      const uint32_t nw = 2 * (uint32_t)min(cnt, cap - o0);
      uint64_t *dst = out + 2 * o0;
      uint64_t v[8];
      if (compact) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
          if (2 * k < nw) {
            const ulonglong2 r = slot_rec(slots, g, u, skip + k, true, cbase, nlex);
            v[2 * k] = r.x;
            v[2 * k + 1] = r.y;
          }
      } else {
        const uint64_t *src = slots + (u * g.slots + skip) * 2;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) v[k] = k < nw ? src[k] : 0;
      }
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k)
        if (k < nw) dst[k] = v[k];
    }
    // The wave's larger units eight at a time: lane l serves records
    // l & 7, + 8, ... of unit 8 grp + (l >> 3), so each load instruction
    // reads 8 units x 128 contiguous bytes (whole lines) and four rounds of
    // loads are in flight before their stores.
    const uint64_t wrec = (copy && !own) ? min(cnt, cap - o0) : 0;
    const uint64_t wsrc = (u * g.slots + skip) * 2, wdst = 2 * o0;
    // compact units: the record base (c0) rides along (~0 marks u64 records),
    // the lexer's records are u32 from the unit's slot start, the tail's u64
    // from its end
    // (lex_rec32 / lex_row16 rows: the unit's u32 base and its last row)
    const uint64_t wcb = compact ? cbase : ~0ull, wsrc32 = (u >> 6) * 256 * (uint64_t)g.slots + (u & 63) * 4;
    const uint64_t wlex = compact ? (nlex > skip ? nlex - skip : 0) : 0;
    const uint64_t wend = compact ? 2 * lex_row16(g, u, g.slots - 1) : 0;  // u64 index of the unit's last row
    const uint64_t wtail0 = compact && skip > nlex ? skip - nlex : 0;
    const uint64_t wskip = skip;
    const uint64_t busy = __ballot(wrec != 0);
    const bool a16 = ((uintptr_t)out & 15) == 0;
#pragma unroll 1
    for (int grp = 0; grp < 8; ++grp) {
      if (!((busy >> (8 * grp)) & 0xFFull)) continue;
      const int ul = 8 * grp + (int)(lane >> 3);
      const uint64_t cu = __shfl(wrec, ul), su = __shfl(wsrc, ul), du = __shfl(wdst, ul);
      const uint64_t cb = __shfl(wcb, ul), su32 = __shfl(wsrc32, ul);
      const uint64_t nl = __shfl(wlex, ul), se = __shfl(wend, ul), t0 = __shfl(wtail0, ul);
      const uint64_t sk = __shfl(wskip, ul);
      uint64_t mx = cu;
      mx = max(mx, (uint64_t)__shfl_xor(mx, 8));
      mx = max(mx, (uint64_t)__shfl_xor(mx, 16));
      mx = max(mx, (uint64_t)__shfl_xor(mx, 32));
      const ulonglong2 *src = (const ulonglong2 *)(slots + su);
      const uint32_t *src32 = (const uint32_t *)slots + su32;
      uint64_t *dst = out + du;
      for (uint64_t i = lane & 7; i < mx; i += 32) {
        ulonglong2 v[4];
        if (LEX && cb != ~0ull) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const uint64_t j = i + 8 * t;
            if (j < cu) {
              if (j < nl) {
                const uint64_t ii = sk + j;
                const uint32_t r = src32[(ii >> 2) * 256 + (ii & 3)];
                v[t] = make_ulonglong2(cb + (r & 0xFFFFu), cb + (r >> 16));
              } else {  // the tail pass's records, backwards from the last row
                v[t] = *(const ulonglong2 *)(slots + se - 128 * (t0 + j - nl));
              }
            }
          }
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (i + 8 * t < cu) v[t] = src[i + 8 * t];
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint64_t j = i + 8 * t;
          if (j < cu) {
            if (a16) {
              *(ulonglong2 *)(dst + 2 * j) = v[t];
            } else {
              dst[2 * j] = v[t].x;
              dst[2 * j + 1] = v[t].y;
            }
          }
        }
      }
    }
    if (!__syncthreads_or(rerun)) continue;
    if (!staged) {
      rlds = stage_tables(f, r, lds);
      staged = true;
    }
    if (!rerun) continue;
    const Unit U = units[u];
    uint64_t h, len, c0, c1;
    const uint8_t *base;
    unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
    UnitIter it;
    it.init(U.entry, c1);
    uint64_t s, e, i = 0;
    while (i < cnt && it.next(f, r, lds, rlds, base, len, &s, &e)) {
      if (o0 + i < cap) {
        out[2 * (o0 + i)] = s;
        out[2 * (o0 + i) + 1] = e;
      }
      ++i;
    }
  }
}

__global__ __launch_bounds__(1024) void iter_emit_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r,
                                                        const Unit *units, const uint64_t *slots, const uint64_t *off,
                                                        uint64_t *out, uint64_t cap, int copies) {
  if (gated_off(b)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  emit_body<true>(b, g, nunits, f, r, units, slots, off, out, cap, lds, copies != 0);
}

// The copies of a lexer pass by lexer group (U_COMPACT interleaved rows,
// lex_rec32): one block per group of 64 units, whose output records are one
// contiguous range.  Per window of kGrpWin output records the four waves
// read the rows overlapping it (each row one coalesced 1 KiB load, four
// records per unit) and scatter the records into LDS at their output
// places, tagged with their unit; then the block writes the window out
// front to back, 1 KiB per wave store.  Both HBM streams stay whole-line.
// (A row-by-row copy straight from registers wrote 64 units' scattered
// 64-byte pieces per store: 0.26 ms for the strip's 35 M records; an
// output-ordered copy gathering 4-byte records: 0.20 ms.)  The tail pass's
// few absolute records are written directly; positions of units that are
// re-run stay untagged, for iter_emit_kernel.
constexpr uint32_t kGrpWin = 4096;
__global__ __launch_bounds__(256) void iter_copy_group_kernel(BatchDev b, Geo g, uint64_t nunits, const Unit *units,
                                                              const uint64_t *slots, const uint64_t *off,
                                                              uint64_t *out, uint64_t cap) {
  if (gated_off(b)) return;
  __shared__ uint32_t wrec[kGrpWin];
  __shared__ uint8_t wtag[kGrpWin];  // unit in the group, 0xFF: nothing to write here
  __shared__ uint64_t sbase[64];
  const uint64_t obase = off[0];
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint64_t ngroups = (nunits + 63) / 64;
  const uint4 *rows = (const uint4 *)slots;
  for (uint64_t G = blockIdx.x; G < ngroups; G += gridDim.x) {
    const uint64_t u = G * 64 + lane;
    uint32_t skip = 0, nl = 0, i1 = 0;  // records [skip, i1) go to out[o0 + i - skip]
    uint64_t o0 = 0, c0 = 0;
    if (u < nunits) {
      const uint64_t a = off[u] - obase, cnt = off[u + 1] - off[u];
      const uint4 tl = ((const uint4 *)(units + u))[3];  // spec_count, flags, skip, pad
      const bool rerun = ((tl.y & U_FIXED) && !(tl.y & U_COPY)) || cnt > g.slots;
      if (cnt && a < cap && !rerun) {
        o0 = a;
        skip = (tl.y & U_COPY) ? tl.z : 0;
        nl = tl.w;
        i1 = skip + (uint32_t)min(cnt, cap - a);
        uint64_t hh, ll, c1;
        const uint8_t *bb;
        unit_bounds(b, g, u, &hh, &bb, &ll, &c0, &c1);
      }
    }
    if (wv == 0) {
      sbase[lane] = c0;
      for (uint32_t i = max(skip, nl); i < i1; ++i)  // the tail pass's records
        ((ulonglong2 *)out)[o0 + i - skip] = ((const ulonglong2 *)slots)[lex_row16(g, u, g.slots - 1 - (i - nl))];
    }
    const uint32_t le = min(i1, nl);  // the lexer's records: [skip, le)
    const uint64_t O0 = off[G * 64] - obase, O1 = min(off[min(G * 64 + 64, nunits)] - obase, cap);
    const uint64_t rbase = G * 64 * (uint64_t)g.slots + lane;  // lex_row16(g, u, 0)
    for (uint64_t w0 = O0; w0 < O1; w0 += kGrpWin) {
      const uint64_t w1 = min(O1, w0 + kGrpWin);
      for (uint32_t i = t; i < kGrpWin / 4; i += 256) ((uint32_t *)wtag)[i] = 0xFFFFFFFFu;
      // this unit's records in the window: i in [ia, ib)
      uint32_t ia = skip, ib = skip;
      if (le > skip && o0 < w1 && o0 + (le - skip) > w0) {
        ia = o0 >= w0 ? skip : skip + (uint32_t)(w0 - o0);
        ib = min(le, skip + (uint32_t)(w1 - o0));
      }
      uint32_t k0 = ib > ia ? ia / 4 : 0xFFFFFFFFu, k1 = ib > ia ? (ib + 3) / 4 : 0;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        k0 = min(k0, (uint32_t)__shfl_xor((int)k0, d));
        k1 = max(k1, (uint32_t)__shfl_xor((int)k1, d));
      }
      __syncthreads();
      // eight rows per wave in flight (a loop of one load and its scatter
      // waited out a load latency per row)
      for (uint32_t k = k0 + wv; k < k1; k += 32) {
        uint4 v[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j)
          if (k + 4 * j < k1) v[j] = rows[rbase + (uint64_t)(k + 4 * j) * 64];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
          const uint32_t kk = k + 4 * j;
          const uint32_t x[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
          for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t i = 4 * kk + q;
            if (kk < k1 && i >= ia && i < ib) {
              const uint32_t pp = (uint32_t)(o0 + (i - skip) - w0);
              wrec[pp] = x[q];
              wtag[pp] = (uint8_t)lane;
            }
          }
        }
      }
      __syncthreads();
      ulonglong2 *dst = (ulonglong2 *)out + w0;
      for (uint32_t pp = t; pp < (uint32_t)(w1 - w0); pp += 256) {
        const uint32_t tg = wtag[pp];
        if (tg != 0xFFu) {
          const uint32_t r = wrec[pp];
          const uint64_t cb = sbase[tg];
          dst[pp] = make_ulonglong2(cb + (r & 0xFFFFu), cb + (r >> 16));
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------- one wave per haystack
// exec.rs:473-514 per search: the DFA on lane 0; the Pike VM on the whole
// wave when the DFA quits (or when there is no DFA).
template <bool EMIT>
__global__ __launch_bounds__(64) void iter_wave_kernel(BatchDev b, FwdDfaDev f, RevDfaDev r, NfaDev nf, int has_dfa,
                                                       uint32_t *counts, const uint64_t *off, uint64_t *out,
                                                       uint64_t cap, uint8_t *scratch, const uint64_t *entry,
                                                       uint64_t hi, uint64_t *exit, MatchDev m) {
  if (gated_off(b)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_mem[];
  uint8_t *mem = scratch ? scratch + (size_t)blockIdx.x * nfa_wave_bytes(nf.nleaves) : lds_mem;
  pike::Lists W;
  const uint32_t N = nf.nleaves;
  W.st[0] = (uint64_t *)mem;
  W.st[1] = W.st[0] + N;
  W.stamp = (uint32_t *)(W.st[1] + N);
  W.leaf[0] = W.stamp + N;
  W.leaf[1] = W.leaf[0] + N;
  const uint32_t lane = pike::lane_id();
  for (uint32_t i = lane; i < N; i += 64) W.stamp[i] = 0xFFFFFFFFu;
  pike::wave_sync();
  pike::TagGen tg;
  FwdDfaDev fg = f;
  fg.hot = 0;  // global-table stepping only (the LDS holds the Pike VM lists)
  fg.all = 0;
  for (uint64_t h = blockIdx.x; h < b.count; h += gridDim.x) {
    const uint8_t *base;
    uint64_t len;
    if (b.offs) {
      const uint64_t o0 = b.offs[h], o1 = b.offs[h + 1];
      base = b.hay + o0;
      len = o1 - o0;
    } else {
      base = b.hay + h * b.stride;
      len = b.length;
    }
    uint64_t p = b.start, lm = NONE, n = 0;
    if (entry && !entry[2]) {  // span entered with the previous span's state
      p = entry[0];
      lm = entry[1];
    }
    const uint64_t o0 = EMIT ? off[h] : 0, cnt = EMIT ? off[h + 1] - off[h] : 0;
    while (p <= len && (!EMIT || n < cnt)) {
      uint64_t s = NONE, e = NONE;
      int k = 2;
      if (has_dfa || m.mt >= 0) {
        uint64_t s0 = NONE, e0 = NONE;
        int k0 = 0;
        // one search: the reference's Literal / DfaSuffix search (m.mt >= 0,
        // match_device.hpp) or find_dfa_forward
        if (lane == 0)
          k0 = m.mt >= 0 ? mt_search<MODE_FIND>(m, fg, r, base, len, p, &s0, &e0)
                         : dfa_find(fg, r, nullptr, nullptr, base, len, p, &s0, &e0);
        k = __shfl(k0, 0);
        s = __shfl(s0, 0);
        e = __shfl(e0, 0);
      }
      if (k == 2) {
        uint64_t r0, r1;
        pike::pike_one<MODE_FIND>(nf, W, tg, base, len, p, &r0, &r1);
        k = r1 == NONE ? 0 : 1;
        s = r0;
        e = r1;
      }
      if (k == 0) break;
      if (s >= hi) break;  // owned by the next span
      if (s == e) {
        p = e + 1;
        if (lm == e) continue;
      } else {
        p = e;
      }
      lm = e;
      if (EMIT && lane == 0 && o0 + n < cap) {
        out[2 * (o0 + n)] = s;
        out[2 * (o0 + n) + 1] = e;
      }
      ++n;
    }
    if (!EMIT && lane == 0) {
      counts[h] = (uint32_t)n;
      if (exit) {
        exit[0] = p;
        exit[1] = lm;
        exit[2] = (p == hi && (lm != hi || f.nonempty)) ? 1 : 0;
      }
    }
  }
}

// counts[h] = matches of haystack h, total = all matches.
__device__ __forceinline__ void counts_body(uint64_t nh, uint64_t nk, const uint64_t *off, uint64_t *hcounts,
                                            uint64_t *total) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += (uint64_t)gridDim.x * blockDim.x)
    hcounts[h] = off[(h + 1) * nk] - off[h * nk];
  if (blockIdx.x == 0 && threadIdx.x == 0) *total = off[nh * nk] - off[0];
}
__global__ void iter_counts_kernel(uint64_t nh, uint64_t nk, const uint64_t *off, uint64_t *hcounts,
                                   uint64_t *total, BatchDev b) {
  if (gated_off(b)) return;
  counts_body(nh, nk, off, hcounts, total);
}

hipError_t scan_counts(const uint32_t *counts, uint64_t *off, uint64_t n, hipStream_t st) {
  // off[0..n] = exclusive prefix sums of counts[0..n) (off[n] = total)
  size_t tmp = 0;
  hipError_t e = rocprim::exclusive_scan(nullptr, tmp, counts, off, (uint64_t)0, (size_t)(n + 1),
                                         rocprim::plus<uint64_t>(), st);
  if (e != hipSuccess) return e;
  void *buf = nullptr;
  if ((e = scratch_malloc(&buf, tmp, st)) != hipSuccess) return e;
  e = rocprim::exclusive_scan(buf, tmp, counts, off, (uint64_t)0, (size_t)(n + 1), rocprim::plus<uint64_t>(), st);
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

// Dynamic LDS beyond 64 KiB must be opted into per kernel (a gfx950
// workgroup may use all 160 KiB).
template <typename K>
hipError_t allow_lds(K kernel, size_t bytes) {
  if (bytes <= 64 * 1024) return hipSuccess;
  return hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

int grid_cap(uint64_t items, int threads, int cus, int per_cu) {
  uint64_t g = (items + threads - 1) / threads;
  uint64_t cap = (uint64_t)cus * per_cu;
  if (g > cap) g = cap;
  return (int)(g < 1 ? 1 : g);
}

// ------------------------------------------ one search over long haystacks
// find / is_match / shortest_match (exec.rs:473-514, 382-420) when a batch
// holds few, long haystacks: every unit scans its chunk with the cut-bounded
// search (threads started in [c0, c1) only).  The leftmost-first match lives
// in the first unit whose threads reach a match state: its forward end equals
// the unrestricted search's (the earlier-started threads never match and the
// later-started ones are cut by the match or never outrank it), and the
// reverse pass runs over text[start..end] as the reference's does.  The
// earliest match end (shortest_match) is the minimum over units.
template <int MODE, bool PFX>
__global__ __launch_bounds__(256) void long_scan_kernel(BatchDev b, Geo g, uint64_t nunits, FwdDfaDev f, RevDfaDev r,
                                                        uint64_t *ures, unsigned long long *best) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint8_t *rlds = stage_tables(f, r, lds);
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nunits; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h, len, c0, c1;
    const uint8_t *base;
    unit_bounds(b, g, u, &h, &base, &len, &c0, &c1);
    LaneState L;
    lane_start(L, f, base, len, c0);
    if (c1 > c0 && c1 - 1 <= len) {
      fwd_range<MODE, PFX>(L, f, lds, base, c0, c1 - 1);
      if (!L.done) {
        L.s = f.strip[L.s];
        if (L.s == f.dead) L.done = true;
      }
      fwd_range<MODE>(L, f, lds, base, c1 - 1, len);
    } else {
      fwd_range<MODE, PFX>(L, f, lds, base, c0, len);
    }
    if (!L.done && f.eof[L.s]) L.last = len;
    if (L.last == NONE) continue;
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)best)[h] = 1;  // best = the u8 output itself (long_scan_m)
    } else if (MODE == MODE_SHORTEST) {
      atomicMin(&best[h], (unsigned long long)L.last);  // the u64 output itself
    } else {
      uint64_t ms, me = L.last;
      if (me == b.start) ms = me;  // exec.rs:647
      else {
        const uint64_t rs = rev_scan(r, rlds, base, len, b.start, me);
        ms = rs;
        if (rs == NONE) me = NONE;  // reverse NoMatch -> the search has no match
      }
      ures[2 * u] = ms;
      ures[2 * u + 1] = me;
      atomicMin(&best[h], (unsigned long long)u);
    }
  }
}

template <int MODE>
__global__ void long_finish_kernel(uint64_t count, const uint64_t *ures, const unsigned long long *best, void *out) {
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < count; h += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long v = best[h];
    if (MODE == MODE_ISMATCH) {
      ((uint8_t *)out)[h] = v == 1 ? 1 : 0;
    } else if (MODE == MODE_SHORTEST) {
      ((uint64_t *)out)[h] = v;
    } else {
      ((uint64_t *)out)[2 * h] = v == ~0ull ? NONE : ures[2 * v];
      ((uint64_t *)out)[2 * h + 1] = v == ~0ull ? NONE : ures[2 * v + 1];
    }
  }
}

template <int MODE>
hipError_t long_scan_m(const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, uint64_t chunk, void *out,
                       hipStream_t st, int cus) {
  Geo g;
  g.chunk = chunk;
  g.end = ~0ull;
  g.slots = 0;
  const uint64_t span = b.length > b.start ? b.length - b.start : 0;
  g.nk = span <= chunk ? 1 : (span + chunk - 1) / chunk;
  const uint64_t nunits = b.count * g.nk;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  // is_match / shortest_match write the output directly (a byte store / an
  // atomic min per haystack): no scratch and no finish pass — the scratch
  // cache's event per call had cost the latency-bound C1 step ~5 us
  const size_t sz_u = MODE == MODE_FIND ? nunits * 16 : 0, sz_b = MODE == MODE_FIND ? b.count * 8 : 0;
  uint8_t *buf = nullptr;
  hipError_t e = MODE == MODE_FIND ? scratch_malloc((void **)&buf, al(sz_u) + al(sz_b), st) : hipSuccess;
  if (e != hipSuccess) return e;
  uint64_t *ures = (uint64_t *)buf;
  unsigned long long *best = MODE == MODE_FIND ? (unsigned long long *)(buf + al(sz_u)) : (unsigned long long *)out;
  do {
    if (MODE == MODE_FIND)
      e = hipMemsetAsync(best, 0xFF, sz_b, st);
    else
      e = hipMemsetAsync(out, MODE == MODE_ISMATCH ? 0 : 0xFF, b.count * (MODE == MODE_ISMATCH ? 1 : 8), st);
    if (e != hipSuccess) break;
    const int per_cu = std::max<int>(1, std::min<int>(8, (int)((160u * 1024u) / std::max<size_t>(iter_lds_bytes(f, r), 1))));
    const dim3 lg(grid_cap(nunits, 256, cus, per_cu));
    // the start-state prefix skip (fwd_range<MODE, true>) for one prefix
    // first byte: measured faster there (Sherlock\s+\w+ 1.76 -> 1.54 ms per
    // GiB, >[^\n]*\n 1.10 -> 0.31) and slower with two ((?i)holmes\w*:
    // 1.46 -> 1.73 ms; profiles/r03_prefix_ab.jsonl)
    if (f.pfx_n == 1 || f.rare_on) {
      if ((e = allow_lds(long_scan_kernel<MODE, true>, iter_lds_bytes(f, r))) != hipSuccess) break;
      hipLaunchKernelGGL((long_scan_kernel<MODE, true>), lg, dim3(256), iter_lds_bytes(f, r), st, b, g, nunits, f, r,
                         ures, best);
    } else {
      if ((e = allow_lds(long_scan_kernel<MODE, false>, iter_lds_bytes(f, r))) != hipSuccess) break;
      hipLaunchKernelGGL((long_scan_kernel<MODE, false>), lg, dim3(256), iter_lds_bytes(f, r), st, b, g, nunits, f, r,
                         ures, best);
    }
    if ((e = hipGetLastError()) != hipSuccess) break;
    if (MODE == MODE_FIND) {
      hipLaunchKernelGGL(long_finish_kernel<MODE>, dim3(grid_cap(b.count, 256, cus, 4)), dim3(256), 0, st, b.count,
                         (const uint64_t *)ures, (const unsigned long long *)best, out);
      e = hipGetLastError();
    }
  } while (false);
  hipError_t e2 = buf ? scratch_free(buf, st) : hipSuccess;
  return e != hipSuccess ? e : e2;
}

}  // namespace

hipError_t launch_long_scan(int mode, const BatchDev &b, const FwdDfaDev &f, const RevDfaDev &r, uint64_t chunk,
                            void *out, hipStream_t st, int cus) {
  note_fwd_path(-4);
  switch (mode) {
    case MODE_FIND: return long_scan_m<MODE_FIND>(b, f, r, chunk, out, st, cus);
    case MODE_ISMATCH: return long_scan_m<MODE_ISMATCH>(b, f, r, chunk, out, st, cus);
    default: return long_scan_m<MODE_SHORTEST>(b, f, r, chunk, out, st, cus);
  }
}

// Unit geometry of a chunked find_iter: units of `chunk` bytes per haystack
// (offset batches: one unit per haystack); returns the number of units.
// Lexer engine (terminal matches + first-byte rule); RURE_AMD_LEX=0 disables.
// (haystacks below 4 GiB: the lexer's records are u32 offsets from the unit
// start, U_COMPACT; units of at most 64 KiB: its record queue packs two u16
// per register)
static bool lex_usable(const FwdDfaDev &f, const BatchDev &b, const Geo &g) {
  return f.lex_bytes && knob(Knob::Lex) != 0 && !b.offs && g.nk >= 2 && (g.chunk % 128) == 0 &&
         (b.count == 1 || (b.stride % 16) == 0) && (((uintptr_t)(b.hay + b.start)) & 15) == 0 &&
         b.length < (1ull << 32) && g.chunk <= 65536;
}

static uint64_t iter_geo(const BatchDev &b, uint64_t chunk, uint64_t hi, Geo *g) {
  const uint64_t lim = std::min<uint64_t>(b.length, hi);
  const uint64_t span = (!b.offs && lim > b.start) ? lim - b.start : 0;
  g->chunk = chunk;
  g->end = hi;
  g->nk = (b.offs || span <= chunk) ? 1 : (span + chunk - 1) / chunk;
  if (b.offs) g->chunk = ~0ull >> 2;
  g->slots = b.offs ? 16 : unit_slots(std::min<uint64_t>(g->chunk, span ? span : 1));
  return b.count * g->nk;
}

// Scratch of one chunked find_iter: units, slots, counts (n + 1), offsets
// (n + 1), repair queue, its length and the dirty flag; one allocation.
struct IterScratch {
  uint8_t *buf = nullptr;
  Unit *units;
  uint64_t *slots, *off, *queue;
  uint32_t *counts, *dirty;
  unsigned long long *qlen;
};

static hipError_t iter_scratch(uint64_t nunits, uint32_t nslots, hipStream_t st, IterScratch *sc) {
  // slots for whole groups of 64 units: the lexer's lanes past the last unit
  // flush their (empty) record queues unconditionally
  const size_t sz_units = nunits * sizeof(Unit), sz_slots = ((nunits + 63) & ~(uint64_t)63) * (size_t)nslots * 16;
  const size_t sz_counts = (nunits + 1) * 4, sz_off = (nunits + 1) * 8, sz_queue = nunits * 8;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t total = al(sz_units) + al(sz_slots) + al(sz_counts) + al(sz_off) + al(sz_queue) + 256;
  hipError_t e;
  if ((e = scratch_malloc((void **)&sc->buf, total, st)) != hipSuccess) return e;
  uint8_t *buf = sc->buf;
  sc->units = (Unit *)buf;
  sc->slots = (uint64_t *)(buf + al(sz_units));
  sc->counts = (uint32_t *)(buf + al(sz_units) + al(sz_slots));
  sc->off = (uint64_t *)(buf + al(sz_units) + al(sz_slots) + al(sz_counts));
  sc->queue = (uint64_t *)(buf + al(sz_units) + al(sz_slots) + al(sz_counts) + al(sz_off));
  sc->qlen = (unsigned long long *)(buf + total - 256);
  sc->dirty = (uint32_t *)(buf + total - 256 + 8);
  if ((e = hipMemsetAsync(sc->counts + nunits, 0, 4, st)) != hipSuccess) return e;
  return hipMemsetAsync(sc->qlen, 0, 16, st);  // qlen, dirty
}

static int iter_bs() {
  int bs = 256;
  if (knob(Knob::IterBs) > 0) bs = std::max(64, std::min<int>(1024, (int)knob(Knob::IterBs)));
  return bs;
}

static bool sa_usable(const FwdDfaDev &f) {
  return f.sa_len && knob(Knob::Sa) != 0 && knob(Knob::Lit) != 1;
}

static bool sa_tile_ok(const BatchDev &b, const Geo &g) {
  return !b.offs && g.nk >= 2 && (g.chunk % 128) == 0 && (b.count == 1 || (b.stride % 16) == 0) &&
         (((uintptr_t)(b.hay + b.start)) & 15) == 0 && knob(Knob::Sa) != 2;
}

// The passes after the speculative one (same for every engine): a span's
// entry, the repairs (fix, walk), the output offsets, emission, per-haystack
// counts and a span's exit.
// wnf: the wave-served iteration (U_QUIT units on the Pike VM, above):
// its blocks, threads per block, LDS bytes (and the walker's), kWave* mode.
struct WaveGeo {
  int grid = 0, threads = 64;
  size_t lds = 0, lds1 = 0;
  uint32_t mode = 0;
};
static hipError_t iter_post_body(const BatchDev &b, const Geo &g, uint64_t nunits, const FwdDfaDev &f,
                                 const RevDfaDev &r, const IterScratch &sc, const IterOut &o, const IterSpan *spn,
                                 hipStream_t st, int cus, bool dense, const NfaDev *wnf, uint8_t *wscr,
                                 const WaveGeo &wg);

static hipError_t iter_post(const BatchDev &b, const Geo &g, uint64_t nunits, const FwdDfaDev &f, const RevDfaDev &r,
                            const IterScratch &sc, const IterOut &o, const IterSpan *spn, hipStream_t st, int cus,
                            bool dense = false, const NfaDev *wnf = nullptr) {
  if (!wnf) return iter_post_body(b, g, nunits, f, r, sc, o, spn, st, cus, dense, nullptr, nullptr, WaveGeo{});
  // one wave per block, the Pike VM's lists in LDS (else global scratch)
  const size_t wb = nfa_wave_bytes(wnf->nleaves);
  // Lists in LDS where 16 waves per CU fit (kWaveLds).  Else 8 waves per
  // block share the NFA's tables in the LDS, each with its stamps there
  // (kWaveTables), where that fits; else stamps alone in the LDS at 16 waves
  // per CU (kWaveSplit), else all in scratch.  The waves' work is chains of
  // dependent loads, so waves in flight and LDS latency both count
  // (\b\w+n\b over 1 GiB of sherlock as it is, 2460 NFA leaves: 2 waves
  // per CU in LDS 186 ms; in scratch at 4 / 8 / 16 waves per CU 134 / 112 /
  // 102 ms; profiles/r06_wave_iter_bench.jsonl).  Knobs: wave_cu (waves per
  // CU, all in scratch), wave_split (0: no LDS stamps), wave_tables (0).
  const long long kw = knob(Knob::WaveCu);
  const int lds_cu = (int)std::min<size_t>(32, (160u * 1024u) / wb);
  const size_t tb = wave_table_bytes(*wnf), sb = wave_stamp_bytes(*wnf);
  constexpr int kWpb = 8;
  uint32_t mode;
  int wcu, wpb = 1;
  if (wb <= kNfaLdsMax && kw <= 0 && (lds_cu >= 16 || knob(Knob::WaveLds) == 1)) {
    mode = kWaveLds, wcu = lds_cu;
  } else if (kw <= 0 && knob(Knob::WaveTables) != 0 && tb + kWpb * sb <= 160u * 1024u) {
    mode = kWaveTables, wcu = kWpb, wpb = kWpb;
  } else {
    wcu = kw > 0 ? (int)std::min<long long>(kw, 32) : 16;
    mode = knob(Knob::WaveSplit) != 0 && sb * (size_t)wcu <= 160u * 1024u ? kWaveSplit : kWaveScratch;
  }
  const int wgrid = mode == kWaveTables ? std::max<int>(1, std::min<int>(cus, (int)((nunits + wpb - 1) / wpb)))
                                        : grid_cap(nunits, 1, cus, wcu);
  uint8_t *wscr = nullptr;
  hipError_t e = hipSuccess;
  if (mode != kWaveLds && (e = scratch_malloc((void **)&wscr, wb * (size_t)wgrid * wpb, st)) != hipSuccess) return e;
  const size_t wlds = mode == kWaveLds ? wb : mode == kWaveSplit ? sb : mode == kWaveTables ? tb + wpb * sb : 0;
  const size_t wlds1 = mode == kWaveTables ? tb + sb : wlds;  // the walker: one wave
  if (wlds > 64 * 1024 &&
      ((e = allow_lds(iter_wspec_kernel<false>, wlds)) != hipSuccess ||
       (e = allow_lds(iter_wspec_kernel<true>, wlds)) != hipSuccess || (e = allow_lds(iter_wfix_kernel, wlds)) != hipSuccess ||
       (e = allow_lds(iter_wwalk_kernel, wlds)) != hipSuccess || (e = allow_lds(iter_wemit_kernel, wlds)) != hipSuccess)) {
    (void)scratch_free(wscr, st);
    return e;
  }
  const WaveGeo wg{wgrid, wpb * 64, wlds, wlds1, mode};
  e = iter_post_body(b, g, nunits, f, r, sc, o, spn, st, cus, dense, wnf, wscr, wg);
  const hipError_t e2 = scratch_free(wscr, st);
  return e != hipSuccess ? e : e2;
}

static hipError_t iter_post_body(const BatchDev &b, const Geo &g, uint64_t nunits, const FwdDfaDev &f,
                                 const RevDfaDev &r, const IterScratch &sc, const IterOut &o, const IterSpan *spn,
                                 hipStream_t st, int cus, bool dense, const NfaDev *wnf, uint8_t *wscr,
                                 const WaveGeo &wg) {
  hipError_t e;
  const int bs = iter_bs();
  const size_t lb = iter_lds_bytes(f, r);
  const int per_cu = std::max<int>(1, std::min<int>(2048 / bs, (int)((160u * 1024u) / std::max<size_t>(lb, 1))));
  const int grid = grid_cap(nunits, bs, cus, per_cu);
  if ((e = allow_lds(iter_fix_kernel, lb)) != hipSuccess || (e = allow_lds(iter_emit_kernel, lb)) != hipSuccess)
    return e;
  FwdDfaDev fw0 = f;  // the wave kernels: global tables
  fw0.hot = 0;
  RevDfaDev rw0 = r;
  rw0.hot = 0;
  if (wnf) {
    // The quit units' speculation: a wave answers the search that quit and
    // hands the unit back to the lanes (kWaveRounds times: most units quit
    // once or twice, at a cluster of non-ASCII bytes), then the waves finish
    // what is still pending.
    if ((e = allow_lds(iter_spec_burst_kernel, lb)) != hipSuccess) return e;
    for (int k = 0; k < kWaveRounds; ++k) {
      hipLaunchKernelGGL(iter_wspec_kernel<true>, dim3(wg.grid), dim3(wg.threads), wg.lds, st, b, g, nunits, fw0, rw0, *wnf,
                         sc.units, sc.slots, sc.counts, sc.dirty, wscr, wg.mode);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      hipLaunchKernelGGL(iter_spec_burst_kernel, dim3(grid), dim3(bs), lb, st, b, g, nunits, f, r, sc.units, sc.slots,
                         sc.counts, sc.dirty, (uint32_t *)nullptr, 3u);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(iter_wspec_kernel<false>, dim3(wg.grid), dim3(wg.threads), wg.lds, st, b, g, nunits, fw0, rw0, *wnf,
                       sc.units, sc.slots, sc.counts, sc.dirty, wscr, wg.mode);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (spn && spn->entry) {
    FwdDfaDev fw = f;
    fw.hot = 0;
    RevDfaDev rw = r;
    rw.hot = 0;
    hipLaunchKernelGGL(iter_entry_kernel, dim3(1), dim3(64), 0, st, b, g, nunits, fw, rw, sc.units, sc.counts,
                       (const uint64_t *)sc.slots, spn->entry, sc.queue, sc.qlen);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (g.nk > 1) {
    hipLaunchKernelGGL(iter_fix_kernel, dim3(grid), dim3(bs), lb, st, b, g, nunits, f, r, sc.units, sc.counts,
                       (const uint64_t *)sc.slots, sc.queue, sc.qlen, (const uint32_t *)sc.dirty);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (wnf) {
      hipLaunchKernelGGL(iter_wfix_kernel, dim3(wg.grid), dim3(wg.threads), wg.lds, st, b, g, nunits, fw0, rw0, *wnf, sc.units,
                         sc.counts, (const uint64_t *)sc.slots, sc.queue, sc.qlen, (const uint32_t *)sc.dirty, wscr, wg.mode);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      hipLaunchKernelGGL(iter_wwalk_kernel, dim3(1), dim3(64), wg.lds1, st, b, g, nunits, fw0, rw0, *wnf, sc.units,
                         sc.counts, (const uint64_t *)sc.slots, sc.queue, sc.qlen, wscr, wg.mode);
    } else {
      hipLaunchKernelGGL(iter_walk_kernel, dim3(1), dim3(64), 0, st, b, g, nunits, fw0, rw0, sc.units, sc.counts,
                         (const uint64_t *)sc.slots, sc.queue, sc.qlen);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if ((e = scan_counts(sc.counts, sc.off, nunits, st)) != hipSuccess) return e;
  // a lexer pass (match-dense): its copies in output order first, then the
  // emit pass only re-runs units (needs a 16-byte aligned output)
  dense = dense && (((uintptr_t)o.matches) & 15) == 0;
  if (dense) {
    hipLaunchKernelGGL(iter_copy_group_kernel, dim3(grid_cap((nunits + 63) / 64, 1, cus, 8)), dim3(256), 0, st, b, g,
                       nunits, (const Unit *)sc.units, (const uint64_t *)sc.slots, (const uint64_t *)sc.off, o.matches,
                       o.cap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(iter_emit_kernel, dim3(grid), dim3(bs), lb, st, b, g, nunits, f, r, sc.units, sc.slots, sc.off,
                     o.matches, o.cap, dense ? 0 : 1);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (wnf) {
    hipLaunchKernelGGL(iter_wemit_kernel, dim3(wg.grid), dim3(wg.threads), wg.lds, st, b, g, nunits, fw0, rw0, *wnf,
                       (const Unit *)sc.units, (const uint64_t *)sc.off, o.matches, o.cap, wscr, wg.mode);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(iter_counts_kernel, dim3(grid_cap(b.count, 256, cus, 4)), dim3(256), 0, st, b.count, g.nk,
                     sc.off, o.counts, o.total, b);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (spn && spn->exit) {
    hipLaunchKernelGGL(iter_exit_kernel, dim3(1), dim3(64), 0, st, (const Unit *)sc.units, nunits, spn->exit,
                       spn->tail, f.nonempty);
    e = hipGetLastError();
  }
  return e;
}

template <int NW, int MQ>
__global__ __launch_bounds__(256) void iter_spec_sa_multi_tile_kernel(BatchDev b, Geo g, uint64_t nunits, SaMulti m) {
  multi_tile_body<NW, false, MQ>(b, g, nunits, m);
}
// The k-mer engine holds no Shift-And words: capped at 128 VGPRs for 4 waves
// per SIMD (16 per CU; HIP's second bound is waves per SIMD).  Blocks of 8
// waves share one bitmap: two blocks of 72.1 KB LDS per CU (four of 4 waves
// held 4 x 40 KB, all 160 KB).
template <int MQ>
__global__ __launch_bounds__(512, 4) void iter_spec_kmer_multi_tile_kernel(BatchDev b, Geo g, uint64_t nunits,
                                                                           SaMulti m) {
  multi_tile_body<1, true, MQ, 8>(b, g, nunits, m);
}

// The passes after a fused speculative pass for all its regexes at once:
// one launch per pass, blockIdx.y = the regex, its buffers and tables in a
// descriptor (the per-regex passes of iter_post took ~70 launches for the 9
// regex-dna variants).  The regexes' unit counts are segments of one array
// scanned once (emit / counts read their segment relative to its base).
struct PostDesc {
  FwdDfaDev f;
  RevDfaDev r;
  Unit *units;
  uint32_t *counts;
  const uint64_t *slots;
  uint64_t *off, *queue;
  unsigned long long *qlen;
  const uint32_t *dirty;
  uint64_t *out, cap, *hcounts, *total;
  const uint64_t *entry;
  uint64_t *exit, tail;
  uint32_t nonempty;
};

__global__ void multi_entry_kernel(BatchDev b, Geo g, uint64_t nunits, const PostDesc *d) {
  const PostDesc &P = d[blockIdx.y];
  if (threadIdx.x != 0 || blockIdx.x != 0 || !P.entry || P.entry[2]) return;
  FwdDfaDev fw = P.f;
  fw.hot = 0;
  RevDfaDev rw = P.r;
  rw.hot = 0;
  if (repair_unit(b, g, fw, rw, fw.lds_image /* unused: hot = 0 */, nullptr, 0, IterSt{P.entry[0], P.entry[1]},
                  P.units, P.counts, P.slots) &&
      g.nk > 1) {
    const unsigned long long q = atomicAdd(P.qlen, 1ull);
    P.queue[q] = 0;
  }
}

__global__ __launch_bounds__(1024) void multi_fix_kernel(BatchDev b, Geo g, uint64_t nunits, const PostDesc *d) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const PostDesc &P = d[blockIdx.y];
  fix_body(b, g, nunits, P.f, P.r, P.units, P.counts, P.slots, P.queue, P.qlen, P.dirty, lds);
}

__global__ void multi_walk_kernel(BatchDev b, Geo g, uint64_t nunits, const PostDesc *d) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const PostDesc &P = d[blockIdx.y];
  if (*P.qlen == 0) return;
  FwdDfaDev fw = P.f;
  fw.hot = 0;
  RevDfaDev rw = P.r;
  rw.hot = 0;
  walk_body(b, g, nunits, fw, rw, P.units, P.counts, P.slots, P.queue, P.qlen);
}

__global__ __launch_bounds__(1024) void multi_emit_kernel(BatchDev b, Geo g, uint64_t nunits, const PostDesc *d) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const PostDesc &P = d[blockIdx.y];
  emit_body<false>(b, g, nunits, P.f, P.r, P.units, P.slots, P.off, P.out, P.cap, lds);
}

__global__ void multi_counts_exit_kernel(BatchDev b, Geo g, uint64_t nunits, const PostDesc *d) {
  const PostDesc &P = d[blockIdx.y];
  counts_body(b.count, g.nk, P.off, P.hcounts, P.total);
  if (P.exit && blockIdx.x == 0 && threadIdx.x == 0) exit_body(P.units, nunits, P.exit, P.tail, P.nonempty);
}

// Several Shift-And regexes over the same span in one speculative pass
// (iter_spec_sa_multi_tile_kernel), then each regex's own passes.  Returns
// hipErrorNotSupported (nothing launched) when they do not qualify: every
// regex on the Shift-And engine with one string length, the tile geometry,
// at most kSaMultiMax regexes in at most kSaMultiWords (8) words of 32 bits,
// at most 32 bits per regex (a regex never straddles two words).
hipError_t launch_find_iter_multi(const BatchDev &b, int nre, const FwdDfaDev *const *f, const RevDfaDev *const *r,
                                  uint64_t chunk, const IterOut *o, hipStream_t st, int cus, const IterSpan *spn,
                                  const KmerDev *km) {
  if (nre < 1 || nre > kSaMultiMax || b.count != 1) return hipErrorNotSupported;
  Geo g;
  const uint64_t nunits = iter_geo(b, chunk, spn ? spn[0].hi : ~0ull, &g);
  if (!sa_tile_ok(b, g)) return hipErrorNotSupported;
  // every regex's scratch is live at once: fewer speculative slots per unit
  // (a unit with more matches is re-run by the emit pass instead of copied)
  g.slots = std::min<uint32_t>(g.slots, 16);
  SaMulti m{};
  m.nre = (uint32_t)nre;
  m.len = f[0]->sa_len;
  // knob kmer=0 keeps the Shift-And words (A/B)
  const bool kmer = km && km->bitmap && km->len == m.len && m.len == 8 && knob(Knob::Kmer) != 0;
  if (kmer) m.km = *km;
  // packed per-regex state (multi_record): positions up to chunk + L, and at
  // most one match per L bytes of a unit
  m.pbits = 1;
  while (m.pbits < 31 && (1ull << m.pbits) <= g.chunk + m.len + 1) ++m.pbits;
  if (m.len == 0 || m.pbits > 24 || (g.chunk / m.len + 2) >= (1ull << (32 - m.pbits))) return hipErrorNotSupported;
  uint32_t word = 0, used = 0;
  for (int q = 0; q < nre; ++q) {
    if (!sa_usable(*f[q]) || f[q]->sa_len != m.len || f[q]->sa_bits > 32) return hipErrorNotSupported;
    if (spn && spn[q].hi != spn[0].hi) return hipErrorNotSupported;
    if (used + f[q]->sa_bits > 32) { ++word; used = 0; }
    if (word >= (uint32_t)kSaMultiWords) return hipErrorNotSupported;
    m.word[q] = word;
    m.shift[q] = used;
    m.fin[q] = (uint32_t)f[q]->sa_final << used;
    m.init[word] |= (uint32_t)f[q]->sa_init << used;
    m.facc[word] |= m.fin[q];
    m.fany |= m.fin[q];
    m.nonempty[q] = f[q]->nonempty;
    m.sa_image[q] = f[q]->sa_image;
    used += f[q]->sa_bits;
  }
  const int nw = (int)word + 1;
  // one scratch for every regex: units, slots, the counts segments (one
  // scan), offsets, walker queues, control words, the image, descriptors
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const uint64_t seg = nunits + 1;
  const size_t sz_units = al(nunits * sizeof(Unit)), sz_slots = al(nunits * (size_t)g.slots * 16);
  const size_t sz_counts = al(nre * seg * 4), sz_off = al(nre * seg * 8), sz_queue = al(nunits * 8);
  const size_t sz_ctl = al((size_t)nre * 16), sz_img = al(256 * kSaMultiWords * 4), sz_desc = al(nre * sizeof(PostDesc));
  const size_t total = nre * (sz_units + sz_slots + sz_queue) + sz_counts + sz_off + sz_ctl + sz_img + sz_desc;
  uint8_t *buf = nullptr;
  hipError_t e = scratch_malloc((void **)&buf, total, st);
  if (e != hipSuccess) return e;
  uint8_t *q0 = buf;
  auto take = [&](size_t n) { uint8_t *r = q0; q0 += n; return r; };
  uint32_t *counts_all = (uint32_t *)take(sz_counts);
  uint64_t *off_all = (uint64_t *)take(sz_off);
  uint8_t *ctl = take(sz_ctl);
  m.image = (uint32_t *)take(sz_img);
  PostDesc *ddesc = (PostDesc *)take(sz_desc);
  std::vector<PostDesc> hd(nre);
  size_t lb = 0;
  bool entries = false;
  for (int q = 0; q < nre; ++q) {
    PostDesc &P = hd[q];
    P.f = *f[q];
    P.r = *r[q];
    P.units = (Unit *)take(sz_units);
    P.slots = (const uint64_t *)take(sz_slots);
    P.queue = (uint64_t *)take(sz_queue);
    P.counts = counts_all + q * seg;
    P.off = off_all + q * seg;
    P.qlen = (unsigned long long *)(ctl + 16 * q);
    P.dirty = (const uint32_t *)(ctl + 16 * q + 8);
    P.out = o[q].matches;
    P.cap = o[q].cap;
    P.hcounts = o[q].counts;
    P.total = o[q].total;
    P.entry = spn ? spn[q].entry : nullptr;
    P.exit = spn ? spn[q].exit : nullptr;
    P.tail = spn ? spn[q].tail : ~0ull;
    P.nonempty = f[q]->nonempty;
    entries = entries || P.entry;
    m.units[q] = P.units;
    m.slots[q] = (uint64_t *)P.slots;
    m.counts[q] = P.counts;
    m.dirty[q] = (uint32_t *)P.dirty;
    lb = std::max(lb, iter_lds_bytes(*f[q], *r[q]));
  }
  do {
    if ((e = hipMemsetAsync(counts_all, 0, nre * seg * 4, st)) != hipSuccess) break;
    if ((e = hipMemsetAsync(ctl, 0, (size_t)nre * 16, st)) != hipSuccess) break;
    if ((e = hipMemcpyAsync(ddesc, hd.data(), nre * sizeof(PostDesc), hipMemcpyHostToDevice, st)) != hipSuccess) break;
    const dim3 sg(grid_cap((nunits + 63) / 64, 4, cus, 4));
#define RURE_SAM(NWc)                                                                                   \
  case NWc:                                                                                             \
    hipLaunchKernelGGL(sa_multi_image_kernel<NWc>, dim3(1), dim3(256), 0, st, m);                       \
    ktimer_begin(st);                                                                                   \
    hipLaunchKernelGGL((iter_spec_sa_multi_tile_kernel<NWc, kSaMultiMax>), sg, dim3(256), 0, st, b, g,        \
                       nunits, m);                                                                      \
    ktimer_end(st);                                                                                     \
    break;
    if (kmer) {
      ktimer_begin(st);
      const dim3 kg(grid_cap((nunits + 63) / 64, 8, cus, 2));
      if (nre <= 4)
        hipLaunchKernelGGL((iter_spec_kmer_multi_tile_kernel<4>), kg, dim3(512), 0, st, b, g, nunits, m);
      else if (nre <= 9)
        hipLaunchKernelGGL((iter_spec_kmer_multi_tile_kernel<9>), kg, dim3(512), 0, st, b, g, nunits, m);
      else
        hipLaunchKernelGGL((iter_spec_kmer_multi_tile_kernel<kSaMultiMax>), kg, dim3(512), 0, st, b, g, nunits, m);
      ktimer_end(st);
    } else {
      switch (nw) {
        RURE_SAM(1) RURE_SAM(2) RURE_SAM(3) RURE_SAM(4) RURE_SAM(5) RURE_SAM(6) RURE_SAM(7) RURE_SAM(8)
        default: e = hipErrorNotSupported;
      }
    }
#undef RURE_SAM
    if (e != hipSuccess) break;
    if ((e = hipGetLastError()) != hipSuccess) break;
    // the passes of iter_post, each once for all regexes (blockIdx.y)
    const int bs = iter_bs();
    const int per_cu = std::max<int>(1, std::min<int>(2048 / bs, (int)((160u * 1024u) / std::max<size_t>(lb, 1))));
    const uint32_t grid = (uint32_t)grid_cap(nunits, bs, cus, per_cu);
    if ((e = allow_lds(multi_fix_kernel, lb)) != hipSuccess || (e = allow_lds(multi_emit_kernel, lb)) != hipSuccess)
      break;
    if (entries) hipLaunchKernelGGL(multi_entry_kernel, dim3(1, nre), dim3(64), 0, st, b, g, nunits, ddesc);
    if (g.nk > 1) {
      hipLaunchKernelGGL(multi_fix_kernel, dim3(grid, nre), dim3(bs), lb, st, b, g, nunits, ddesc);
      hipLaunchKernelGGL(multi_walk_kernel, dim3(1, nre), dim3(64), 0, st, b, g, nunits, ddesc);
    }
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = scan_counts(counts_all, off_all, nre * seg - 1, st)) != hipSuccess) break;
    hipLaunchKernelGGL(multi_emit_kernel, dim3(grid, nre), dim3(bs), lb, st, b, g, nunits, ddesc);
    hipLaunchKernelGGL(multi_counts_exit_kernel, dim3(grid_cap(b.count, 256, cus, 4), nre), dim3(256), 0, st, b, g,
                       nunits, ddesc);
    e = hipGetLastError();
  } while (false);
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

hipError_t launch_find_iter(const BatchDev &b, const FwdDfaDev *f, const RevDfaDev &r, const NfaDev *nf,
                            bool chunked, uint64_t chunk, const IterOut &o, hipStream_t st, int cus,
                            const IterSpan *spn, const MatchDev *mtd, bool *quit, uint32_t *quit_dev) {
  const uint64_t hi = spn ? spn->hi : ~0ull;
  if (quit_dev && (!chunked || spn || b.gate || !f || !f->can_quit)) return hipErrorInvalidValue;
  // chunked, a DFA that can quit, no quit flag asked for: the wave-served
  // iteration (the quit units' searches on the Pike VM; no span)
  const bool wq = chunked && f && f->can_quit && !quit && !quit_dev && nf;
  if (wq && spn) return hipErrorInvalidValue;
  hipError_t e = hipSuccess;
  if (b.count == 0) {
    return hipMemsetAsync(o.total, 0, 8, st);
  }
  if (chunked) {
    Geo g;
    const uint64_t nunits = iter_geo(b, chunk, hi, &g);
    // Dense matches: the caller's capacity tells how many to expect; slots
    // that hold them spare the emit pass re-running every unit (\b\w+\b over
    // English, ~750 matches per 4 KiB unit: 128 slots re-ran them all, 19 of
    // 33 ms).  Not for the lexer (its compact rows), at most 4 GiB.
    if (!lex_usable(*f, b, g) && !b.offs && o.cap > (uint64_t)g.slots * nunits) {
      const uint64_t per = (o.cap + nunits - 1) / nunits;
      const uint64_t want = std::min<uint64_t>(per + per / 4 + 4, std::min<uint64_t>(g.chunk + 1, 8192));
      if (want > g.slots && want * nunits * 16 <= (4ull << 30)) g.slots = (uint32_t)want;
    }
    IterScratch sc;
    if ((e = iter_scratch(nunits, g.slots, st, &sc)) != hipSuccess) return e;
    // threads per block: the hot tables are staged once per block, so larger
    // blocks let more waves share one LDS copy (occupancy of these latency-
    // bound per-lane scans); RURE_AMD_ITER_BS overrides (tuning)
    const int bs = iter_bs();
    const int per_cu = std::max<int>(1, std::min<int>(2048 / bs, (int)((160u * 1024u) / std::max<size_t>(iter_lds_bytes(*f, r), 1))));
    const int grid = grid_cap(nunits, bs, cus, per_cu);
    Unit *units = sc.units;
    uint64_t *slots = sc.slots;
    uint32_t *counts = sc.counts, *dirty = sc.dirty;
    do {
      const size_t lb = iter_lds_bytes(*f, r);
      if ((e = allow_lds(iter_spec_burst_kernel, lb)) != hipSuccess || (e = allow_lds(iter_fix_kernel, lb)) != hipSuccess ||
          (e = allow_lds(iter_emit_kernel, lb)) != hipSuccess)
        break;
      // Literal engine: where the DFA does not fit LDS exactly (> 255 states,
      // e.g. alternations of many words) it wins clearly (tools/lit_vs_dfa.py:
      // 16 words 2.29 -> 0.72 ms, 64 words 5.43 -> 2.29 ms per GiB); with a
      // small DFA it depends on the text (English -25 %, DNA +25 %), so the
      // DFA stays.  Knob lit=1 / 0 forces it on / off.
      // (a DFA that can quit takes the burst kernel: it alone hands quits
      // and starts after a byte >= 0x80 over, iter_next)
      const bool use_lit = !f->can_quit && f->lit_n && (knob(Knob::Lit) >= 0 ? knob(Knob::Lit) == 1 : !f->all);
      // Shift-And engine for equal-length string sets; RURE_AMD_SA=0 disables
      const bool use_sa = !f->can_quit && sa_usable(*f);
      const bool sa_tile = sa_tile_ok(b, g);
      // Lexer engine (terminal matches + first-byte rule); RURE_AMD_LEX=0 disables
      const bool use_lex = !f->can_quit && lex_usable(*f, b, g);
      // the quit flag (a caller that re-runs on a quit): zeroed here, set by
      // the burst kernel's first quit (the others stop) and by iter_quit_kernel
      uint32_t *qd = quit_dev;
      if (!qd && f->can_quit && quit) {
        if ((e = scratch_malloc((void **)&qd, 8, st)) != hipSuccess) break;
        if ((e = hipMemsetAsync(qd, 0, 4, st)) != hipSuccess) { (void)scratch_free(qd, st); break; }
      }
      ktimer_begin(st);  // bench diagnostics: the speculative kernel's duration
      if (use_lex) {
        const dim3 lg(grid_cap((nunits + 63) / 64, 4, cus, 4));
        const bool one = b.count == 1;
        if (f->lex4_image && one)
          hipLaunchKernelGGL((iter_spec_lex_tile_kernel<true, true>), lg, dim3(256), 0, st, b, g, nunits, *f, units,
                             slots, counts);
        else if (f->lex4_image)
          hipLaunchKernelGGL((iter_spec_lex_tile_kernel<true, false>), lg, dim3(256), 0, st, b, g, nunits, *f, units,
                             slots, counts);
        else if (one)
          hipLaunchKernelGGL((iter_spec_lex_tile_kernel<false, true>), lg, dim3(256), 0, st, b, g, nunits, *f, units,
                             slots, counts);
        else
          hipLaunchKernelGGL((iter_spec_lex_tile_kernel<false, false>), lg, dim3(256), 0, st, b, g, nunits, *f, units,
                             slots, counts);
        ktimer_end(st);
        if ((e = hipGetLastError()) != hipSuccess) break;
        if ((e = allow_lds(iter_lex_tail_kernel, lb)) != hipSuccess) break;
        if (knob(Knob::LexTail) != 0)
          hipLaunchKernelGGL(iter_lex_tail_kernel, dim3(grid_cap(nunits, 256, cus, 8)), dim3(256), lb, st, b, g, nunits,
                           *f, r, units, slots, counts, dirty);
      } else if (use_sa && sa_tile) {
        const dim3 sg(grid_cap((nunits + 63) / 64, 4, cus, 4));
        if (f->sa_bits <= 32)
          hipLaunchKernelGGL((iter_spec_sa_tile_kernel<uint32_t>), sg, dim3(256), 0, st, b, g, nunits, *f, units,
                             slots, counts, dirty);
        else
          hipLaunchKernelGGL((iter_spec_sa_tile_kernel<uint64_t>), sg, dim3(256), 0, st, b, g, nunits, *f, units,
                             slots, counts, dirty);
      } else if (use_sa) {
        const dim3 sg(grid_cap(nunits, 256, cus, 8));
        if (f->sa_bits <= 32)
          hipLaunchKernelGGL((iter_spec_sa_kernel<uint32_t>), sg, dim3(256), 0, st, b, g, nunits, *f, units, slots,
                             counts, dirty);
        else
          hipLaunchKernelGGL((iter_spec_sa_kernel<uint64_t>), sg, dim3(256), 0, st, b, g, nunits, *f, units, slots,
                             counts, dirty);
      } else if (use_lit) {
        const dim3 lg(grid_cap(nunits, bs, cus, 2048 / bs));
        if (f->lit_k8)
          hipLaunchKernelGGL((iter_spec_lit_kernel<true, true>), lg, dim3(bs), kLitImage, st, b, g, nunits, *f, units,
                             slots, counts, dirty);
        else if (f->lit_k == 4)
          hipLaunchKernelGGL((iter_spec_lit_kernel<true, false>), lg, dim3(bs), kLitImage, st, b, g, nunits, *f, units,
                             slots, counts, dirty);
        else
          hipLaunchKernelGGL((iter_spec_lit_kernel<false, false>), lg, dim3(bs), kLitImage, st, b, g, nunits, *f,
                             units, slots, counts, dirty);
      } else {
        hipLaunchKernelGGL(iter_spec_burst_kernel, dim3(grid), dim3(bs), iter_lds_bytes(*f, r), st, b, g, nunits, *f,
                           r, units, slots, counts, dirty, qd, wq ? 1u : 0u);
      }
      if (!use_lex) ktimer_end(st);
      if ((e = hipGetLastError()) != hipSuccess) {
        if (qd && !quit_dev) (void)scratch_free(qd, st);
        break;
      }
      // deferred: the quit check stays on the device and gates the rest
      if (quit_dev) {
        hipLaunchKernelGGL(iter_quit_kernel, dim3(grid_cap(nunits, 256, cus, 4)), dim3(256), 0, st, units, nunits,
                           quit_dev);
        if ((e = hipGetLastError()) != hipSuccess) break;
        BatchDev bg = b;
        bg.gate = quit_dev;
        bg.gate_set = 0;
        e = iter_post(bg, g, nunits, *f, r, sc, o, spn, st, cus, use_lex);
        break;
      }
      // a quit in the speculative pass ends the call here: the caller re-runs
      // the batch on the full automaton or the wave path, and the fix walk
      // over quit units is serial (the ASCII shadow over sherlock as it is,
      // a non-ASCII byte every few KiB: 17 s; then 47.6 ms with the whole
      // speculative pass run, against 38.4 ms on the full automaton alone;
      // profiles/r05_shadow_bench.jsonl)
      if (qd) {
        uint32_t q = 0;
        if (e == hipSuccess) {
          hipLaunchKernelGGL(iter_quit_kernel, dim3(grid_cap(nunits, 256, cus, 4)), dim3(256), 0, st, units, nunits,
                             qd);
          e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&q, qd, 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        const hipError_t e2 = scratch_free(qd, st);
        if (e == hipSuccess) e = e2;
        if (e != hipSuccess) break;
        if (q) {
          *quit = true;
          break;
        }
      }
      e = iter_post(b, g, nunits, *f, r, sc, o, spn, st, cus, use_lex, wq ? nf : nullptr);
      if (e == hipSuccess && f->can_quit && quit) {  // did any search quit?
        uint32_t q = 0;
        if ((e = hipMemsetAsync(dirty, 0, 4, st)) != hipSuccess) break;
        hipLaunchKernelGGL(iter_quit_kernel, dim3(grid_cap(nunits, 256, cus, 4)), dim3(256), 0, st, units, nunits,
                           dirty);
        if ((e = hipMemcpyAsync(&q, dirty, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) break;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) break;
        *quit = q != 0;
      }
    } while (false);
    hipError_t e2 = scratch_free(sc.buf, st);
    return e != hipSuccess ? e : e2;
  }
  // one wavefront per haystack (assertions, DFA quit, or no DFA)
  const size_t wb = nfa_wave_bytes(nf->nleaves);
  const bool use_lds = wb <= kNfaLdsMax;
  const int grid = grid_cap(b.count, 1, cus, use_lds ? std::max<int>(1, std::min<int>(32, (int)((160u * 1024u) / wb))) : 4);
  uint8_t *buf = nullptr;
  const size_t sz_counts = (b.count + 1) * 4, sz_off = (b.count + 1) * 8;
  const size_t sz_scr = use_lds ? 0 : wb * (size_t)grid;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  if ((e = scratch_malloc((void **)&buf, al(sz_counts) + al(sz_off) + al(sz_scr), st)) != hipSuccess) return e;
  uint32_t *counts = (uint32_t *)buf;
  uint64_t *off = (uint64_t *)(buf + al(sz_counts));
  uint8_t *scr = use_lds ? nullptr : buf + al(sz_counts) + al(sz_off);
  const size_t lds = use_lds ? wb : 0;
  FwdDfaDev fz{};
  const FwdDfaDev &fa = f ? *f : fz;
  const MatchDev md = mtd ? *mtd : MatchDev{-1, {}, {}, nullptr, 0};
  do {
    if (lds > 64 * 1024) {
      if ((e = hipFuncSetAttribute((const void *)iter_wave_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds)) != hipSuccess)
        break;
      if ((e = hipFuncSetAttribute((const void *)iter_wave_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds)) != hipSuccess)
        break;
    }
    if ((e = hipMemsetAsync(counts + b.count, 0, 4, st)) != hipSuccess) break;
    hipLaunchKernelGGL(iter_wave_kernel<false>, dim3(grid), dim3(64), lds, st, b, fa, r, *nf, f ? 1 : 0, counts,
                       (const uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t)0, scr,
                       spn ? spn->entry : (const uint64_t *)nullptr, hi, spn ? spn->exit : (uint64_t *)nullptr, md);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = scan_counts(counts, off, b.count, st)) != hipSuccess) break;
    hipLaunchKernelGGL(iter_wave_kernel<true>, dim3(grid), dim3(64), lds, st, b, fa, r, *nf, f ? 1 : 0, counts,
                       (const uint64_t *)off, o.matches, o.cap, scr,
                       spn ? spn->entry : (const uint64_t *)nullptr, hi, (uint64_t *)nullptr, md);
    if ((e = hipGetLastError()) != hipSuccess) break;
    hipLaunchKernelGGL(iter_counts_kernel, dim3(grid_cap(b.count, 256, cus, 4)), dim3(256), 0, st, b.count,
                       (uint64_t)1, off, o.counts, o.total, b);
    e = hipGetLastError();
  } while (false);
  hipError_t e2 = scratch_free(buf, st);
  return e != hipSuccess ? e : e2;
}

}  // namespace rure_amd
