// Offline (eager) DFA materialization of a byte Program.
//
// The reference builds its DFA lazily during search (src/dfa.rs: exec_byte
// 910-1048, follow_epsilons 1073-1134, cached_state_key 1196-1244,
// start_state 1370-1409, start_flags 1415-1464).  A GPU cannot build states
// on the fly, so we run the very same subset construction eagerly over every
// state reachable from every start-flag combination, then minimise it
// (Moore partition refinement).  Laziness, cache flushes and state numbering
// only change *when* states are built, never which language they accept
// (dfa.rs:1176-1183, prog.rs:63-68), so offsets stay bit-identical.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "program.hpp"

namespace rure_amd {

// One materialized + minimised DFA.  State numbering (kernel contract):
//   [0, n_normal)            ordinary states (no match flag)
//   [n_normal, n_match_end)  states carrying the (one-byte delayed) match flag
//                            (sets: states whose entry reports matches, now_mask)
//   dead                     == n_match_end      (absorbing, never matches)
//   quit                     == n_match_end + 1  (only if has_quit)
struct DenseDfa {
  int nstates = 0;
  int n_normal = 0;
  int n_match_end = 0;
  int dead = 0;
  int quit = -1;
  bool is_set = false;
  bool reverse = false;
  std::vector<uint32_t> trans;     // nstates * 256, next state per byte
  std::vector<uint8_t> eof_match;  // per state: EOF transition yields a match flag
  std::vector<uint64_t> eof_mask;  // sets: Match slots reached at the end of the text (EOF step)
  std::vector<uint64_t> now_mask;  // sets: Match slots reached by the step into this state
                                   // ([n_normal, n_match_end) are exactly the states with now_mask != 0)
  uint32_t start[128];             // start state per 7-bit start-flag index (dfa.rs:1381-1390)
  int raw_states = 0;              // states before minimisation (diagnostics)
  int n_ascii = 0;                 // normal states reachable through ASCII bytes (numbered first)
  // With DfaBuildLimits::strip: strip[s] = the state holding the same threads
  // as s minus the `.*?` prefix, i.e. no new match may start from here on
  // (used to end a search once it crosses a chunk cut).
  std::vector<uint32_t> strip;
  // Column form (DfaBuildLimits::columns, the u32 tables of automata past
  // 65535 states): trans is empty and ctrans holds nstates * ncol next states,
  // column colmap[b] for byte b (the byte classes, split at 0x80 when a
  // Unicode word boundary makes non-ASCII bytes quit).
  uint32_t ncol = 0;
  uint8_t colmap[256] = {0};
  std::vector<uint32_t> ctrans;
};

struct DfaBuildLimits {
  int max_raw_states = 1 << 16;
  bool strip = false;
  bool columns = false;   // emit ctrans / colmap instead of the 256-wide trans
  bool minimise = true;   // false: raw states kept (same language, more states)
  size_t max_bytes = 0;   // construction memory budget (state keys + rows, estimated); 0 = none
  bool ascii_only = false;  // every byte >= 0x80 goes to QUIT (an ASCII shadow of the automaton)
};
// Drops the states no start state reaches (through transitions and strip
// links), keeping the numbering's classes and order (normal with the ASCII-
// reachable ones first, match-flag, dead, quit).  Row form, non-set only.
void prune_unreachable(DenseDfa *d);
// Raw-state budget of the eager u32 (column form) automata; past it the
// on-demand DFA (LazyDfa) builds only the states a batch visits.  (At 1 << 21
// the failed eager attempt for (?:a|b)*a(?:a|b){20} cost ~5 s.)
constexpr int kBigDfaRawStates = 1 << 18;
// Construction memory budget of the u32 automata (RURE_AMD_BIG_BYTES overrides).
constexpr size_t kBigDfaBytes = (size_t)1 << 30;

// Builds the DFA for `prog` (a forward DFA program with `.*?` unless anchored,
// or a reverse program).  Returns false (with `err`) if the state budget is
// exceeded.
bool build_dense_dfa(const Program &prog, const DfaBuildLimits &lim, DenseDfa *out,
                     std::string *err);

// On-demand construction past the eager budgets: the reference's lazy DFA
// (dfa.rs:910-1048 exec_byte, 1282-1320 cache) restated for batched scans.
// States are the subset construction's raw ids (0 = dead), numbered as they
// are discovered; a row is built when a scan first needs it (or ahead, in
// discovery order, by expand).  Table entries for the device: the next
// state's id, | kLazyMatch when that state carries the (one-byte delayed)
// match flag; kLazyUnknown for a row not built yet (the kernel parks the
// lane there).  Columns are the program's byte classes (no quit states:
// Unicode word boundaries keep the Pike VM).
constexpr uint32_t kLazyMatch = 0x80000000u, kLazyUnknown = 0x7FFFFFFFu;
class LazyDfa {
 public:
  LazyDfa(const Program &prog, size_t max_bytes);
  ~LazyDfa();
  LazyDfa(const LazyDfa &) = delete;
  LazyDfa &operator=(const LazyDfa &) = delete;
  // Builds state s's row (false: the memory budget is spent).
  bool build_row(uint32_t s);
  // Builds up to `rows` more rows in discovery order.
  bool expand(size_t rows);
  uint32_t nstates() const { return (uint32_t)eof.size(); }
  size_t nbuilt() const { return nbuilt_; }
  uint32_t ncol = 0;
  uint8_t colmap[256] = {0};
  uint32_t start[128];            // entries (id | kLazyMatch) per start-flag index
  std::vector<uint32_t> trans;    // nstates * ncol entries
  std::vector<uint8_t> eof;       // per state: the EOF step yields a match
  std::vector<uint8_t> built;     // per state: its row is built
 private:
  struct Impl;
  Impl *impl_ = nullptr;
  size_t max_bytes_ = 0, nbuilt_ = 0;
  std::vector<uint32_t> todo_;
  size_t todo_head_ = 0;
  uint32_t entry_of(uint32_t s) const;
  void sync_new();
};

// Start-flag index for a forward search starting at `at` (dfa.rs:1415-1434).
int start_flag_index_fwd(const uint8_t *text, size_t len, size_t at);
// Start-flag index for a reverse search ending at `at` (dfa.rs:1440-1464).
int start_flag_index_rev(const uint8_t *text, size_t len, size_t at);

}  // namespace rure_amd
