// Flattened Pike-VM tables for the GPU NFA kernel.
//
// The reference Pike VM (src/pikevm.rs:130-352) keeps an ordered thread list
// per position; `add` walks epsilon edges depth first (Split: goto1 before
// goto2, pikevm.rs:319-352) and records a thread at every Bytes / Match
// instruction it reaches, skipping instructions already in the list.  The
// kernel replaces the walk by precomputed *closures*: for every instruction a
// thread can resume at (the program start and every Bytes goto) we list, in
// the walk's order, the leaf instructions (Bytes / Match) it reaches and the
// look-around assertions (EmptyLook, prog.rs:334-351) on the path to each.
// At run time a leaf is taken if its assertions hold at the position and it
// is not in the list yet; that reproduces the walk exactly, because the
// assertions are the same for every walk done at one position.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "program.hpp"

namespace rure_amd {

struct NfaLeaf {         // 12 bytes, device layout
  uint8_t kind;          // 0 = Bytes, 1 = Match
  uint8_t lo, hi, pad;
  uint32_t closure;      // Bytes: closure id of its goto
  uint32_t slot;         // Match: match slot (pattern index)
};

struct NfaEntry {        // 8 bytes, device layout
  uint32_t leaf;         // leaf index
  uint32_t cond_prev;    // bits 0-7: required looks (1 << Look); bits 8-31: 1 + index (within
                         // the closure) of the previous entry with the same leaf, 0 if none
};

struct NfaTables {
  std::vector<NfaLeaf> leaves;
  std::vector<uint32_t> cl_off;     // closures, CSR offsets (n_closures + 1)
  std::vector<NfaEntry> entries;
  uint32_t root = 0;                // closure of the program start
  uint32_t nmatch = 1;              // Match instructions (patterns)
  bool anchored_start = false;
  bool unicode_wb = false;          // needs Unicode word-character tests
  uint32_t looks_used = 0;          // union of all assertion bits
  size_t max_closure = 0;
  // Capture slots set on the path to each entry (pikevm.rs:319-352: every
  // Save on the walk sets its slot to the current position): CSR by entry.
  std::vector<uint32_t> save_off;   // entries.size() + 1
  std::vector<uint16_t> save_slot;
};

bool build_nfa_tables(const Program &prog, NfaTables *out, std::string *err);

}  // namespace rure_amd
