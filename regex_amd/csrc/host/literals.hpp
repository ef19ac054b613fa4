// Finite-language expansion of a compiled byte program, for the literal
// find_iter engine (the GPU counterpart of the reference's complete-prefix
// Literal engine: exec.rs:1148-1166 choose_match_type, exec.rs:601-625
// find_literals, literals.rs:28-250 LiteralSearcher).
//
// The reference uses its literal searchers (memchr / Teddy / Aho-Corasick)
// only when the regex's prefix literals are "complete", i.e. the regex is a
// finite set of strings.  Here the set is read off the NFA program itself:
// every path from the start to Match, in the Pike VM's priority order (a
// Split's first branch first, pikevm.rs:284-352), is one literal, so at any
// start position the first literal of the list that matches is the
// leftmost-first match (the path the reference's engines prefer).  Programs
// with look-around, loops, the empty string, or more than `max_lits` strings
// or strings longer than `max_len` bytes do not qualify (the DFA runs).
#pragma once
#include <cstddef>
#include <string>
#include <vector>

#include "program.hpp"

namespace rure_amd {

struct LiteralSet {
  std::vector<std::string> lits;  // leftmost-first priority order, distinct
  size_t minlen = 0, maxlen = 0;
};

bool extract_literals(const Program &prog, size_t max_lits, size_t max_len, LiteralSet *out);

// True if a Match instruction is reachable from the start without consuming
// a byte (look-around assertions taken as passable): the regex may match the
// empty string, so re_trait.rs:205-214's empty-match rule can apply.
bool can_match_empty(const Program &prog);

}  // namespace rure_amd
