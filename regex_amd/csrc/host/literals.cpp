// See literals.hpp.
#include "literals.hpp"

#include <algorithm>
#include <set>

namespace rure_amd {

namespace {

struct Walk {
  const Program &p;
  size_t max_lits, max_len;
  std::vector<std::string> lits;
  std::set<std::string> seen;
  std::string cur;
  size_t steps = 0;
  bool fail = false;

  // Depth-first over the program in priority order; `eps` counts the
  // epsilon instructions since the last byte (a longer chain is a loop).
  void go(uint32_t pc, size_t eps) {
    if (fail) return;
    if (++steps > 200000 || eps > p.insts.size() || pc >= p.insts.size()) {
      fail = true;
      return;
    }
    const Inst &in = p.insts[pc];
    switch (in.op) {
      case OP_MATCH:
        if (cur.empty()) { fail = true; return; }  // empty matches: the DFA's rules apply
        if (seen.insert(cur).second) {             // a later duplicate can never win
          lits.push_back(cur);
          if (lits.size() > max_lits) fail = true;
        }
        return;
      case OP_SAVE:
        go(in.x, eps + 1);
        return;
      case OP_SPLIT:
        go(in.x, eps + 1);
        go(in.y, eps + 1);
        return;
      case OP_EMPTY:  // look-around: not a plain string set
        fail = true;
        return;
      case OP_BYTES:
        if (cur.size() >= max_len) { fail = true; return; }
        for (uint32_t b = in.lo; b <= in.hi && !fail; ++b) {
          cur.push_back((char)b);
          go(in.x, 0);
          cur.pop_back();
        }
        return;
      default:
        fail = true;
    }
  }
};

}  // namespace

bool extract_literals(const Program &prog, size_t max_lits, size_t max_len, LiteralSet *out) {
  if (prog.is_dfa || prog.is_reverse || prog.matches.size() != 1 || prog.anchored_start || prog.anchored_end)
    return false;
  Walk w{prog, max_lits, max_len, {}, {}, {}};
  w.go(prog.start, 0);
  if (w.fail || w.lits.empty()) return false;
  out->lits = std::move(w.lits);
  out->minlen = out->lits[0].size();
  out->maxlen = 0;
  for (const std::string &s : out->lits) {
    out->minlen = std::min(out->minlen, s.size());
    out->maxlen = std::max(out->maxlen, s.size());
  }
  return true;
}

bool can_match_empty(const Program &prog) {
  std::vector<uint8_t> seen(prog.insts.size(), 0);
  std::vector<uint32_t> stack{prog.start};
  while (!stack.empty()) {
    const uint32_t pc = stack.back();
    stack.pop_back();
    if (pc >= prog.insts.size() || seen[pc]) continue;
    seen[pc] = 1;
    const Inst &in = prog.insts[pc];
    switch (in.op) {
      case OP_MATCH: return true;
      case OP_SAVE:
      case OP_EMPTY: stack.push_back(in.x); break;
      case OP_SPLIT: stack.push_back(in.x); stack.push_back(in.y); break;
      default: break;  // OP_BYTES consumes a byte
    }
  }
  return false;
}

}  // namespace rure_amd
