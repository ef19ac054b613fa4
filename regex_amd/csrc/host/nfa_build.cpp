// Closure tables for the GPU Pike VM (see nfa_build.hpp).
#include "nfa_build.hpp"

#include <map>
#include <utility>

namespace rure_amd {

namespace {

struct Builder {
  const Program &p;
  NfaTables &t;
  std::vector<int32_t> leaf_of;          // inst -> leaf index (-1: not a leaf)
  std::map<uint32_t, uint32_t> cl_of;    // resume inst -> closure id
  std::vector<uint32_t> pending;         // resume insts whose closure is not built yet

  Builder(const Program &p_, NfaTables &t_) : p(p_), t(t_), leaf_of(p_.insts.size(), -1) {}

  uint32_t closure_id(uint32_t ip) {
    auto it = cl_of.find(ip);
    if (it != cl_of.end()) return it->second;
    uint32_t id = (uint32_t)cl_of.size();
    cl_of.emplace(ip, id);
    pending.push_back(ip);
    return id;
  }

  uint32_t leaf_id(uint32_t ip) {
    if (leaf_of[ip] >= 0) return (uint32_t)leaf_of[ip];
    const Inst &in = p.insts[ip];
    NfaLeaf l{};
    if (in.op == OP_MATCH) {
      l.kind = 1;
      l.slot = in.x;
    } else {
      l.kind = 0;
      l.lo = in.lo;
      l.hi = in.hi;
      l.closure = closure_id(in.x);
    }
    leaf_of[ip] = (int32_t)t.leaves.size();
    t.leaves.push_back(l);
    return (uint32_t)leaf_of[ip];
  }

  // Depth-first walk in the reference's order (pikevm.rs:319-352): Split
  // follows goto1 first; Save is transparent but recorded; EmptyLook adds its
  // assertion.  An instruction already walked with a subset of the current
  // assertions is not walked again (everything it reaches was already
  // listed, by a path that is taken whenever this one would be); entries
  // dominated by an earlier entry of the same leaf with a subset of its
  // assertions are dropped.
  struct Raw {
    uint32_t ip, cond;
    int32_t saves;  // node in `snodes` (the Saves on the path), -1 if none
  };
  std::vector<std::pair<uint16_t, int32_t>> snodes;  // (slot, parent node)

  std::vector<Raw> walk(uint32_t ip0) {
    std::vector<Raw> out;
    std::map<uint32_t, std::vector<uint32_t>> seen;  // inst -> assertion sets walked
    std::vector<Raw> stack{{ip0, 0, -1}};
    while (!stack.empty()) {
      Raw f = stack.back();
      stack.pop_back();
      while (true) {
        auto &sv = seen[f.ip];
        bool covered = false;
        for (uint32_t c : sv)
          if ((c & ~f.cond) == 0) { covered = true; break; }  // walked with fewer assertions
        if (covered) break;
        sv.push_back(f.cond);
        const Inst &in = p.insts[f.ip];
        if (in.op == OP_SPLIT) {
          stack.push_back({in.y, f.cond, f.saves});
          f.ip = in.x;
        } else if (in.op == OP_SAVE) {
          snodes.push_back({(uint16_t)in.y, f.saves});
          f.saves = (int32_t)snodes.size() - 1;
          f.ip = in.x;
        } else if (in.op == OP_EMPTY) {
          f.cond |= 1u << in.look;
          f.ip = in.x;
        } else {
          out.push_back(f);
          break;
        }
      }
    }
    return out;
  }

  void build_closure(uint32_t ip0) {
    snodes.clear();
    auto raw = walk(ip0);
    std::vector<NfaEntry> ents;
    std::map<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>> by_leaf;  // leaf -> (cond, index)
    for (auto &pc : raw) {
      uint32_t leaf = leaf_id(pc.ip);
      uint32_t cond = pc.cond;
      auto &prev = by_leaf[leaf];
      bool dominated = false;
      for (auto &q : prev)
        if ((q.first & ~cond) == 0) { dominated = true; break; }
      if (dominated) continue;
      uint32_t prev_idx = prev.empty() ? 0 : prev.back().second + 1;
      prev.push_back({cond, (uint32_t)ents.size()});
      ents.push_back({leaf, (cond & 0xFF) | (prev_idx << 8)});
      t.looks_used |= cond;
      for (int32_t n = pc.saves; n >= 0; n = snodes[n].second) t.save_slot.push_back(snodes[n].first);
      t.save_off.push_back((uint32_t)t.save_slot.size());
    }
    t.entries.insert(t.entries.end(), ents.begin(), ents.end());
    if (ents.size() > t.max_closure) t.max_closure = ents.size();
  }
};

}  // namespace

bool build_nfa_tables(const Program &prog, NfaTables *out, std::string *err) {
  NfaTables t;
  Builder b(prog, t);
  t.root = b.closure_id(prog.start);
  t.cl_off.push_back(0);
  t.save_off.push_back(0);
  // Closures are built in id order; building one may create new ids.
  for (size_t k = 0; k < b.pending.size(); ++k) {
    b.build_closure(b.pending[k]);
    t.cl_off.push_back((uint32_t)t.entries.size());
    if (t.entries.size() > (1u << 24) || t.leaves.size() > (1u << 24)) {
      if (err) *err = "NFA closure tables too large";
      return false;
    }
  }
  t.nmatch = (uint32_t)prog.matches.size();
  t.anchored_start = prog.anchored_start;
  t.unicode_wb = (t.looks_used & ((1u << LOOK_WORD_BOUNDARY) | (1u << LOOK_NOT_WORD_BOUNDARY))) != 0;
  *out = std::move(t);
  return true;
}

}  // namespace rure_amd
