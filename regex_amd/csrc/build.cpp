// Host side of a regex / set (src/exec.rs:273-327 construction): the
// automata restated from the reference (host/*.cpp) are materialised, packed
// into the kernels' table images and uploaded once per device.
#include "runtime.hpp"
#include "host/byte_freq.h"

namespace rt {


// 1 + the start state when all start flags a search can present (dfa.rs:
// 1415-1464: text start / empty text / line start / word before / word
// after, in the index layout of fwd_flag_index) map to one state — always
// so without look-around assertions; 0 otherwise.
uint32_t uniform_start(const DenseDfa &d) {
  int found = -1;
  for (int st = 0; st < 2; ++st)
    for (int en = 0; en < 2; ++en)
      for (int nl = 0; nl < 2; ++nl)
        for (int wl = 0; wl < 2; ++wl)
          for (int wn = 0; wn < 2; ++wn) {
            if (st && (wl || !nl)) continue;  // no byte before the text start
            if (nl && wl) continue;           // '\n' is not a word byte
            if (en && (wn || !st)) continue;  // empty text: no byte after, start == end
            const int idx = (st ? 1 : 0) | (en ? 2 : 0) | (nl ? 4 : 0) | (en ? 8 : 0) | (wl != wn ? 16 : 32) |
                            (wl ? 64 : 0);
            const int v = (int)d.start[idx];
            if (found < 0) found = v;
            else if (found != v) return 0;
          }
  return found < 0 ? 0 : (uint32_t)found + 1;
}

// Multi-byte fast table over the ASCII-hot sub-DFA (states [0, A)): bytes
// are grouped into K local classes (identical columns over the hot states,
// non-hot targets folded into the sentinel A); if K^stride is small the
// table maps (state, class_1..class_stride) -> next state in one lookup.
void build_stride_image(const DenseDfa &d, PackedFwd *p) {
  const int A = std::min(std::min(d.n_ascii, d.n_normal), 255);
  p->stride = 1;
  if (A <= 0) return;
  std::vector<int> cls(256, -1);
  std::vector<int> rep;
  std::map<std::vector<uint16_t>, int> seen;
  for (int b = 0; b < 256; ++b) {
    std::vector<uint16_t> col(A);
    for (int s = 0; s < A; ++s) {
      uint32_t t = d.trans[(size_t)s * 256 + b];
      col[s] = (uint16_t)(t < (uint32_t)A ? t : A);
    }
    auto it = seen.find(col);
    if (it == seen.end()) { it = seen.emplace(col, (int)rep.size()).first; rep.push_back(b); }
    cls[b] = it->second;
  }
  const int K = (int)rep.size();
  int stride = 1;
  const long budget = (16384 - 1024) / 2;  // u16 entries after the 1 KiB class tables
  if (K <= 4 && (long)(A + 1) * K * K * K * K <= budget) stride = 4;
  else if (K <= 16 && (long)(A + 1) * K * K <= budget) stride = 2;
  if (stride == 1) return;
  uint32_t P = 1;
  for (int i = 0; i < stride; ++i) P *= (uint32_t)K;
  std::vector<uint8_t> img(1024, 0);
  for (int pos = 0; pos < stride; ++pos) {
    uint32_t mul = 1;
    for (int i = pos + 1; i < stride; ++i) mul *= (uint32_t)K;
    for (int b = 0; b < 256; ++b) img[pos * 256 + b] = (uint8_t)(cls[b] * mul);
  }
  const size_t nent = (size_t)(A + 1) * P;
  std::vector<uint16_t> tab(nent);
  for (int s = 0; s <= A; ++s) {
    for (uint32_t combo = 0; combo < P; ++combo) {
      uint32_t t = (uint32_t)s;
      uint32_t c = combo, div = P / (uint32_t)K;
      for (int pos = 0; pos < stride; ++pos) {
        int k = (int)(c / div);
        c %= div;
        if (div > 1) div /= (uint32_t)K;
        if (t < (uint32_t)A) {
          uint32_t nx = d.trans[(size_t)t * 256 + rep[k]];
          t = nx < (uint32_t)A ? nx : (uint32_t)A;
        }
      }
      tab[(size_t)s * P + combo] = (uint16_t)(t * P);
    }
  }
  img.resize(1024 + nent * 2);
  memcpy(img.data() + 1024, tab.data(), nent * 2);
  img.resize((img.size() + 15) & ~(size_t)15, 0);
  p->lds_s = std::move(img);
  p->stride = (uint32_t)stride;
  p->hot_s = (uint32_t)A;
  p->P = P;
  p->sent = (uint32_t)A * P;
}

bool pack_forward(const DenseDfa &d, PackedFwd *p, std::string *err, bool all) {
  if (d.nstates > 65535) {
    if (err) *err = "DFA has too many states for u16 tables";
    return false;
  }
  p->ustart1 = uniform_start(d);
  if (all && d.nstates <= 255) {
    // small automata (find_iter / reverse scans): every state's exact row in
    // LDS, so match, dead and restart steps never touch the global table
    p->all = 1;
    p->hot = (uint32_t)d.nstates;
    p->lds.assign(((size_t)d.nstates * kRow + 15) & ~(size_t)15, 0);
    for (int st = 0; st < d.nstates; ++st)
      for (int b = 0; b < 256; ++b) p->lds[(size_t)st * kRow + b] = (uint8_t)d.trans[(size_t)st * 256 + b];
    p->full.resize((size_t)d.nstates * 256);
    for (size_t i = 0; i < p->full.size(); ++i) p->full[i] = (uint16_t)d.trans[i];
    p->eof.assign(d.eof_match.begin(), d.eof_match.end());
    p->start.resize(128);
    for (int i = 0; i < 128; ++i) p->start[i] = (uint16_t)d.start[i];
    return true;
  }
  // LDS fast table: the normal states reachable through ASCII bytes are
  // numbered first; hold them plus further BFS-order states in the smallest
  // of three table sizes (4 KiB / 16 KiB / 64 KiB) that fits the ASCII set,
  // so that several workgroups stay resident per CU.
  int need = std::min(d.n_ascii, d.n_normal);
  int cap = need + 1 <= 16 ? 15 : need + 1 <= 64 ? 63 : 255;
  uint32_t hot = (uint32_t)std::min(d.n_normal, cap);
  p->hot = hot;
  size_t lds_bytes = ((size_t)(hot + 1) * kRow + 15) & ~(size_t)15;
  p->lds.assign(lds_bytes, 0);
  for (uint32_t s = 0; s <= hot; ++s) {
    for (int b = 0; b < 256; ++b) {
      uint32_t t = (s < hot) ? d.trans[(size_t)s * 256 + b] : hot;
      p->lds[(size_t)s * kRow + b] = (uint8_t)(t < hot ? t : hot);
    }
    // column 256 (row padding): the identity, for the bytes outside a masked
    // head / tail block of the line kernel (dfa_line_kernel)
    p->lds[(size_t)s * kRow + kIdCol] = (uint8_t)s;
  }
  build_stride_image(d, p);
  p->full.resize((size_t)d.nstates * 256);
  for (size_t i = 0; i < p->full.size(); ++i) p->full[i] = (uint16_t)d.trans[i];
  p->eof.assign(d.eof_match.begin(), d.eof_match.end());
  p->eof_mask.assign(d.eof_mask.begin(), d.eof_mask.end());
  p->now_mask.assign(d.now_mask.begin(), d.now_mask.end());
  p->start.resize(128);
  for (int i = 0; i < 128; ++i) p->start[i] = (uint16_t)d.start[i];
  return true;
}


// LDS budget of the core table (RURE_AMD_CORE_LDS overrides, tuning).
size_t core_lds_budget() {
  size_t b = 150 * 1024;
  if (knob(Knob::CoreLds) > 0) b = std::max<size_t>(4096, std::min<size_t>(150 * 1024, knob(Knob::CoreLds)));
  return b;
}

// weights (optional, by core in first-appearance numbering): rank the cores
// by decreasing weight (measured visits), ties in BFS order.
// mask_weights: how often each reported mask occurred on a sample (the
// profile of adapt_cores); the 62 most frequent masks get the LDS codes.
// Without it, masks rank by the number of hot transitions reporting them.
bool build_set_cores(const DenseDfa &d, size_t lds_budget, CoreSet *cs,
                     const std::vector<uint64_t> *weights,
                     const std::unordered_map<uint64_t, uint64_t> *mask_weights,
                     const std::vector<uint64_t> *state_weights) {
  const int S = d.nstates;
  std::unordered_map<std::string, uint32_t> key_core;
  std::vector<uint32_t> core_of(S);
  std::vector<int> rep;
  for (int s = 0; s < S; ++s) {
    std::string k((const char *)&d.trans[(size_t)s * 256], 256 * 4);
    k.append((const char *)&d.eof_mask[s], 8);
    auto it = key_core.emplace(k, (uint32_t)rep.size());
    if (it.second) rep.push_back(s);
    core_of[s] = it.first->second;
  }
  const uint32_t nc = (uint32_t)rep.size();
  if (nc >= 65535) return false;
  // BFS order over ASCII bytes from the start cores, then everything else
  std::vector<int32_t> rank(nc, -1);
  std::vector<uint32_t> order;
  std::deque<uint32_t> dq;
  auto push = [&](uint32_t c) { if (rank[c] < 0) { rank[c] = (int32_t)order.size(); order.push_back(c); dq.push_back(c); } };
  for (int i = 0; i < 128; ++i) push(core_of[d.start[i]]);
  while (!dq.empty()) {
    uint32_t c = dq.front(); dq.pop_front();
    for (int b = 0; b < 128; ++b) push(core_of[d.trans[(size_t)rep[c] * 256 + b]]);
  }
  for (uint32_t c = 0; c < nc; ++c) push(c);
  std::vector<uint64_t> sw;
  if (!weights && state_weights) {  // per-state visit counts summed per core
    sw.assign(nc, 0);
    for (int s2 = 0; s2 < S; ++s2) sw[core_of[s2]] += (*state_weights)[s2];
    weights = &sw;
  }
  if (weights) {
    std::vector<uint32_t> bfs = order;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b2) { return (*weights)[a] > (*weights)[b2]; });
    for (uint32_t r = 0; r < nc; ++r) rank[order[r]] = (int32_t)r;
    (void)bfs;
  }
  // byte classes: identical (next core, output) columns over all cores
  std::unordered_map<std::string, uint32_t> col_id;
  uint8_t cls[256];
  std::vector<int> col_rep;
  for (int b = 0; b < 256; ++b) {
    std::string k;
    k.reserve(nc * 12);
    for (uint32_t r = 0; r < nc; ++r) {
      const uint32_t nxt = d.trans[(size_t)rep[order[r]] * 256 + b];
      const uint32_t ncore = (uint32_t)rank[core_of[nxt]];
      k.append((const char *)&ncore, 4);
      k.append((const char *)&d.now_mask[nxt], 8);
    }
    auto it = col_id.emplace(k, (uint32_t)col_rep.size());
    if (it.second) col_rep.push_back(b);
    if (it.first->second > 255) return false;
    cls[b] = (uint8_t)it.first->second;
  }
  const uint32_t K = (uint32_t)col_rep.size();
  if (K > 127) return false;  // the kernel's LDS class map holds 2k in a byte
  if (lds_budget < 256 + 64 * 8 + 16 + 4 * (K + 1)) return false;
  // LDS rows have K + 1 entries: column K is the identity (same core, no
  // output), the class of the bytes outside a masked head / tail chunk
  const uint32_t KL = K + 1;
  // (the image: class map, (hot + 1) rows, the 64 code masks)
  uint32_t hot = (uint32_t)std::min<size_t>({(size_t)nc, 1023, (lds_budget - 256 - 64 * 8 - 16) / (2 * KL) - 1});
  cs->hot_visits = 0;
  if (weights)
    for (uint32_t r = 0; r < hot; ++r) cs->hot_visits += (*weights)[order[r]];
  cs->K = K;
  cs->ncores = nc;
  cs->hot = hot;
  cs->gcore.assign((size_t)nc * K, 0);
  cs->gout.assign((size_t)nc * K, 0);
  cs->eof.assign(nc, 0);
  cs->mid.assign((size_t)nc * K, 0);
  cs->masks.clear();
  std::unordered_map<uint64_t, uint32_t> mask_idx;
  std::unordered_map<uint64_t, uint64_t> hot_uses;
  for (uint32_t r = 0; r < nc; ++r) {
    const int s = rep[order[r]];
    cs->eof[r] = d.eof_mask[s];
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t nxt = d.trans[(size_t)s * 256 + col_rep[k]];
      const uint64_t out = d.now_mask[nxt];
      cs->gcore[(size_t)r * K + k] = (uint16_t)rank[core_of[nxt]];
      cs->gout[(size_t)r * K + k] = out;
      if (!out) continue;
      auto it = mask_idx.emplace(out, (uint32_t)cs->masks.size());
      if (it.second) cs->masks.push_back(out);
      if (cs->masks.size() >= 65535) return false;
      cs->mid[(size_t)r * K + k] = (uint16_t)(it.first->second + 1);
      if (r < hot) ++hot_uses[out];
    }
  }
  // output codes 1..62 for the most frequent masks (measured when profiled)
  std::vector<uint64_t> ranked = cs->masks;
  auto weight = [&](uint64_t m) -> uint64_t {
    if (mask_weights) {
      auto it = mask_weights->find(m);
      return it == mask_weights->end() ? 0 : it->second;
    }
    auto it = hot_uses.find(m);
    return it == hot_uses.end() ? 0 : it->second;
  };
  std::stable_sort(ranked.begin(), ranked.end(), [&](uint64_t a, uint64_t b2) { return weight(a) > weight(b2); });
  std::unordered_map<uint64_t, uint32_t> code_of;
  memset(cs->codemask, 0, sizeof(cs->codemask));
  for (uint32_t i = 0; i < ranked.size() && i < 62; ++i) {
    code_of[ranked[i]] = i + 1;
    cs->codemask[i + 1] = ranked[i];
  }
  const size_t t_end = 256 + (size_t)(hot + 1) * KL * 2;
  cs->mt_off = (uint32_t)((t_end + 7) & ~(size_t)7);
  cs->lds.assign(cs->mt_off + 64 * 8, 0);
  memcpy(cs->lds.data(), cls, 256);
  memcpy(cs->lds.data() + cs->mt_off, cs->codemask, 64 * 8);
  uint16_t *T = (uint16_t *)(cs->lds.data() + 256);
  for (uint32_t r = 0; r < hot; ++r) {
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t ncore = cs->gcore[(size_t)r * K + k];
      const uint64_t out = cs->gout[(size_t)r * K + k];
      uint32_t code = 0;
      if (out) {
        auto it = code_of.find(out);
        code = it == code_of.end() ? 63 : it->second;
      }
      const uint32_t tgt = ncore < hot ? ncore : hot;
      T[(size_t)r * KL + k] = (uint16_t)((tgt << 6) | (ncore < hot ? code : 0));
    }
    T[(size_t)r * KL + K] = (uint16_t)(r << 6);  // identity column
  }
  for (uint32_t k = 0; k < KL; ++k) T[(size_t)hot * KL + k] = (uint16_t)(hot << 6);  // sentinel row
  for (int i = 0; i < 128; ++i) cs->start[i] = (uint16_t)rank[core_of[d.start[i]]];
  cs->dead = (uint32_t)rank[core_of[d.dead]];
  cs->quit = d.quit >= 0 ? (uint32_t)rank[core_of[d.quit]] : 0xFFFFFFFFu;
  cs->lds.resize((cs->lds.size() + 15) & ~(size_t)15, 0);
  cs->order = order;
  cs->ok = true;
  return true;
}


SyntaxFlags syntax_flags(uint32_t flags) {  // rure.rs:119-124
  SyntaxFlags f;
  f.casei = (flags & RURE_FLAG_CASEI) != 0;
  f.multi = (flags & RURE_FLAG_MULTI) != 0;
  f.dotnl = (flags & RURE_FLAG_DOTNL) != 0;
  f.swap_greed = (flags & RURE_FLAG_SWAP_GREED) != 0;
  f.ignore_space = (flags & RURE_FLAG_SPACE) != 0;
  f.unicode = (flags & RURE_FLAG_UNICODE) != 0;
  f.allow_bytes = true;  // bytes::RegexBuilder (re_builder.rs:171, exec.rs:225)
  return f;
}

// Builds the automata of a regex once: the DFAs (when they materialise
// within budget) and always the Pike VM closure tables.  Returns whether a
// search engine is available.
// Automata past the u16 tables (more than 65535 states): both directions in
// column form with the larger raw-state budget, for the big_dfa.hip kernels.
// Programs with a Unicode word boundary (quit states) keep the Pike VM, and
// so does a search the reference runs as DfaAnchoredReverse.
void build_big_dfas(rure *re) {
  re->big_ok = false;
  if (!re->nfa_ok) return;
  if (re->fwd.has_unicode_word_boundary || re->rev.has_unicode_word_boundary) return;
  if (!re->nfa.anchored_start && re->nfa.anchored_end) return;
  DfaBuildLimits lim;
  lim.max_raw_states = kBigDfaRawStates;
  lim.max_bytes = kBigDfaBytes;
  if (knob(Knob::BigBytes) > 0) lim.max_bytes = (size_t)knob(Knob::BigBytes);
  lim.columns = true;
  lim.minimise = false;   // construction already shares step targets; refinement doubled the build time
  std::string e1, e2;
  bool rok = false;
  std::thread rt([&] { rok = build_dense_dfa(re->rev, lim, &re->brev, &e2); });
  const bool fok = build_dense_dfa(re->fwd, lim, &re->bfwd, &e1);
  rt.join();
  if (!fok || !rok || re->bfwd.quit >= 0 || re->brev.quit >= 0) {
    re->bfwd = DenseDfa();
    re->brev = DenseDfa();
    return;
  }
  re->big_ok = true;
}

bool build_regex(rure *re) {
  std::lock_guard<std::mutex> g(re->mu);
  if (re->built) return re->dfa_ok || re->nfa_ok;
  re->built = true;
  std::string nerr;
  re->nfa_ok = build_nfa_tables(re->nfa, &re->nt, &nerr);
  DfaBuildLimits lim;
  std::string err, rerr;
  // the forward and reverse automata are independent: build them on two threads
  bool rev_ok = false;
  std::thread rt([&] { rev_ok = build_dense_dfa(re->rev, lim, &re->drev, &rerr); });
  const bool fwd_ok = build_dense_dfa(re->fwd, lim, &re->dfwd, &err);
  rt.join();
  re->rev_ok = rev_ok;
  if (fwd_ok && !rev_ok) err = rerr;
  if (!fwd_ok || !rev_ok || !pack_forward(re->dfwd, &re->pf, &err) || !pack_forward(re->drev, &re->pr, &err, true)) {
    re->dfa_err = err.empty() ? "reverse DFA too large" : err;
    re->dfa_ok = false;   // the big automata are built on first need (big_device)
    if (!re->nfa_ok) re->dfa_err += "; " + nerr;
    return re->nfa_ok;
  }
  re->dfa_ok = true;
  return true;
}

bool build_regex_dfas(rure *re) {
  build_regex(re);
  return re->dfa_ok;
}

bool build_set(rure_set *rs) {
  std::lock_guard<std::mutex> g(rs->mu);
  if (rs->built) return rs->dfa_ok || rs->nfa_ok;
  rs->built = true;
  if (rs->exprs.empty()) { rs->dfa_ok = true; return true; }
  std::string nerr;
  rs->nfa_ok = build_nfa_tables(rs->nfa, &rs->nt, &nerr);
  if (!rs->groups.empty()) {  // searched group by group; no combined DFA
    rs->dfa_err = "set of more than 64 patterns: automata are built per 64-pattern group";
    return rs->nfa_ok;
  }
  DfaBuildLimits lim;
  std::string err;
  if (!build_dense_dfa(rs->fwd, lim, &rs->dfa, &err) || !pack_forward(rs->dfa, &rs->pf, &err)) {
    rs->dfa_err = err;
    rs->dfa_ok = false;
    if (!rs->nfa_ok) rs->dfa_err += "; " + nerr;
    return rs->nfa_ok;
  }
  // Large sets: the byte-row hot table holds at most 255 states; switch to
  // the core form when more normal or match-reporting states than that exist.
  if (rs->dfa.n_normal > 255 || rs->dfa.n_match_end - rs->dfa.n_normal > 255)
    build_set_cores(rs->dfa, core_lds_budget(), &rs->cores);
  rs->dfa_ok = true;
  return true;
}

bool build_set_dfa(rure_set *rs) {
  build_set(rs);
  return rs->dfa_ok;
}

// Appends the Pike VM tables to an upload blob; fix_nfa() then points the
// descriptor into the device copy.

NfaOffsets add_nfa(Blob &b, const NfaTables &nt) {
  NfaOffsets o;
  std::vector<uint32_t> lv(nt.leaves.size() * 3);
  for (size_t i = 0; i < nt.leaves.size(); ++i) {
    const NfaLeaf &l = nt.leaves[i];
    lv[3 * i] = (uint32_t)l.kind | ((uint32_t)l.lo << 8) | ((uint32_t)l.hi << 16);
    lv[3 * i + 1] = l.closure;
    lv[3 * i + 2] = l.slot;
  }
  o.leaves = b.add(lv.data(), lv.size() * 4);
  o.cl_off = b.add(nt.cl_off.data(), nt.cl_off.size() * 4);
  o.entries = b.add(nt.entries.data(), nt.entries.size() * 8);
  namespace U = rure_amd_unicode;
  o.perlw = b.add(U::kPairs + 2 * U::kPerlW.first, (size_t)U::kPerlW.count * 8);
  o.save_off = b.add(nt.save_off.data(), nt.save_off.size() * 4);
  o.save_slot = b.add(nt.save_slot.data(), nt.save_slot.size() * 2);
  // per closure (NfaDev::cl_info, 9 words): the bytes its Bytes leaves take
  // (256 bits), then the looks every entry requires | 0x100 if it holds a
  // Match leaf -- append_closure skips a closure none of whose entries can
  // pass (the Pike VM's root closure at a position inside a word of \bfox\b)
  const size_t ncl = nt.cl_off.empty() ? 0 : nt.cl_off.size() - 1;
  std::vector<uint32_t> ci(ncl * 9, 0);
  for (size_t c = 0; c < ncl; ++c) {
    uint32_t need = 0xFF, match = 0;
    for (uint32_t k = nt.cl_off[c]; k < nt.cl_off[c + 1]; ++k) {
      const NfaEntry &e = nt.entries[k];
      need &= e.cond_prev & 0xFF;
      const NfaLeaf &l = nt.leaves[e.leaf];
      if (l.kind == 0) {
        for (uint32_t x = l.lo; x <= l.hi; ++x) ci[c * 9 + (x >> 5)] |= 1u << (x & 31);
      } else {
        match = 0x100;
      }
    }
    if (nt.cl_off[c] == nt.cl_off[c + 1]) need = 0;
    ci[c * 9 + 8] = need | match;
  }
  o.cl_info = b.add(ci.data(), ci.size() * 4);
  // Closures of more than 64 entries, bucketed by the next byte
  // (NfaDev::cl_big / cl_boff / cl_sub): bucket x (256 = the end of the
  // text) holds, in order, the entries whose leaf is a Match or takes x, with
  // their same-leaf links renumbered -- append_closure then scans the few
  // entries that can pass instead of all (the loop closure of Unicode \w+
  // holds every alternative of the class).
  std::vector<uint32_t> big(ncl, 0xFFFFFFFFu), boff;
  std::vector<NfaEntry> sub;
  for (size_t c = 0; c < ncl; ++c) {
    const uint32_t k0 = nt.cl_off[c], k1 = nt.cl_off[c + 1];
    if (k1 - k0 <= 64) continue;
    // (bounded: a closure of wide leaves -- `.` takes every byte -- would
    // copy each entry into hundreds of buckets)
    size_t want = 0;
    for (uint32_t k = k0; k < k1; ++k) {
      const NfaLeaf &l = nt.leaves[nt.entries[k].leaf];
      want += l.kind == 0 ? (size_t)l.hi - l.lo + 1 : 257;
    }
    if (want > 16 * (size_t)(k1 - k0) || sub.size() + want > (1u << 22)) continue;
    big[c] = (uint32_t)(boff.size() / 258);
    for (uint32_t x = 0; x <= 256; ++x) {
      boff.push_back((uint32_t)sub.size());
      const size_t base = sub.size();
      for (uint32_t k = k0; k < k1; ++k) {
        const NfaEntry &e = nt.entries[k];
        const NfaLeaf &l = nt.leaves[e.leaf];
        if (l.kind == 0 && (x > 255 || x < l.lo || x > l.hi)) continue;
        uint32_t prev = 0;
        for (size_t q = sub.size(); q > base; --q)
          if (sub[q - 1].leaf == e.leaf) { prev = (uint32_t)(q - base); break; }
        sub.push_back(NfaEntry{e.leaf, (e.cond_prev & 0xFF) | (prev << 8)});
      }
    }
    boff.push_back((uint32_t)sub.size());
  }
  o.cl_big = b.add(big.data(), big.size() * 4);
  o.cl_boff = boff.empty() ? o.cl_big : b.add(boff.data(), boff.size() * 4);
  o.cl_sub = sub.empty() ? o.cl_big : b.add(sub.data(), sub.size() * 8);
  return o;
}

void fix_nfa(NfaDev *n, uint8_t *base, const NfaOffsets &o, const NfaTables &nt, bool single) {
  n->leaves = (const uint32_t *)(base + o.leaves);
  n->cl_off = (const uint32_t *)(base + o.cl_off);
  n->entries = (const uint2 *)(base + o.entries);
  n->perlw = (const uint32_t *)(base + o.perlw);
  n->perlw_n = rure_amd_unicode::kPerlW.count;
  n->save_off = (const uint32_t *)(base + o.save_off);
  n->save_slot = (const uint16_t *)(base + o.save_slot);
  n->cl_info = (const uint32_t *)(base + o.cl_info);
  n->cl_big = (const uint32_t *)(base + o.cl_big);
  n->cl_boff = (const uint32_t *)(base + o.cl_boff);
  n->cl_sub = (const uint2 *)(base + o.cl_sub);
  n->nleaves = (uint32_t)nt.leaves.size();
  n->root = nt.root;
  n->nmatch = nt.nmatch;
  n->anchored = nt.anchored_start ? 1 : 0;
  n->single = single ? 1 : 0;
  n->looks = nt.looks_used;
  n->unicode_wb = nt.unicode_wb ? 1 : 0;
  n->ncl_off = (uint32_t)nt.cl_off.size();
  n->nentries = (uint32_t)nt.entries.size();
}

bool upload_blob(const Blob &b, DevTables *t, std::string *err) {
  if (!hip_ok(hipMalloc(&t->blob, b.bytes.size()), err)) return false;
  if (!hip_ok(hipMemcpy(t->blob, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice), err)) {
    (void)hipFree(t->blob);
    t->blob = nullptr;
    return false;
  }
  return true;
}

// A literal list (bytes, n + 1 u32 offsets) into an upload blob.
LitOffsets add_litlist(Blob &b, const Literals &l) {
  std::string cat;
  std::vector<uint32_t> off{0};
  for (const Lit &x : l.lits) {
    cat += x.v;
    off.push_back((uint32_t)cat.size());
  }
  cat.resize(cat.size() + 16, 0);
  LitOffsets o;
  o.bytes = b.add(cat.data(), cat.size());
  o.off = b.add(off.data(), off.size() * 4);
  o.n = (uint32_t)l.lits.size();
  return o;
}

// Whether the reference's match type makes this regex's searches differ from
// a forward DFA search (DevTables::mt_lane).
bool needs_mt_lane(const ExecLiterals &x) {
  return x.match_type == MT_DFA_SUFFIX || x.match_type == MT_LITERAL_ANCHORED_START ||
         (x.match_type == MT_LITERAL_UNANCHORED && !x.prefixes.complete);
}

// FwdDfaDev::pfx_*: the start-state prefix skip (dfa.rs:700-711), for a
// DFA whose start does not depend on look-behind, from the regex's prefix
// literals (dfa.prefixes, exec.rs:308-311; not for anchored starts,
// dfa.rs:1516-1522 has_prefix) when they have at most 4 first bytes.
// FwdDfaDev::rare_*: the same skip on the prefixes' rarest byte or pair of
// bytes at most 3 apart (host/byte_freq.h), where they have more than one
// first byte.  Knob prefix: 0 off, 1 first byte only, 2 rare bytes only.
// (A filter over the prefixes' first two or three positions lost to the
// first-byte one on English text in round 4 — Sherlock\s+\w+ 1.47 -> 1.62
// ms per GiB, (?i)watson\w* 1.46 -> 1.89, profiles/r04_prefix_depth_ab.jsonl
// — and was deleted in round 5.)
void set_prefix_skip(const rure *re, FwdDfaDev *f) {
  f->pfx_n = 0;
  f->rare_on = 0;
  const long long mode = knob(Knob::Prefix);
  if (mode == 0 || !f->ustart1 || re->nfa.anchored_start) return;
  const LitSearcher &p = re->xl.prefixes;
  if (p.matcher == 0 || p.lits.lits.empty()) return;
  bool seen[256] = {false};
  uint32_t n = 0;
  bool first_ok = true;
  for (const Lit &l : p.lits.lits) {
    if (l.v.empty()) return;
    const uint8_t b = (uint8_t)l.v[0];
    if (seen[b]) continue;
    if (n == 4) { first_ok = false; break; }
    seen[b] = true;
    f->pfx_rep[n++] = b * 0x01010101u;
  }
  if (!first_ok) n = 0;
  // the byte class of every prefix at position j, as one entry (x | or ==
  // rep: one byte, or an ASCII letter's two cases), and its frequency
  size_t minlen = ~(size_t)0;
  for (const Lit &l : p.lits.lits) minlen = std::min(minlen, l.v.size());
  const size_t J = std::min<size_t>(minlen, 16);
  std::vector<int> rep(J, -1), orm(J, 0);
  std::vector<uint64_t> fr(J, 0);
  for (size_t j = 0; j < J; ++j) {
    bool in[256] = {false};
    for (const Lit &l : p.lits.lits) in[(uint8_t)l.v[j]] = true;
    int c = 0, x0 = -1;
    for (int x = 0; x < 256; ++x)
      if (in[x]) ++c, x0 = x0 < 0 ? x : x0;
    const bool letter = (x0 | 0x20) >= 'a' && (x0 | 0x20) <= 'z';
    if (c == 1) {
      rep[j] = x0, orm[j] = 0, fr[j] = kByteFreq[x0];
    } else if (c == 2 && letter && in[x0 ^ 0x20]) {
      rep[j] = x0 | 0x20, orm[j] = 0x20, fr[j] = kByteFreq[x0] + kByteFreq[x0 ^ 0x20];
    }
  }
  // the rarest single byte class or pair (i1, i1 + d), d <= 3, i1 + d <= 15
  // (a pair's frequency: the product, as if independent)
  double best = 1e30;
  int bi = -1, bd = 0;
  for (size_t i = 0; i < J; ++i) {
    if (rep[i] < 0) continue;
    if ((double)fr[i] < best) best = (double)fr[i], bi = (int)i, bd = 0;
    for (int d = 1; d <= 3 && i + d < J && i + d <= 15; ++d) {
      if (rep[i + d] < 0) continue;
      const double pf = (double)fr[i] * (double)fr[i + d] / (double)(1u << 20);
      if (pf < best) best = pf, bi = (int)i, bd = d;
    }
  }
  // Which, by measurement (tools/prefix_ab.py, profiles/r05_prefix_ab.jsonl,
  // 1 GiB of sherlock, long scan): one first byte wins where there is one
  // (Sherlock\s+\w+ 1.55 ms against 1.73 for the rare pair, >[^\n]*\n 0.31
  // against 0.39: a single-byte SWAR test per word is cheaper, and English
  // pairs are not independent: "l..k" of Sherlock is in "look"); the rare
  // skip where the first bytes are several ((?i)holmes\w* 1.41 -> 1.14 ms,
  // (?i)watson\w* 1.68 -> 1.61, (?i)zqxj\w* 1.11 -> 0.54; (?i)baker\s+street
  // loses, 1.48 -> 1.56: "b.k" of "back", "book").
  // ... and the rare skip only where the byte it keys on is rare by the
  // reference's own ranking (freqs.rs: rank <= 150 — q, j, z, most capitals,
  // control and high bytes), the way FreqyPacked picks a byte for memchr
  // (literals.rs:390-510): on English text a pair of common letters is in
  // most 128-byte bursts whatever the product of their frequencies says
  // (r06 A/B: (?i)moriarty's "mo" cost 58 %, (?i)baker's "ba" 15 %), and a
  // burst that holds a candidate is tested and then stepped anyway
  auto cls_rank = [&](int j) {
    return orm[j] ? std::max(kByteRank[rep[j]], kByteRank[rep[j] ^ 0x20]) : kByteRank[rep[j]];
  };
  const bool rare_byte = bi >= 0 && std::min(cls_rank(bi), cls_rank(bi + bd)) <= 150;
  const bool rare_ok = bi >= 0 && mode != 1 && (mode == 2 || rare_byte);
  const bool first_use = n > 0 && mode != 2;
  if (rare_ok && (mode == 2 || !(first_use && n == 1))) {
    f->rare_on = 1;
    f->rare_d = (uint32_t)bd;
    f->rare_rep[0] = (uint32_t)rep[bi] * 0x01010101u;
    f->rare_or[0] = (uint32_t)orm[bi] * 0x01010101u;
    f->rare_rep[1] = (uint32_t)rep[bi + bd] * 0x01010101u;
    f->rare_or[1] = (uint32_t)orm[bi + bd] * 0x01010101u;
    return;
  }
  f->pfx_n = first_use ? n : 0;
}

// Upload (once per device) and return device descriptors.
DevTables *regex_device(rure *re, std::string *err) {
  if (!build_regex(re)) { if (err) *err = re->dfa_err; return nullptr; }
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  std::lock_guard<std::mutex> g(re->mu);
  auto it = re->dev.find(d);
  if (it != re->dev.end()) return &it->second;
  Blob b;
  DevTables t;
  t.cus = device_cus(d);
  NfaOffsets no{};
  if (re->nfa_ok) no = add_nfa(b, re->nt);
  size_t o_lds = 0, o_lds_s = 0, o_full = 0, o_eof = 0, o_start = 0, o_rfull = 0, o_reof = 0, o_rstart = 0,
         o_rlds = 0;
  const PackedFwd &pf = re->pf;
  const DenseDfa &rv = re->drev;
  if (re->dfa_ok) {
    std::vector<uint16_t> rfull(rv.trans.size()), rstart(128);
    for (size_t i = 0; i < rv.trans.size(); ++i) rfull[i] = (uint16_t)rv.trans[i];
    for (int i = 0; i < 128; ++i) rstart[i] = (uint16_t)rv.start[i];
    o_lds = b.add(pf.lds.data(), pf.lds.size());
    o_lds_s = b.add(pf.lds_s.data(), pf.lds_s.size());
    o_full = b.add(pf.full.data(), pf.full.size() * 2);
    o_eof = b.add(pf.eof.data(), pf.eof.size());
    o_start = b.add(pf.start.data(), 256);
    o_rfull = b.add(rfull.data(), rfull.size() * 2);
    o_reof = b.add(rv.eof_match.data(), rv.eof_match.size());
    o_rstart = b.add(rstart.data(), 256);
    o_rlds = b.add(re->pr.lds.data(), re->pr.lds.size());
  }
  const bool mt_lane = needs_mt_lane(re->xl);
  LitOffsets lp{}, ls{};
  size_t o_lcs = 0;
  if (mt_lane) {
    lp = add_litlist(b, re->xl.prefixes.lits);
    ls = add_litlist(b, re->xl.suffixes.lits);
    std::string lcs = re->xl.suffixes.lcs;
    lcs.resize(lcs.size() + 16, 0);
    o_lcs = b.add(lcs.data(), lcs.size());
  }
  if (!upload_blob(b, &t, err)) return nullptr;
  uint8_t *base = (uint8_t *)t.blob;
  if (re->nfa_ok) fix_nfa(&t.n, base, no, re->nt, true);
  if (mt_lane) {
    t.mt_lane = true;
    t.m.mt = re->xl.match_type;
    t.m.pre = LitListDev{base + lp.bytes, (const uint32_t *)(base + lp.off), lp.n, re->xl.prefixes.matcher};
    t.m.suf = LitListDev{base + ls.bytes, (const uint32_t *)(base + ls.off), ls.n, re->xl.suffixes.matcher};
    t.m.lcs = base + o_lcs;
    t.m.lcs_len = (uint32_t)re->xl.suffixes.lcs.size();
    // no proper prefix of the lcs is also its suffix: its occurrences never
    // overlap, so the greedy walk of exec.rs:736-741 visits every occurrence
    const std::string &l = re->xl.suffixes.lcs;
    bool border = false;
    for (size_t k = 1; k < l.size() && !border; ++k) border = l.compare(0, k, l, l.size() - k, k) == 0;
    t.lcs_free = !l.empty() && !border;
  }
  if (re->dfa_ok) {
    const DenseDfa &fw = re->dfwd;
    t.has_dfa = true;
    t.quit_possible = fw.quit >= 0 || rv.quit >= 0;
    t.f.lds_image = base + o_lds;
    t.f.lds_bytes = (uint32_t)pf.lds.size();
    t.f.hot = pf.hot;
    t.f.lds_image_s = base + o_lds_s;
    t.f.lds_bytes_s = (uint32_t)pf.lds_s.size();
    t.f.stride = pf.stride;
    t.f.hot_s = pf.hot_s;
    t.f.P = pf.P;
    t.f.sent = pf.sent;
    t.f.cus = (uint32_t)t.cus;
    t.f.full = (const uint16_t *)(base + o_full);
    t.f.eof = base + o_eof;
    t.f.start = (const uint16_t *)(base + o_start);
    t.f.n_normal = fw.n_normal;
    t.f.n_match_end = fw.n_match_end;
    t.f.dead = fw.dead;
    t.f.quit = fw.quit < 0 ? 0xFFFFFFFFu : (uint32_t)fw.quit;
    t.r.lds_image = base + o_rlds;
    t.r.lds_bytes = (uint32_t)re->pr.lds.size();
    t.r.hot = re->pr.hot;
    t.r.full = (const uint16_t *)(base + o_rfull);
    t.r.eof = base + o_reof;
    t.r.start = (const uint16_t *)(base + o_rstart);
    t.r.n_normal = rv.n_normal;
    t.r.n_match_end = rv.n_match_end;
    t.r.dead = rv.dead;
    t.r.quit = rv.quit < 0 ? 0xFFFFFFFFu : (uint32_t)rv.quit;
    t.r.all = re->pr.all;
    t.r.ustart1 = re->pr.ustart1;
    t.f.ustart1 = pf.ustart1;
    t.f.nonempty = can_match_empty(re->nfa) ? 0 : 1;
    set_prefix_skip(re, &t.f);
    // a regex anchored at the end and not at the start runs the reverse DFA
    // from the end of the text (exec.rs:1175-1177, 671-688)
    t.anchored_rev = !re->nfa.anchored_start && re->nfa.anchored_end;
  }
  t.owner = re;
  if (t.quit_possible && !re->nfa_ok) {
    (void)hipFree(t.blob);
    if (err) *err = "the DFA can quit and the NFA tables could not be built";
    return nullptr;
  }
  return &(re->dev[d] = t);
}

// Automata past the u16 tables, built and uploaded on the first batch that
// would run them (big_batch): their construction can take seconds and
// hundreds of MB of host memory (bounded by kBigDfaBytes), which a regex
// searched on the Pike VM only (few long haystacks) never needs.  Returns
// whether t now has them.
bool big_device(const DevTables &tc) {
  DevTables &t = const_cast<DevTables &>(tc);  // the regex's own entry of rure::dev
  rure *re = t.owner;
  if (!re) return false;
  std::lock_guard<std::mutex> g(re->mu);
  if (t.big_tried) return t.has_big;
  t.big_tried = true;
  if (!re->big_built) {
    re->big_built = true;
    build_big_dfas(re);
  }
  if (!re->big_ok) return false;
  Blob b;
  size_t o_big[8];
  const DenseDfa *bd[2] = {&re->bfwd, &re->brev};
  for (int k = 0; k < 2; ++k) {
    o_big[4 * k] = b.add(bd[k]->ctrans.data(), bd[k]->ctrans.size() * 4);
    o_big[4 * k + 1] = b.add(bd[k]->colmap, 256);
    o_big[4 * k + 2] = b.add(bd[k]->eof_match.data(), bd[k]->eof_match.size());
    o_big[4 * k + 3] = b.add(bd[k]->start, 128 * 4);
  }
  DevTables tmp;
  std::string err;
  if (!upload_blob(b, &tmp, &err)) return false;
  uint8_t *base = (uint8_t *)tmp.blob;
  BigDfaDev *dst[2] = {&t.bf, &t.br};
  for (int k = 0; k < 2; ++k) {
    const DenseDfa &D = *bd[k];
    BigDfaDev &x = *dst[k];
    x.trans = (const uint32_t *)(base + o_big[4 * k]);
    x.colmap = base + o_big[4 * k + 1];
    x.eof = base + o_big[4 * k + 2];
    x.start = (const uint32_t *)(base + o_big[4 * k + 3]);
    x.ncol = D.ncol;
    x.nstates = (uint32_t)D.nstates;
    x.hot = k == 0 ? big_dfa_hot_rows(D.ncol, (uint32_t)D.nstates) : 0;
    x.n_normal = (uint32_t)D.n_normal;
    x.n_match_end = (uint32_t)D.n_match_end;
    x.dead = (uint32_t)D.dead;
    x.ustart1 = uniform_start(D);
  }
  t.big_blob = tmp.blob;
  t.has_big = true;
  return true;
}

// The on-demand forward DFA (host LazyDfa, big_dfa.hip lazy_dfa_kernel) for
// automata past the eager budgets: built on the first batch that needs it.
// Its reverse partner is the regular u16 reverse DFA (t.r, or drev packed
// and uploaded here when the forward DFA did not materialise).  Programs
// with a Unicode word boundary keep the Pike VM, as for the big automata.
bool lazy_device(const DevTables &tc) {
  DevTables &t = const_cast<DevTables &>(tc);
  rure *re = t.owner;
  if (!re) return false;
  std::lock_guard<std::mutex> g(re->mu);
  if (t.lazy_tried) return t.has_lazy;
  t.lazy_tried = true;
  if (!re->nfa_ok || re->fwd.has_unicode_word_boundary || re->rev.has_unicode_word_boundary) return false;
  if (!re->nfa.anchored_start && re->nfa.anchored_end) return false;  // DfaAnchoredReverse
  if (t.has_dfa) {
    t.lr = t.r;
  } else {
    if (!re->rev_ok || re->drev.quit >= 0) return false;
    std::string e;
    if (re->pr.full.empty() && !pack_forward(re->drev, &re->pr, &e, true)) return false;
    const DenseDfa &rv = re->drev;
    std::vector<uint16_t> rfull(rv.trans.size()), rstart(128);
    for (size_t i = 0; i < rv.trans.size(); ++i) rfull[i] = (uint16_t)rv.trans[i];
    for (int i = 0; i < 128; ++i) rstart[i] = (uint16_t)rv.start[i];
    Blob bl;
    const size_t o_full = bl.add(rfull.data(), rfull.size() * 2), o_eof = bl.add(rv.eof_match.data(), rv.eof_match.size()),
                 o_start = bl.add(rstart.data(), 256);
    DevTables tmp;
    if (!upload_blob(bl, &tmp, &e)) return false;
    uint8_t *base = (uint8_t *)tmp.blob;
    t.lazy_rblob = tmp.blob;
    RevDfaDev &r = t.lr;
    r = RevDfaDev{};
    r.full = (const uint16_t *)(base + o_full);
    r.eof = base + o_eof;
    r.start = (const uint16_t *)(base + o_start);
    r.n_normal = rv.n_normal;
    r.n_match_end = rv.n_match_end;
    r.dead = rv.dead;
    r.quit = 0xFFFFFFFFu;
    r.ustart1 = re->pr.ustart1;
  }
  if (!re->lazy) {
    size_t budget = kBigDfaBytes;
    if (knob(Knob::BigBytes) > 0) budget = (size_t)knob(Knob::BigBytes);
    re->lazy.reset(new LazyDfa(re->fwd, budget));
  }
  t.has_lazy = true;
  return true;
}

DevTables *set_device(rure_set *rs, std::string *err) {
  if (!build_set(rs)) { if (err) *err = rs->dfa_err; return nullptr; }
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  std::lock_guard<std::mutex> g(rs->mu);
  auto it = rs->dev.find(d);
  if (it != rs->dev.end()) return &it->second;
  const PackedFwd &pf = rs->pf;
  Blob b;
  DevTables t;
  t.cus = device_cus(d);
  NfaOffsets no{};
  if (rs->nfa_ok) no = add_nfa(b, rs->nt);
  size_t o_lds = 0, o_full = 0, o_mask = 0, o_now = 0, o_start = 0;
  size_t c_lds = 0, c_core = 0, c_out = 0, c_eof = 0, c_start = 0;
  const CoreSet &cs = rs->cores;
  if (rs->dfa_ok && cs.ok) {
    c_lds = b.add(cs.lds.data(), cs.lds.size());
    c_core = b.add(cs.gcore.data(), cs.gcore.size() * 2);
    c_out = b.add(cs.gout.data(), cs.gout.size() * 8);
    c_eof = b.add(cs.eof.data(), cs.eof.size() * 8);
    c_start = b.add(cs.start, 256);
  }
  if (rs->dfa_ok) {
    o_lds = b.add(pf.lds.data(), pf.lds.size());
    o_full = b.add(pf.full.data(), pf.full.size() * 2);
    o_mask = b.add(pf.eof_mask.data(), pf.eof_mask.size() * 8);
    o_now = b.add(pf.now_mask.data(), pf.now_mask.size() * 8);
    o_start = b.add(pf.start.data(), 256);
  }
  if (!upload_blob(b, &t, err)) return nullptr;
  uint8_t *base = (uint8_t *)t.blob;
  // set programs: several Match instructions, no leftmost-first cut (pikevm.rs:196-212)
  if (rs->nfa_ok) fix_nfa(&t.n, base, no, rs->nt, rs->nt.nmatch <= 1);
  if (rs->dfa_ok) {
    const DenseDfa &fw = rs->dfa;
    t.has_dfa = true;
    t.quit_possible = fw.quit >= 0;
    t.s.lds_image = base + o_lds;
    t.s.lds_bytes = (uint32_t)pf.lds.size();
    t.s.hot = pf.hot;
    t.s.full = (const uint16_t *)(base + o_full);
    t.s.eof_mask = (const uint64_t *)(base + o_mask);
    t.s.now_mask = (const uint64_t *)(base + o_now);
    t.s.all = rs->exprs.size() >= 64 ? ~0ull : ((1ull << rs->exprs.size()) - 1);
    t.s.start = (const uint16_t *)(base + o_start);
    t.s.n_normal = fw.n_normal;
    t.s.n_match_end = fw.n_match_end;
    t.s.dead = fw.dead;
    t.s.quit = fw.quit < 0 ? 0xFFFFFFFFu : (uint32_t)fw.quit;
    if (cs.ok) {
      t.use_cores = true;
      t.c.lds_image = base + c_lds;
      t.c.lds_bytes = (uint32_t)cs.lds.size();
      t.c.hot = cs.hot;
      t.c.K = cs.K;
      t.c.gcore = (const uint16_t *)(base + c_core);
      t.c.gout = (const uint64_t *)(base + c_out);
      t.c.eof = (const uint64_t *)(base + c_eof);
      t.c.start = (const uint16_t *)(base + c_start);
      t.c.all = t.s.all;
      t.c.dead = cs.dead;
      t.c.quit = cs.quit;
      t.c.mt_off = cs.mt_off;
    }
  }
  if (t.quit_possible && !rs->nfa_ok) {
    (void)hipFree(t.blob);
    if (err) *err = "the DFA can quit and the NFA tables could not be built";
    return nullptr;
  }
  return &(rs->dev[d] = t);
}


// The first-byte start rule of FwdDfaDev::fb_n, decided on the find_iter DFA
// (with strip states, no look-around, flag-independent start).  F = the
// ASCII bytes on which the anchored start state strip[start] does not die
// (every match starts with a byte on which it does not die).  Every state
// reachable from it through F and then ASCII bytes, before a match-flag state
// is entered, must have no ASCII transition to `dead` or `quit`: an anchored
// run from an F byte over ASCII text then cannot fail except by reaching the
// end of the text.  So in a forward search (`.*?` prefix, leftmost-first)
// from p over ASCII text, the thread started at the first c >= p with text[c]
// in F stays alive until it has matched, the DFA reaches `dead` before the
// end only after that, and the match it reports starts at c (threads from
// earlier starts have priority, dfa.rs:910-1048).  The kernel applies the
// rule to a search only when every byte it loaded was ASCII (Unicode classes
// such as `[^\n]` die on invalid UTF-8).  Returns |F| (1..4) or 0.
uint32_t first_byte_rule(const DenseDfa &d, uint32_t ustart1, bool nonempty, uint8_t bytes[4], bool *holds) {
  *holds = false;
  if (!ustart1 || !nonempty || d.strip.empty()) return 0;
  const uint32_t a0 = d.strip[ustart1 - 1];
  if ((int)a0 >= d.n_normal) return 0;
  // (a quit state is allowed only on bytes >= 0x80: the ASCII shadow)
  auto fails = [&](uint32_t t) { return (int)t == d.dead || (int)t == d.quit; };
  uint32_t nf = 0;
  std::vector<uint32_t> todo;
  std::vector<uint8_t> seen(d.nstates, 0);
  for (int c = 0; c < 128; ++c) {
    const uint32_t t = d.trans[(size_t)a0 * 256 + c];
    if ((int)t == d.dead) continue;
    if ((int)t == d.quit) return 0;
    if (nf < 4) bytes[nf] = (uint8_t)c;
    ++nf;
    if ((int)t < d.n_normal && !seen[t]) { seen[t] = 1; todo.push_back(t); }
  }
  while (!todo.empty()) {  // pre-match states: normal states reached before a match flag
    const uint32_t x = todo.back();
    todo.pop_back();
    for (int c = 0; c < 128; ++c) {
      const uint32_t t = d.trans[(size_t)x * 256 + c];
      if (fails(t)) return 0;
      if ((int)t < d.n_normal && !seen[t]) { seen[t] = 1; todo.push_back(t); }
    }
  }
  *holds = nf > 0;
  // the generic kernels' SWAR test holds at most four bytes (FwdDfaDev::fb_rep);
  // the lexer needs only that the rule holds
  return nf <= 4 && d.quit < 0 ? nf : 0;
}

// The run engine's class (FwdDfaDev::run_cls, run_iter.hip): true when the
// find_iter DFA's anchored automaton (strip[start], flag-independent start)
// is, over its byte columns (all 256, or ASCII: `ascii`, or an automaton
// whose bytes >= 0x80 quit — the ASCII shadow; the bytes >= 0x80 then quit
// the run engine too), the automaton of C+ for the byte class C on which it
// survives its first byte — checked state by state against the ideal
// automaton R0 -C-> R1, R1 / R2 -C-> R2 (match flag: a match ended one byte
// before), R1 / R2 -not C-> T (flagged), T -> dead, R0 -not C-> dead, with
// the one-byte-delayed match flags and dead states of dfa.rs:658-668 and
// 728-731 agreeing in every reachable pair.  Then the leftmost-first match
// of a search from p is the maximal run of C bytes starting at the first C
// byte at or after p (the first-byte rule holds: a run never dies before it
// has matched), and find_iter (re_trait.rs:197-221) yields exactly the
// maximal runs.
bool run_class(const DenseDfa &d, uint32_t ustart1, bool nonempty, uint8_t cls[256], bool ascii) {
  if (!ustart1 || !nonempty || d.strip.empty()) return false;
  const int NC = ascii || d.quit >= 0 ? 128 : 256;
  const uint32_t a0 = d.strip[ustart1 - 1];
  if ((int)a0 >= d.n_normal) return false;
  bool in_c[256] = {false};
  int nc = 0;
  for (int c = 0; c < NC; ++c) {
    const uint32_t t = d.trans[(size_t)a0 * 256 + c];
    if ((int)t == d.quit) return false;
    in_c[c] = (int)t != d.dead;
    nc += in_c[c];
  }
  if (!nc) return false;
  auto flagged = [&](uint32_t t) { return (int)t >= d.n_normal && (int)t < d.n_match_end; };
  // ideal states: 0 = R0, 1 = R1, 2 = R2 (flagged), 3 = T (flagged), 4 = dead
  auto ideal = [](int r, bool c) { return r == 0 ? (c ? 1 : 4) : (r == 1 || r == 2) ? (c ? 2 : 3) : 4; };
  std::vector<uint8_t> seen((size_t)d.nstates * 5, 0);
  std::vector<std::pair<uint32_t, int>> todo{{a0, 0}};
  seen[(size_t)a0 * 5] = 1;
  while (!todo.empty()) {
    const auto [x, r] = todo.back();
    todo.pop_back();
    for (int c = 0; c < NC; ++c) {
      const uint32_t t = d.trans[(size_t)x * 256 + c];
      const int r2 = ideal(r, in_c[c]);
      if ((int)t == d.quit) return false;
      const bool dd = (int)t == d.dead;
      if (dd != (r2 == 4)) return false;
      if (dd) continue;
      if (flagged(t) != (r2 == 2 || r2 == 3)) return false;
      if (!seen[(size_t)t * 5 + r2]) {
        seen[(size_t)t * 5 + r2] = 1;
        todo.push_back({t, r2});
      }
    }
  }
  for (int c = 0; c < 256; ++c) cls[c] = c < NC ? (in_c[c] ? 1 : 0) : 2;
  return true;
}

// The code points of a regex that is one Unicode class repeated, greedy and
// unbounded (C+: \w+, \pL+, \S+, [^\n]+ in Unicode mode), read off the
// syntax tree (groups around the class or the repetition only bound
// captures, which find_iter does not report).  Its program matches exactly
// the valid UTF-8 encodings of C's code points one or more times
// (compile.rs:386-396 c_class over utf8 ranges), so its leftmost-first
// matches are the maximal runs of such encodings: run_iter.hip decodes the
// bytes >= 0x80 against the bitmap.
static const Expr *unwrap(const Expr *e) {  // groups, one-element sequences
  while ((e->kind == EK::Group || e->kind == EK::Concat || e->kind == EK::Alternate) && e->subs.size() == 1)
    e = &e->subs[0];
  return e;
}

static bool unicode_run_set(const Expr &e0, std::vector<CRange> *out) {
  const Expr *e = unwrap(&e0);
  if (e->kind != EK::Repeat || !e->greedy || e->subs.size() != 1) return false;
  if (!(e->rep == Rep::OneOrMore || (e->rep == Rep::Range && e->rmin == 1 && !e->has_max))) return false;
  const Expr *c = unwrap(&e->subs[0]);
  if (c->kind == EK::AnyChar) *out = {{0, 0x10FFFF}};
  else if (c->kind == EK::AnyCharNoNL) *out = {{0, 9}, {11, 0x10FFFF}};
  else if (c->kind == EK::Class && !c->cls.empty()) *out = c->cls;
  else return false;
  return true;
}

// Whether every match of the regex is exactly one byte of a class (read off
// the syntax tree: one byte literal, a byte class, or a Unicode class of
// ASCII code points; a case-insensitive literal is left out, its Unicode
// folds can be multi-byte): then its find_iter is the positions of those
// bytes and replace_all needs no match list (launch_replace_class).
bool class_one_set(const Expr &e0, uint8_t cls[256]) {
  const Expr *e = unwrap(&e0);
  std::memset(cls, 0, 256);
  switch (e->kind) {
    case EK::LiteralBytes:
      if (e->bytes.size() != 1 || e->casei) return false;
      cls[e->bytes[0]] = 1;
      return true;
    case EK::Literal:
      if (e->chars.size() != 1 || e->casei || e->chars[0] >= 0x80) return false;
      cls[e->chars[0]] = 1;
      return true;
    case EK::ClassBytes:
      if (e->bcls.empty()) return false;
      for (const BRange &r : e->bcls)
        for (uint32_t b = r.lo; b <= r.hi; ++b) cls[b] = 1;
      return true;
    case EK::Class:
      if (e->cls.empty()) return false;
      for (const CRange &r : e->cls)
        if (r.hi >= 0x80) return false;
      for (const CRange &r : e->cls)
        for (uint32_t b = r.lo; b <= r.hi; ++b) cls[b] = 1;
      return true;
    case EK::AnyByte:
      std::memset(cls, 1, 256);
      return true;
    case EK::AnyByteNoNL:
      std::memset(cls, 1, 256);
      cls['\n'] = 0;
      return true;
    default:
      return false;
  }
}

// The lexer table of FwdDfaDev::lex_image (iter_spec_lex_tile_kernel).
// Needs the first-byte start rule (a match's start is the first F byte of its
// search on ASCII text) and terminal match states: every state carrying the
// (one-byte delayed) match flag has only dead transitions, so entering one at
// byte x ends the search with the match [start, x), and the iteration's next
// search begins at x with the start state S0 (re_trait.rs:197-221; the regex
// is nonempty).  The table composes the two: the transition into a match
// state on byte b becomes S0's transition on b into a *twin* of its target
// (same row; entering a twin = a match ended here).  u8 state numbers, rows
// of kRow bytes (the forward kernels' LDS layout), numbered [other states,
// S0, twin(S0), other twins] so that one clamp of the state number gives the
// byte's flags (FwdDfaDev::lex_z).  Returns false if the rule does not hold
// or the states do not fit u8.
bool build_lex(const DenseDfa &d, uint32_t ustart1, bool fb_holds, std::vector<uint8_t> *img,
                      uint32_t *s0_idx) {
  img->clear();
  if (!fb_holds || !ustart1) return false;
  // An automaton that quits (the ASCII shadow: bytes >= 0x80 quit) is read
  // on ASCII columns only: the kernel leaves any block holding a byte >= 0x80
  // to the tail pass, so its other columns are never stepped.
  const int NC = d.quit >= 0 ? 128 : 256;
  const uint32_t s0 = ustart1 - 1;
  for (int m = d.n_normal; m < d.n_match_end; ++m)
    for (int c = 0; c < NC; ++c)
      if ((int)d.trans[(size_t)m * 256 + c] != d.dead) return false;
  auto is_match = [&](uint32_t t) { return (int)t >= d.n_normal && (int)t < d.n_match_end; };
  // states reachable from S0 (match transitions replaced by restarts)
  std::vector<uint8_t> reach(d.nstates, 0);
  std::vector<uint32_t> todo{s0};
  reach[s0] = 1;
  while (!todo.empty()) {
    const uint32_t q = todo.back();
    todo.pop_back();
    for (int c = 0; c < NC; ++c) {
      uint32_t t = d.trans[(size_t)q * 256 + c];
      if (is_match(t)) t = d.trans[(size_t)s0 * 256 + c];
      if (is_match(t)) return false;  // S0 itself matching on one byte: an empty match
      if (!reach[t]) { reach[t] = 1; todo.push_back(t); }
    }
  }
  std::vector<int> plain(d.nstates, -1), twin(d.nstates, -1);
  std::vector<uint32_t> rows;  // DFA state of each lexer row
  for (int q = 0; q < d.nstates; ++q)
    if (reach[q] && (uint32_t)q != s0) { plain[q] = (int)rows.size(); rows.push_back(q); }
  plain[s0] = (int)rows.size();
  rows.push_back(s0);
  twin[s0] = (int)rows.size();
  rows.push_back(s0);
  for (int c = 0; c < NC; ++c) {
    const uint32_t t = d.trans[(size_t)s0 * 256 + c];
    if (twin[t] < 0) { twin[t] = (int)rows.size(); rows.push_back(t); }
  }
  if (rows.size() > kLexMaxRows || plain[s0] < 1) return false;
  // entries 4 row + code (dfa_scan.hpp FwdDfaDev::lex_image): codes 0 for the
  // rows below S0, 1 for S0, 2 for twin(S0), 3 for the other twins
  const uint32_t ps0 = (uint32_t)plain[s0];
  auto code = [&](uint32_t r) -> uint32_t { return r < ps0 ? 0 : r == ps0 ? 1 : r == ps0 + 1 ? 2 : 3; };
  auto entry = [&](uint32_t r) -> uint8_t { return (uint8_t)(4 * r + code(r)); };
  img->assign(((rows.size() - 1) * kRow + 3 * kLexUnit + 256 + 15) & ~(size_t)15, 0);
  for (size_t i = 0; i < rows.size(); ++i)
    for (int c = 0; c < 256; ++c) {
      if (c >= NC) {  // never stepped: S0
        (*img)[(size_t)entry((uint32_t)i) * kLexUnit + c] = entry(ps0);
        continue;
      }
      const uint32_t t = d.trans[(size_t)rows[i] * 256 + c];
      const int to = is_match(t) ? twin[d.trans[(size_t)s0 * 256 + c]] : plain[t];
      (*img)[(size_t)entry((uint32_t)i) * kLexUnit + c] = entry((uint32_t)to);
    }
  *s0_idx = entry(ps0);
  return true;
}

// The lexer four bytes per step (FwdDfaDev::lex4_image): the byte table's
// entries reachable from S0 over ASCII become rows (at most kLex4Rows), the
// ASCII bytes fall into at most 3 classes (bytes with equal columns in every
// row), and a row's entry for four classes is the byte table walked over one
// byte of each; class 3 walks nothing (flags 0), so a partial word's tail
// leaves the state alone as lex16<false> does.  Bytes >= 0x80 never reach
// the lexer (their blocks are the tail pass's).  Returns false when the
// table does not fit.
bool build_lex4(const std::vector<uint8_t> &img, uint32_t s0, std::vector<uint8_t> *out, uint32_t *s0_row) {
  out->clear();
  if (img.empty()) return false;
  auto at = [&](uint32_t e, uint32_t c) -> uint32_t {
    const size_t i = (size_t)e * kLexUnit + c;
    return i < img.size() ? img[i] : 0;
  };
  std::vector<uint32_t> rows{s0};
  std::vector<int> row_of(256, -1);
  row_of[s0] = 0;
  for (size_t i = 0; i < rows.size(); ++i)
    for (uint32_t c = 0; c < 128; ++c) {
      const uint32_t t = at(rows[i], c);
      if (row_of[t] < 0) {
        if (rows.size() == kLex4Rows) return false;
        row_of[t] = (int)rows.size();
        rows.push_back(t);
      }
    }
  uint8_t cls[256] = {0};
  std::vector<uint32_t> rep;  // a byte of each class
  for (uint32_t c = 0; c < 128; ++c) {
    int k = -1;
    for (size_t j = 0; j < rep.size() && k < 0; ++j) {
      bool same = true;
      for (uint32_t e : rows) same = same && at(e, c) == at(e, rep[j]);
      if (same) k = (int)j;
    }
    if (k < 0) {
      if (rep.size() == 3) return false;
      k = (int)rep.size();
      rep.push_back(c);
    }
    cls[c] = (uint8_t)k;
  }
  out->assign(kLex4Bytes, 0);
  for (size_t r = 0; r < rows.size(); ++r)
    for (uint32_t c = 0; c < 256; ++c) {
      uint32_t e = rows[r], fl = 0;
      for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t ck = (c >> (2 * k)) & 3;
        if (ck == 3 || ck >= rep.size()) continue;
        e = at(e, rep[ck]);
        fl |= (e & 3) << (2 * k);
      }
      (*out)[r * 256 + c] = (uint8_t)row_of[e];
      (*out)[kLex4Flags + r * 256 + c] = (uint8_t)fl;
    }
  for (uint32_t j = 0; j < 4; ++j)
    for (uint32_t c = 0; c < 256; ++c) (*out)[kLex4Cls + 256 * j + c] = (uint8_t)(cls[c] << (2 * j));
  *s0_row = 0;
  return true;
}

bool build_iter_dfa(rure *re) {
  if (!build_regex_dfas(re)) return false;
  std::lock_guard<std::mutex> g(re->mu);
  if (!re->iter_built) {
    re->iter_built = true;
    DfaBuildLimits lim;
    lim.strip = true;
    std::string e;
    re->iter_ok = build_dense_dfa(re->fwd, lim, &re->dfwd_iter, &e) && pack_forward(re->dfwd_iter, &re->pf_iter, &e, true);
    if (!re->lits_done) re->lit_ok = extract_literals(re->nfa, kLitMax, kLitLen, &re->lits);
    re->lits_done = true;
    bool fb_holds = false;
    if (re->iter_ok)
      re->fb_n = first_byte_rule(re->dfwd_iter, re->pf_iter.ustart1, !can_match_empty(re->nfa), re->fb_bytes,
                                 &fb_holds);
    // (the lexer of the full automaton keeps the rule's original bound of four
    // first bytes: wider F are served by the ASCII shadow's lexer below)
    if (re->iter_ok && fb_holds && build_lex(re->dfwd_iter, re->pf_iter.ustart1, fb_holds, &re->lex, &re->lex_s0))
      build_lex4(re->lex, re->lex_s0, &re->lex4, &re->lex4_s0);
    // (over all bytes, else over ASCII text: Unicode \S+, \d+, [^\n]+)
    const bool ne = !can_match_empty(re->nfa);
    // (a Unicode class: its code point bitmap, preferred to the ASCII-only
    // table whose bytes >= 0x80 quit)
    std::vector<CRange> ucls;
    re->run_cp.clear();
    const bool run_base = re->iter_ok && !re->nt.looks_used && re->dfwd_iter.quit < 0;
    re->run_ok = run_base && run_class(re->dfwd_iter, re->pf_iter.ustart1, ne, re->run_cls, false);
    if (run_base && !re->run_ok && unicode_run_set(re->expr, &ucls)) {
      re->run_cp.assign(0x110000 / 32, 0);
      for (const CRange &r : ucls)
        for (uint32_t c = r.lo; c <= r.hi && c < 0x110000; ++c) re->run_cp[c >> 5] |= 1u << (c & 31);
      for (int c = 0; c < 256; ++c) re->run_cls[c] = c < 0x80 ? (re->run_cp[c >> 5] >> (c & 31)) & 1u : 4;
      re->run_ok = true;
    }
    if (run_base && !re->run_ok)
      re->run_ok = run_class(re->dfwd_iter, re->pf_iter.ustart1, ne, re->run_cls, true);
    // ASCII shadow (iter_ascii_device): where the automaton is too big for
    // the all-rows LDS table because of its UTF-8 states (Unicode classes),
    // the same automaton with every byte >= 0x80 quitting and the states only
    // those bytes reach dropped
    if (re->iter_ok && !re->pf_iter.all && !re->fwd.has_unicode_word_boundary && !re->lit_ok &&
        knob(Knob::AsciiShadow) != 0) {
      DfaBuildLimits la;
      la.strip = true;
      la.ascii_only = true;
      DenseDfa a;
      PackedFwd pa;
      if (build_dense_dfa(re->fwd, la, &a, &e)) {
        prune_unreachable(&a);
        if (a.nstates <= 255 && pack_forward(a, &pa, &e, true) && pa.all) {
          re->dfwd_iter_a = std::move(a);
          re->pf_iter_a = std::move(pa);
          re->iter_a_ok = true;
          // its lexer (dense find_iter without reverse scans: \w+, \S+,
          // \pL+ over ASCII text): the first-byte rule for any number of
          // first bytes, terminal match states; not with look-around
          bool holds = false;
          uint8_t fbb[4];
          (void)first_byte_rule(re->dfwd_iter_a, re->pf_iter_a.ustart1, !can_match_empty(re->nfa), fbb, &holds);
          if (holds && !re->nt.looks_used &&
              build_lex(re->dfwd_iter_a, re->pf_iter_a.ustart1, true, &re->lex_a, &re->lex_a_s0))
            build_lex4(re->lex_a, re->lex_a_s0, &re->lex4_a, &re->lex4_a_s0);
          re->run_a_ok = !re->nt.looks_used && !re->run_ok &&
                         run_class(re->dfwd_iter_a, re->pf_iter_a.ustart1, !can_match_empty(re->nfa), re->run_cls_a,
                                   true);
        }
      }
    }
  }
  return re->iter_ok;
}


// Forward DFA with stripped states for the chunked find_iter (built and
// uploaded on first use).  Returns null if it does not materialise.
// The Shift-And image of a string set whose strings all have one length L
// (iter_spec_sa_kernel): strings equal but in one position are merged into
// class sequences (the union of that position's classes; the same language),
// until no pair merges; sequence x owns bits [x L, (x + 1) L) of the state.
// mask[b] bit i = byte b is in the class of bit position i.  Returns false
// (and leaves the outputs empty) unless the sequences fit 64 bits.
bool build_shiftand(const LiteralSet &ls, std::vector<uint64_t> *mask, uint64_t *init, uint64_t *fin,
                           uint32_t *len, uint32_t *bits) {
  mask->clear();
  *init = *fin = 0;
  *len = *bits = 0;
  if (ls.lits.empty() || ls.minlen != ls.maxlen || ls.minlen < 1) return false;
  const size_t L = ls.minlen;
  using Cls = std::array<uint64_t, 4>;
  std::vector<std::vector<Cls>> seqs;
  for (const std::string &l : ls.lits) {
    std::vector<Cls> q(L, Cls{0, 0, 0, 0});
    for (size_t i = 0; i < L; ++i) q[i][(uint8_t)l[i] >> 6] |= 1ull << ((uint8_t)l[i] & 63);
    seqs.push_back(q);
  }
  for (bool merged = true; merged;) {
    merged = false;
    for (size_t x = 0; x < seqs.size() && !merged; ++x)
      for (size_t y = x + 1; y < seqs.size() && !merged; ++y) {
        int diff = -1, nd = 0;
        for (size_t i = 0; i < L && nd < 2; ++i)
          if (seqs[x][i] != seqs[y][i]) { diff = (int)i; ++nd; }
        if (nd == 1) {
          for (int w = 0; w < 4; ++w) seqs[x][diff][w] |= seqs[y][diff][w];
          seqs.erase(seqs.begin() + y);
          merged = true;
        }
      }
  }
  if (seqs.size() * L > 64) return false;
  *len = (uint32_t)L;
  *bits = (uint32_t)(seqs.size() * L);
  mask->assign(256, 0);
  for (size_t x = 0; x < seqs.size(); ++x) {
    *init |= 1ull << (x * L);
    *fin |= 1ull << (x * L + L - 1);
    for (size_t i = 0; i < L; ++i)
      for (int c = 0; c < 256; ++c)
        if ((seqs[x][i][c >> 6] >> (c & 63)) & 1) (*mask)[c] |= 1ull << (x * L + i);
  }
  return true;
}

// The ASCII shadow of the find_iter DFA on this device (null if none): DFA
// tables and its lexer (no string engines), can_quit set.
const FwdDfaDev *iter_ascii_device(rure *re, const DevTables &t, std::string *err) {
  if (!build_iter_dfa(re) || !re->iter_a_ok) return nullptr;
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  std::lock_guard<std::mutex> g(re->mu);
  auto it = re->iter_dev_a.find(d);
  if (it != re->iter_dev_a.end()) return &it->second.second;
  const PackedFwd &pf = re->pf_iter_a;
  const DenseDfa &fw = re->dfwd_iter_a;
  std::vector<uint16_t> strip(fw.strip.size());
  for (size_t i = 0; i < strip.size(); ++i) strip[i] = (uint16_t)fw.strip[i];
  Blob b;
  size_t o_lds = b.add(pf.lds.data(), pf.lds.size());
  size_t o_full = b.add(pf.full.data(), pf.full.size() * 2);
  size_t o_eof = b.add(pf.eof.data(), pf.eof.size());
  size_t o_start = b.add(pf.start.data(), 256);
  size_t o_strip = b.add(strip.data(), strip.size() * 2);
  size_t o_run = re->run_a_ok ? b.add(re->run_cls_a, 256) : 0;
  size_t o_lex = re->lex_a.empty() ? 0 : b.add(re->lex_a.data(), re->lex_a.size());
  size_t o_lex4 = re->lex4_a.empty() ? 0 : b.add(re->lex4_a.data(), re->lex4_a.size());
  DevTables tmp;
  if (!upload_blob(b, &tmp, err)) return nullptr;
  uint8_t *base = (uint8_t *)tmp.blob;
  FwdDfaDev f{};
  f.lds_image = base + o_lds;
  f.lds_bytes = (uint32_t)pf.lds.size();
  f.hot = pf.hot;
  f.stride = 1;
  f.cus = (uint32_t)t.cus;
  if (re->run_a_ok) {
    f.run_cls = base + o_run;
    f.run_quit = 1;
  }
  if (!re->lex_a.empty()) {  // the lexer over ASCII blocks (build_iter_dfa)
    f.lex_image = base + o_lex;
    f.lex_bytes = (uint32_t)re->lex_a.size();
    f.lex_s0 = re->lex_a_s0;
  }
  if (!re->lex4_a.empty() && knob(Knob::Lex4) != 0) {
    f.lex4_image = base + o_lex4;
    f.lex4_s0 = re->lex4_a_s0;
  }
  f.full = (const uint16_t *)(base + o_full);
  f.eof = base + o_eof;
  f.start = (const uint16_t *)(base + o_start);
  f.strip = (const uint16_t *)(base + o_strip);
  f.n_normal = fw.n_normal;
  f.n_match_end = fw.n_match_end;
  f.dead = fw.dead;
  f.quit = fw.quit < 0 ? 0xFFFFFFFFu : (uint32_t)fw.quit;
  f.all = pf.all;
  f.ustart1 = pf.ustart1;
  f.nonempty = can_match_empty(re->nfa) ? 0 : 1;
  f.looks = re->nt.looks_used ? 1 : 0;
  f.can_quit = 1;
  // (no set_prefix_skip: the skip is read by the long find / is_match scan
  // only, and the shadow serves find_iter, whose burst kernel has none)
  re->iter_dev_a[d] = {tmp.blob, f};
  return &re->iter_dev_a[d].second;
}

const FwdDfaDev *iter_device(rure *re, const DevTables &t, std::string *err) {
  if (!build_iter_dfa(re)) return nullptr;
  int d = 0;
  if (!hip_ok(hipGetDevice(&d), err)) return nullptr;
  std::lock_guard<std::mutex> g(re->mu);
  auto it = re->iter_dev.find(d);
  if (it != re->iter_dev.end()) return &it->second.second;
  const PackedFwd &pf = re->pf_iter;
  const DenseDfa &fw = re->dfwd_iter;
  std::vector<uint16_t> strip(fw.strip.size());
  for (size_t i = 0; i < strip.size(); ++i) strip[i] = (uint16_t)fw.strip[i];
  Blob b;
  size_t o_lds = b.add(pf.lds.data(), pf.lds.size());
  size_t o_full = b.add(pf.full.data(), pf.full.size() * 2);
  size_t o_eof = b.add(pf.eof.data(), pf.eof.size());
  size_t o_start = b.add(pf.start.data(), 256);
  size_t o_strip = b.add(strip.data(), strip.size() * 2);
  std::vector<uint8_t> lit_img;
  uint32_t lit_k = 0;
  if (re->lit_ok) {
    // literal engine image (dfa_scan.hpp kLit*): prefix-hash bitmap, keys,
    // lengths, bytes
    lit_k = (uint32_t)std::min<size_t>(re->lits.minlen, 4);
    lit_img.assign(kLitImage, 0);
    uint32_t *bitmap = (uint32_t *)lit_img.data();
    for (size_t x = 0; x < re->lits.lits.size(); ++x) {
      const std::string &l = re->lits.lits[x];
      uint32_t key = 0;
      for (uint32_t j = 0; j < lit_k; ++j) key |= (uint32_t)(uint8_t)l[j] << (8 * j);
      const uint32_t h = lit_hash(key);
      bitmap[h >> 5] |= 1u << (h & 31);
      std::memcpy(lit_img.data() + kLitKeys + 4 * x, &key, 4);
      lit_img[kLitLens + x] = (uint8_t)l.size();
      std::memcpy(lit_img.data() + kLitBytes + kLitLen * x, l.data(), l.size());
      if (re->lits.minlen >= 8) {
        uint32_t key2 = 0;
        std::memcpy(&key2, l.data() + 4, 4);
        const uint32_t h2 = lit_hash(key2);
        ((uint32_t *)(lit_img.data() + kLitBitmap2))[h2 >> 5] |= 1u << (h2 & 31);
      }
    }
  }
  size_t o_lit = lit_img.empty() ? 0 : b.add(lit_img.data(), lit_img.size());
  // Shift-And image (build_shiftand)
  std::vector<uint64_t> sa_img;
  uint64_t sa_init = 0, sa_final = 0;
  uint32_t sa_len = 0, sa_bits = 0;
  if (re->lit_ok) build_shiftand(re->lits, &sa_img, &sa_init, &sa_final, &sa_len, &sa_bits);
  size_t o_sa = sa_img.empty() ? 0 : b.add(sa_img.data(), sa_img.size() * 8);
  size_t o_lex = re->lex.empty() ? 0 : b.add(re->lex.data(), re->lex.size());
  size_t o_lex4 = re->lex4.empty() ? 0 : b.add(re->lex4.data(), re->lex4.size());
  size_t o_run = re->run_ok ? b.add(re->run_cls, 256) : 0;
  size_t o_cp = re->run_cp.empty() ? 0 : b.add(re->run_cp.data(), re->run_cp.size() * 4);
  DevTables tmp;
  if (!upload_blob(b, &tmp, err)) return nullptr;
  uint8_t *base = (uint8_t *)tmp.blob;
  FwdDfaDev f{};
  f.lds_image = base + o_lds;
  f.lds_bytes = (uint32_t)pf.lds.size();
  f.hot = pf.hot;
  f.lds_image_s = nullptr;
  f.stride = 1;
  f.cus = (uint32_t)t.cus;
  f.full = (const uint16_t *)(base + o_full);
  f.eof = base + o_eof;
  f.start = (const uint16_t *)(base + o_start);
  f.strip = (const uint16_t *)(base + o_strip);
  f.n_normal = fw.n_normal;
  f.n_match_end = fw.n_match_end;
  f.dead = fw.dead;
  f.quit = fw.quit < 0 ? 0xFFFFFFFFu : (uint32_t)fw.quit;
  f.all = pf.all;
  f.ustart1 = pf.ustart1;
  f.nonempty = can_match_empty(re->nfa) ? 0 : 1;
  set_prefix_skip(re, &f);
  // knob fb=0 turns the first-byte start rule off (reverse scans)
  f.fb_n = knob(Knob::Fb) == 0 ? 0 : re->fb_n;
  for (uint32_t i = 0; i < 4; ++i) f.fb_rep[i] = (i < re->fb_n ? re->fb_bytes[i] : re->fb_bytes[0]) * 0x01010101u;
  if (!lit_img.empty()) {
    f.lit_image = base + o_lit;
    f.lit_bytes = kLitImage;
    f.lit_n = (uint32_t)re->lits.lits.size();
    f.lit_k = lit_k;
    f.lit_minlen = (uint32_t)re->lits.minlen;
    f.lit_maxlen = (uint32_t)re->lits.maxlen;
    f.lit_k8 = re->lits.minlen >= 8 ? 1 : 0;
  }
  if (!re->lex.empty()) {
    f.lex_image = base + o_lex;
    f.lex_bytes = (uint32_t)re->lex.size();
    f.lex_s0 = re->lex_s0;
  }
  // knob lex4=0 keeps the byte-per-step lexer (A/B)
  if (!re->lex4.empty() && knob(Knob::Lex4) != 0) {
    f.lex4_image = base + o_lex4;
    f.lex4_s0 = re->lex4_s0;
  }
  if (re->run_ok) {
    f.run_cls = base + o_run;
    f.run_cp = re->run_cp.empty() ? nullptr : (const uint32_t *)(base + o_cp);
    f.run_quit = (re->run_cls[0x80] >> 1) & 1u;  // (ASCII-only class: bytes >= 0x80 quit)
  }
  if (!sa_img.empty()) {
    f.sa_image = (const uint64_t *)(base + o_sa);
    f.sa_init = sa_init;
    f.sa_final = sa_final;
    f.sa_len = sa_len;
    f.sa_bits = sa_bits;
  }
  if (re->nt.looks_used || t.quit_possible) {
    // look-around: the chunked iteration's slice rules (iter_scan.hip); the
    // literal / Shift-And / lexer engines and the first-byte start rule read
    // no assertions and skip the reverse scan, so they are off
    f.looks = re->nt.looks_used ? 1 : 0;
    // (2: the quit is a Unicode word boundary's, dfa.rs:1487-1496 -- the
    // chunked find_iter then also hands over starts after a byte >= 0x80)
    f.can_quit = t.quit_possible ? (re->fwd.has_unicode_word_boundary ? 2 : 1) : 0;
    f.fb_n = 0;
    f.lit_image = nullptr;
    f.lit_n = 0;
    f.lex_image = nullptr;
    f.lex_bytes = 0;
    f.lex4_image = nullptr;
    f.sa_image = nullptr;
    f.sa_len = f.sa_bits = 0;
    f.run_cls = nullptr;
  }
  re->iter_dev[d] = {tmp.blob, f};
  return &re->iter_dev[d].second;
}


// First batched use of a core-form set on a device: count core visits over a
// sample of the batch, re-rank the cores so the LDS table holds the visited
// ones, and upload the re-ranked tables.  Costs one host sync, once.
bool adapt_cores(rure_set *rs, DevTables *t, const BatchDev &b, hipStream_t st, std::string *err) {
  std::lock_guard<std::mutex> g(rs->mu);
  if (t->cores_adapted) return true;
  t->cores_adapted = true;
  const CoreSet &cs = rs->cores;
  const uint64_t sample = std::min<uint64_t>(b.count, 16384);
  // visits per core and reports per mask (mask ids: cs.mid) over a sample
  unsigned int *visits = nullptr;
  uint16_t *mid = nullptr;
  const size_t nm = cs.masks.size() + 1;
  if (!hip_ok(scratch_malloc((void **)&visits, (cs.ncores + nm) * 4, st), err)) return false;
  if (!hip_ok(scratch_malloc((void **)&mid, cs.mid.size() * 2, st), err)) return false;
  std::vector<unsigned int> h(cs.ncores + nm);
  SetCoreDev pc = t->c;
  pc.mid = mid;
  bool ok = hip_ok(hipMemsetAsync(visits, 0, (cs.ncores + nm) * 4, st), err) &&
            hip_ok(hipMemcpyAsync(mid, cs.mid.data(), cs.mid.size() * 2, hipMemcpyHostToDevice, st), err) &&
            hip_ok(launch_core_profile(b, pc, sample, visits, visits + cs.ncores, st, t->cus), err) &&
            hip_ok(hipMemcpyAsync(h.data(), visits, h.size() * 4, hipMemcpyDeviceToHost, st), err) &&
            hip_ok(scratch_free(visits, st), err) && hip_ok(scratch_free(mid, st), err) &&
            hip_ok(hipStreamSynchronize(st), err);
  if (!ok) return false;
  std::vector<uint64_t> w(cs.ncores, 0);
  for (uint32_t r = 0; r < cs.ncores; ++r) w[cs.order[r]] = h[r];
  std::unordered_map<uint64_t, uint64_t> mw;
  for (size_t i = 1; i < nm; ++i) mw[cs.masks[i - 1]] = h[cs.ncores + i];
  CoreSet c2;
  if (!build_set_cores(rs->dfa, core_lds_budget(), &c2, &w, &mw)) return true;  // keep the BFS ranking
  Blob bl;
  size_t c_lds = bl.add(c2.lds.data(), c2.lds.size());
  size_t c_core = bl.add(c2.gcore.data(), c2.gcore.size() * 2);
  size_t c_out = bl.add(c2.gout.data(), c2.gout.size() * 8);
  size_t c_eof = bl.add(c2.eof.data(), c2.eof.size() * 8);
  size_t c_start = bl.add(c2.start, 256);
  DevTables tmp;
  if (!upload_blob(bl, &tmp, err)) return false;
  uint8_t *base = (uint8_t *)tmp.blob;
  SetCoreDev c = t->c;
  c.lds_image = base + c_lds;
  c.lds_bytes = (uint32_t)c2.lds.size();
  c.hot = c2.hot;
  c.K = c2.K;
  c.gcore = (const uint16_t *)(base + c_core);
  c.gout = (const uint64_t *)(base + c_out);
  c.eof = (const uint64_t *)(base + c_eof);
  c.start = (const uint16_t *)(base + c_start);
  c.dead = c2.dead;
  c.quit = c2.quit;
  c.mt_off = c2.mt_off;
  if (t->core_blob) (void)hipFree(t->core_blob);
  t->core_blob = tmp.blob;
  t->c = c;
  return true;
}

}  // namespace rt
