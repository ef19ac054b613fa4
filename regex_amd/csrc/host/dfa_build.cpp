// Eager DFA materialization + minimisation.  See dfa_build.hpp.
#include "dfa_build.hpp"
#include "knobs.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <unordered_map>

namespace rure_amd {
namespace {

struct EmptyFlags {  // dfa.rs:408-416
  bool start = false, end = false, start_line = false, end_line = false;
  bool wb = false, nwb = false;
};

enum : uint8_t { SF_MATCH = 1, SF_WORD = 2, SF_EMPTY = 4 };  // dfa.rs:1648-1672

// Ordered sparse set of instruction pointers (src/sparse.rs:15-64).
struct SparseSet {
  std::vector<uint32_t> dense, sparse;
  size_t n = 0;
  explicit SparseSet(size_t cap) : dense(cap), sparse(cap) {}
  bool contains(uint32_t v) const { uint32_t i = sparse[v]; return i < n && dense[i] == v; }
  void insert(uint32_t v) { dense[n] = v; sparse[v] = (uint32_t)n; ++n; }
  void clear() { n = 0; }
};

class Builder {
 public:
  Builder(const Program &p, const DfaBuildLimits &lim)
      : p_(p), lim_(lim), qa_(p.insts.size() + 1), qb_(p.insts.size() + 1), qc_(p.insts.size() + 1) {
    is_set_ = p.matches.size() > 1;
    strip_ = lim.strip && p.dotstar_end > 0;
    cont_ = p.is_reverse || is_set_;  // dfa.rs:1557-1559
    word_matters_ = false;
    for (const Inst &i : p.insts)
      if (i.op == OP_EMPTY && i.look >= LOOK_WORD_BOUNDARY) word_matters_ = true;
    quit_ = p.has_unicode_word_boundary || lim.ascii_only;
    stack_.reserve(p.insts.size() + 1);
    stamp_.assign(p.insts.size() + 1, 0);
  }

  // On-demand construction (LazyDfa): the start states, then rows one state
  // at a time in any order; states are raw (unminimised) ids, 0 = dead.
  void lazy_init(uint8_t *colmap, uint32_t *ncol) {
    keys_.push_back(std::string());
    keys_.push_back(std::string());
    compute_starts();
    lazy_ncls_ = p_.num_byte_classes();
    int seen = -1;
    for (int b = 0; b < 256; ++b) {
      if (p_.byte_classes[b] != seen) { seen = p_.byte_classes[b]; lazy_rep_[seen] = (uint8_t)b; }
      colmap[b] = (uint8_t)p_.byte_classes[b];
    }
    *ncol = (uint32_t)lazy_ncls_;
  }
  uint32_t lazy_states() const { return (uint32_t)keys_.size(); }
  size_t lazy_bytes() const { return key_bytes_; }
  void lazy_row(uint32_t s, uint32_t *row) {
    if (s < 2) {
      for (int c = 0; c < lazy_ncls_; ++c) row[c] = s;
      return;
    }
    const std::string key = keys_[s];  // copy: keys_ may grow
    step_row(key, lazy_ncls_, lazy_rep_, row);
  }
  bool lazy_eof(uint32_t s) {
    if (s < 2) return false;
    uint64_t m = 0;
    return step_eof(keys_[s], &m);
  }
  bool lazy_match(uint32_t s) const { return s >= 2 && (keys_[s][0] & SF_MATCH); }
  uint32_t lazy_start(int fi) const { return start_used_[fi] ? start_raw_[fi] : 0; }

  bool build(DenseDfa *out, std::string *err) {
    const auto t_begin = std::chrono::steady_clock::now();
    // raw state 0 = DEAD, raw state 1 = QUIT (always allocated, maybe unused)
    keys_.push_back(std::string());
    keys_.push_back(std::string());
    compute_starts();
    const int ncls = p_.num_byte_classes();
    uint8_t rep[256];
    {
      int seen = -1;
      for (int b = 0; b < 256; ++b)
        if (p_.byte_classes[b] != seen) { seen = p_.byte_classes[b]; rep[seen] = (uint8_t)b; }
    }
    // Transitions of DEAD and QUIT: absorbing.
    trans_cls_.assign((size_t)2 * ncls, 0);
    for (int c = 0; c < ncls; ++c) { trans_cls_[c] = 0; trans_cls_[ncls + c] = 1; }
    eof_match_ = {0, 0};
    eof_mask_ = {0, 0};
    for (size_t s = 2; s < keys_.size(); ++s) {
      if ((int)keys_.size() > lim_.max_raw_states) {
        if (err) *err = "DFA state budget exceeded (" + std::to_string(lim_.max_raw_states) + " states)";
        return false;
      }
      if (lim_.max_bytes && key_bytes_ + trans_cls_.size() * 4 > lim_.max_bytes) {
        if (err) *err = "DFA construction memory budget exceeded (" + std::to_string(lim_.max_bytes) + " bytes)";
        return false;
      }
      std::string key = keys_[s];  // copy: keys_ may grow
      if (strip_) strip_raw_.push_back(strip_key(key));
      trans_cls_.resize((s + 1) * ncls);
      // Sets: states that differ only in the matches their entry reported
      // step identically; compute each thread set's row once.
      size_t cut = key.size();
      if (is_set_) {
        for (size_t k = 1; k + 4 <= key.size(); k += 4) {
          uint32_t ip;
          memcpy(&ip, key.data() + k, 4);
          if (ip == 0xFFFFFFFFu) { cut = k; break; }
        }
        auto it = core_.find(key.substr(0, cut));
        if (it != core_.end()) {
          const size_t o = it->second;
          for (int c = 0; c < ncls; ++c) trans_cls_[s * ncls + c] = trans_cls_[o * ncls + c];
          eof_match_.push_back(eof_match_[o]);
          eof_mask_.push_back(eof_mask_[o]);
          continue;
        }
        core_.emplace(key.substr(0, cut), s);
      }
      step_row(key, ncls, rep, &trans_cls_[s * ncls]);
      uint64_t mask = 0;
      bool m = step_eof(key, &mask);
      eof_match_.push_back(m ? 1 : 0);
      eof_mask_.push_back(mask);
    }
    const int nraw = (int)keys_.size();
    const auto t_built = std::chrono::steady_clock::now();
    // Columns: the byte classes, split at 0x80 when the program has a
    // Unicode word boundary (non-ASCII bytes quit, dfa.rs:1487-1496).
    std::vector<int> colrep;
    {
      std::vector<int> seen(512, -1);
      for (int b = 0; b < 256; ++b) {
        const int key = p_.byte_classes[b] * 2 + ((quit_ && b >= 0x80) ? 1 : 0);
        if (seen[key] < 0) { seen[key] = (int)colrep.size(); colrep.push_back(b); }
        out->colmap[b] = (uint8_t)seen[key];
      }
    }
    const int ncol = (int)colrep.size();
    std::vector<uint32_t> tc((size_t)nraw * ncol);
    for (int s = 0; s < nraw; ++s)
      for (int j = 0; j < ncol; ++j) {
        const int b = colrep[j];
        tc[(size_t)s * ncol + j] = (quit_ && b >= 0x80 && s != 0) ? 1u : trans_cls_[(size_t)s * ncls + p_.byte_classes[b]];
      }
    std::vector<uint32_t>().swap(trans_cls_);
    minimise(nraw, tc, ncol, out);
    out->raw_states = nraw;
    if (knob(Knob::Timing) == 1) {  // diagnostic: construction and minimisation times
      const auto t_end = std::chrono::steady_clock::now();
      fprintf(stderr, "dfa_build: %d raw states, %d classes, %d states: construct %.3f s, minimise %.3f s\n", nraw,
              ncls, out->nstates, std::chrono::duration<double>(t_built - t_begin).count(),
              std::chrono::duration<double>(t_end - t_built).count());
    }
    return true;
  }

 private:
  const Program &p_;
  DfaBuildLimits lim_;
  // host memory held per interned state key beyond its bytes (two strings,
  // the hash node): the estimate max_bytes is checked against
  static constexpr size_t kKeyOverhead = 128;
  size_t key_bytes_ = 0;
  SparseSet qa_, qb_, qc_;
  std::vector<uint32_t> stack_;
  // step_row's cache across states: (flags, slots, target ips) -> raw state
  std::unordered_map<std::string, uint32_t> step_cache_;
  std::string tkey_;
  std::vector<std::string> sig_;   // step_row scratch: per class, the accepting threads' targets
  std::vector<uint32_t> stamp_;
  uint32_t stamp_gen_ = 0;
  bool is_set_, cont_, word_matters_, quit_, strip_ = false;
  std::vector<uint32_t> strip_raw_;  // raw state (from 2) -> stripped raw state
  std::vector<std::string> keys_;
  std::unordered_map<std::string, uint32_t> ids_;
  std::unordered_map<std::string, size_t> core_;  // sets: thread set -> first raw state with it
  std::vector<uint32_t> trans_cls_;
  std::vector<uint8_t> eof_match_;
  std::vector<uint64_t> eof_mask_;
  uint32_t start_raw_[128];
  bool start_used_[128];
  int lazy_ncls_ = 0;
  uint8_t lazy_rep_[256] = {0};

  // dfa.rs:1073-1134
  void follow(uint32_t ip0, SparseSet &q, const EmptyFlags &f) {
    stack_.push_back(ip0);
    while (!stack_.empty()) {
      uint32_t ip = stack_.back();
      stack_.pop_back();
      if (q.contains(ip)) continue;
      q.insert(ip);
      const Inst &in = p_.insts[ip];
      switch (in.op) {
        case OP_MATCH: case OP_BYTES: break;
        case OP_EMPTY: {
          bool ok = false;
          switch (in.look) {
            case LOOK_START_LINE: ok = f.start_line; break;
            case LOOK_END_LINE: ok = f.end_line; break;
            case LOOK_START_TEXT: ok = f.start; break;
            case LOOK_END_TEXT: ok = f.end; break;
            case LOOK_WORD_BOUNDARY_ASCII: case LOOK_WORD_BOUNDARY: ok = f.wb; break;
            case LOOK_NOT_WORD_BOUNDARY_ASCII: case LOOK_NOT_WORD_BOUNDARY: ok = f.nwb; break;
          }
          if (ok) stack_.push_back(in.x);
          break;
        }
        case OP_SAVE: stack_.push_back(in.x); break;
        case OP_SPLIT: stack_.push_back(in.y); stack_.push_back(in.x); break;
      }
    }
  }

  // follow(ip, q, ef2) for the step's flags (only start_line varies: the
  // byte is '\n' or not) from a cached closure list: within one step q is a
  // union of closures under the same flags, so an ip already in q has its
  // whole closure in q, and the DFS that stops at such ips adds exactly the
  // closure's other ips in the closure's own DFS order.
  std::vector<std::vector<uint32_t>> closure_[2];
  std::vector<uint8_t> closure_done_[2];
  void follow_cached(uint32_t ip, SparseSet &q, int nl) {
    if (closure_done_[nl].empty()) {
      closure_done_[nl].assign(p_.insts.size(), 0);
      closure_[nl].resize(p_.insts.size());
    }
    if (q.contains(ip)) return;  // its whole closure is in q already (above)
    if (!closure_done_[nl][ip]) {
      // one scratch set for every closure (clear() is O(1)): a set sized for
      // the program per closure cost a program-sized allocation each time
      SparseSet &tmp = qc_;
      tmp.clear();
      EmptyFlags ef;
      ef.start_line = nl != 0;
      follow(ip, tmp, ef);
      closure_[nl][ip].assign(tmp.dense.begin(), tmp.dense.begin() + tmp.n);
      closure_done_[nl][ip] = 1;
    }
    for (uint32_t x : closure_[nl][ip])
      if (!q.contains(x)) q.insert(x);
  }

  // dfa.rs:1196-1244 plus interning; returns raw id (0 = DEAD).  `now`
  // (sets only): Match slots reached by the step that produced this state.
  std::vector<uint32_t> kips_;  // intern's scratch: the key's instruction pointers
  std::string kbuf_;            // intern's scratch key
  uint32_t intern(const SparseSet &q, uint8_t sflags, uint64_t now = 0) {
    kips_.clear();
    for (size_t k = 0; k < q.n; ++k) {
      uint32_t ip = q.dense[k];
      const Inst &in = p_.insts[ip];
      bool push = false, stop = false;
      switch (in.op) {
        case OP_SAVE: case OP_SPLIT: break;
        case OP_BYTES: push = true; break;
        case OP_EMPTY: sflags |= SF_EMPTY; push = true; break;
        case OP_MATCH: push = true; stop = !cont_; break;
      }
      if (push) kips_.push_back(ip);
      if (stop) break;
    }
    if (kips_.empty() && !now && !(sflags & SF_MATCH)) return 0;
    std::string &key = kbuf_;
    key.resize(1 + 4 * kips_.size() + (now ? 12 : 0));
    key[0] = (char)sflags;
    if (!kips_.empty()) memcpy(&key[1], kips_.data(), 4 * kips_.size());
    if (now) {
      const uint32_t sep = 0xFFFFFFFFu;
      memcpy(&key[1 + 4 * kips_.size()], &sep, 4);
      memcpy(&key[5 + 4 * kips_.size()], &now, 8);
    }
    auto it = ids_.find(key);
    if (it != ids_.end()) return it->second;
    uint32_t id = (uint32_t)keys_.size();
    ids_.emplace(key, id);
    keys_.push_back(key);
    key_bytes_ += 2 * key.size() + kKeyOverhead;
    return id;
  }

  // The same ordered thread set without the `.*?` prefix instructions.
  uint32_t strip_key(const std::string &key) {
    std::string k(1, key[0]);
    for (size_t i = 1; i + 4 <= key.size(); i += 4) {
      uint32_t ip;
      memcpy(&ip, key.data() + i, 4);
      if (ip == 0xFFFFFFFFu) { k.append(key, i, std::string::npos); break; }
      if (ip >= p_.dotstar_end) k.append(key, i, 4);
    }
    if (k.size() == 1 && !(k[0] & SF_MATCH)) return 0;
    auto it = ids_.find(k);
    if (it != ids_.end()) return it->second;
    uint32_t id = (uint32_t)keys_.size();
    key_bytes_ += 2 * k.size() + kKeyOverhead;
    ids_.emplace(k, id);
    keys_.push_back(std::move(k));
    return id;
  }

  uint32_t strip_of(int s) const { return s < 2 ? (uint32_t)s : strip_raw_[s - 2]; }

  void load(const std::string &key, SparseSet &q) {
    q.clear();
    for (size_t k = 1; k + 4 <= key.size(); k += 4) {
      uint32_t ip;
      memcpy(&ip, key.data() + k, 4);
      if (ip == 0xFFFFFFFFu) break;  // sets: the `now` match mask follows
      q.insert(ip);
    }
  }

  static uint64_t now_of(const std::string &key) {
    for (size_t k = 1; k + 4 <= key.size(); k += 4) {
      uint32_t ip;
      memcpy(&ip, key.data() + k, 4);
      if (ip == 0xFFFFFFFFu) {
        uint64_t m;
        memcpy(&m, key.data() + k + 4, 8);
        return m;
      }
    }
    return 0;
  }

  // Shared body of exec_byte (dfa.rs:910-1048) for a real byte (b < 256) or
  // EOF (b == 256).  Leaves the resulting ordered set in *res and flags in *sf.
  void exec(const std::string &key, int b, SparseSet **res, uint8_t *sf, uint64_t *now = nullptr) {
    SparseSet *qcur = &qa_, *qnext = &qb_;
    load(key, *qcur);
    uint8_t flags = (uint8_t)key[0];
    bool is_word_last = (flags & SF_WORD) != 0;
    bool is_word = b < 256 && is_word_byte((uint8_t)b);
    if (flags & SF_EMPTY) {
      EmptyFlags ef;
      if (b == 256) { ef.end = true; ef.end_line = true; }
      else if (b == '\n') ef.end_line = true;
      if (is_word_last == is_word) ef.nwb = true; else ef.wb = true;
      qnext->clear();
      for (size_t k = 0; k < qcur->n; ++k) follow(qcur->dense[k], *qnext, ef);
      std::swap(qcur, qnext);
    }
    EmptyFlags ef2;
    ef2.start_line = (b == '\n');
    uint8_t sflags = 0;
    if (is_word && word_matters_) sflags |= SF_WORD;
    qnext->clear();
    uint64_t m_now = 0;
    for (size_t k = 0; k < qcur->n; ++k) {
      uint32_t ip = qcur->dense[k];
      const Inst &in = p_.insts[ip];
      if (in.op == OP_MATCH) {
        sflags |= SF_MATCH;
        if (!cont_) break;
        // Sets: the reference carries Match instructions forward in the
        // state (dfa.rs:988-993) so the final state holds every pattern seen.
        // Here they are reported by the step instead (the next state records
        // the slots reached now), which gives the same union of matches with
        // far fewer states (no subset-of-patterns-seen in the state).
        if (is_set_ && in.x < 64) m_now |= 1ull << in.x;
      } else if (in.op == OP_BYTES) {
        if (b < 256 && in.lo <= b && b <= in.hi) follow_cached(in.x, *qnext, ef2.start_line ? 1 : 0);
      }
    }
    if (b == 256 && is_set_) std::swap(qcur, qnext);  // dfa.rs:1004-1015
    *res = qnext;
    *sf = sflags;
    if (now) *now = m_now;
  }

  // One state's row over the byte classes.  The step on byte b depends only
  // on b's '\n'-ness and word-ness (the look-around flags) and on which Byte
  // instructions of the (flag-dependent) thread list accept b; classes that
  // agree on all of that share one exec (Unicode classes: a state's hundreds
  // of UTF-8 range instructions split the 100+ classes into few groups).
  void step_row(const std::string &key, int ncls, const uint8_t *rep, uint32_t *row) {
    const uint8_t flags = (uint8_t)key[0];
    std::unordered_map<std::string, uint32_t> memo[4];
    std::vector<std::string> &sig = sig_;
    sig.resize(ncls);
    uint8_t mflag = 0;
    uint64_t m_now = 0;
    bool scanned = false;
    for (int combo = 0; combo < 4; ++combo) {
      const bool nl = combo & 1, w = (combo >> 1) & 1;
      bool any = false;
      for (int c = 0; c < ncls && !any; ++c)
        any = (rep[c] == '\n') == nl && is_word_byte(rep[c]) == w;
      if (!any) continue;
      // the thread list the byte instructions are read from (exec's first
      // follow when the state holds empty-width instructions; without them
      // it is the state's own list for every combination)
      if (!scanned || (flags & SF_EMPTY)) {
        SparseSet &q = qa_;
        load(key, q);
        if (flags & SF_EMPTY) {
          EmptyFlags ef;
          if (nl) ef.end_line = true;
          if (((flags & SF_WORD) != 0) == w) ef.nwb = true; else ef.wb = true;
          qb_.clear();
          for (size_t k = 0; k < q.n; ++k) follow(q.dense[k], qb_, ef);
          std::swap(qa_, qb_);
        }
        SparseSet &qq = qa_;
        // exec_byte's second half (dfa.rs:966-1003) read off qq once: the
        // match flag and set slots of the threads before the first Match
        // (all of them for sets / reverse), and per class the targets of the
        // Byte threads that accept it, in priority order
        mflag = 0;
        m_now = 0;
        for (int c = 0; c < ncls; ++c) sig[c].clear();
        for (size_t k = 0; k < qq.n; ++k) {
          const Inst &in = p_.insts[qq.dense[k]];
          if (in.op == OP_MATCH) {
            mflag = SF_MATCH;
            if (!cont_) break;
            if (is_set_ && in.x < 64) m_now |= 1ull << in.x;
            continue;
          }
          if (in.op != OP_BYTES) continue;
          const int c0 = p_.byte_classes[in.lo], c1 = p_.byte_classes[in.hi];
          const uint32_t x = in.x;
          for (int c = c0; c <= c1; ++c) sig[c].append((const char *)&x, 4);
        }
        scanned = true;
      }
      const uint8_t sflags = (uint8_t)(mflag | (w && word_matters_ ? SF_WORD : 0));
      const uint64_t now = is_set_ ? m_now : 0;
      for (int c = 0; c < ncls; ++c) {
        if ((rep[c] == '\n') != nl || is_word_byte(rep[c]) != w) continue;
        auto it = memo[combo].find(sig[c]);
        if (it != memo[combo].end()) { row[c] = it->second; continue; }
        // The step on this class is the union, in order, of the closures
        // (under start_line = the byte is '\n') of the accepting threads'
        // targets, so it is a function of (that target list, the flags, the
        // set slots): cached across states (a repeated target adds nothing).
        std::string &tk = tkey_;
        tk.assign(1, (char)(sflags | (nl ? 0x80 : 0)));
        tk.append((const char *)&now, 8);
        ++stamp_gen_;
        const size_t nk = sig[c].size() / 4;
        for (size_t j = 0; j < nk; ++j) {
          uint32_t x;
          memcpy(&x, sig[c].data() + 4 * j, 4);
          if (stamp_[x] == stamp_gen_) continue;
          stamp_[x] = stamp_gen_;
          tk.append((const char *)&x, 4);
        }
        uint32_t t;
        auto st = step_cache_.find(tk);
        if (st != step_cache_.end()) {
          t = st->second;
        } else {
          SparseSet &nx = qb_;
          nx.clear();
          for (size_t j = 9; j < tk.size(); j += 4) {
            uint32_t x;
            memcpy(&x, tk.data() + j, 4);
            follow_cached(x, nx, nl ? 1 : 0);
          }
          t = intern(nx, sflags, now);
          step_cache_.emplace(tk, t);
        }
        memo[combo].emplace(sig[c], t);
        row[c] = t;
      }
    }
  }

  uint32_t step(const std::string &key, uint8_t b) {
    SparseSet *q; uint8_t sf; uint64_t now = 0;
    exec(key, b, &q, &sf, &now);
    return intern(*q, sf, is_set_ ? now : 0);
  }

  bool step_eof(const std::string &key, uint64_t *mask) {
    SparseSet *q; uint8_t sf;
    exec(key, 256, &q, &sf);
    uint64_t m = 0;
    if (is_set_) {
      for (size_t k = 0; k < q->n; ++k) {
        const Inst &in = p_.insts[q->dense[k]];
        if (in.op == OP_MATCH && in.x < 64) m |= 1ull << in.x;
      }
    }
    *mask = m;
    return (sf & SF_MATCH) != 0;
  }

  uint32_t start_for(const EmptyFlags &ef, bool word_last) {  // dfa.rs:1370-1409
    qa_.clear();
    follow(p_.start, qa_, ef);
    uint8_t sf = (word_last && word_matters_) ? SF_WORD : 0;
    return intern(qa_, sf);
  }

  static int flag_index(const EmptyFlags &e, bool word) {
    return (e.start ? 1 : 0) | (e.end ? 2 : 0) | (e.start_line ? 4 : 0) | (e.end_line ? 8 : 0) |
           (e.wb ? 16 : 0) | (e.nwb ? 32 : 0) | (word ? 64 : 0);
  }

  void compute_starts() {
    for (int i = 0; i < 128; ++i) { start_raw_[i] = 0; start_used_[i] = false; }
    // ctx: edge = at the text edge the search starts from (at==0 fwd, at==len rev);
    // empty = whole text empty; near: byte before (fwd) / at (rev) the start:
    // 0 none, 1 '\n', 2 word byte, 3 other; far_word: the other neighbour is a word byte.
    for (int edge = 0; edge < 2; ++edge)
      for (int empty = 0; empty < 2; ++empty)
        for (int near = 0; near < 4; ++near)
          for (int far_word = 0; far_word < 2; ++far_word) {
            if (empty && !edge) continue;
            if (edge && near != 0) continue;
            if (!edge && near == 0) continue;
            if (empty && far_word) continue;
            EmptyFlags ef;
            ef.start = edge;
            ef.end = empty;
            ef.start_line = edge || near == 1;
            ef.end_line = empty;
            bool word_last = near == 2;
            bool word_next = far_word;
            if (word_last == word_next) ef.nwb = true; else ef.wb = true;
            int fi = flag_index(ef, word_last);
            if (start_used_[fi]) continue;
            start_used_[fi] = true;
            start_raw_[fi] = start_for(ef, word_last);
          }
  }

  // Moore partition refinement over byte columns; outputs preserved:
  // single: (match flag, EOF match, dead, quit); set: (EOF match mask, dead, quit).
  // t: n raw states x ncol columns (out->colmap maps bytes to columns).
  void minimise(int n, const std::vector<uint32_t> &t, int ncol, DenseDfa *out) {
    std::vector<int> colbyte(ncol, 0);  // a byte of each column
    for (int b = 255; b >= 0; --b) colbyte[out->colmap[b]] = b;
    std::vector<uint32_t> block(n), nb(n);
    auto out_key = [&](int s) {
      std::string k;
      uint8_t tag = (s == 0 || (s == 1 && !quit_)) ? 1 : s == 1 ? 2 : 0;
      k.push_back((char)tag);
      if (s >= 2) {
        if (is_set_) {
          k.append((const char *)&eof_mask_[s], 8);
          uint64_t nm = now_of(keys_[s]);
          k.append((const char *)&nm, 8);
        }
        else {
          uint8_t m = (keys_[s][0] & SF_MATCH) ? 1 : 0;
          k.push_back((char)m);
          k.push_back((char)eof_match_[s]);
        }
      }
      return k;
    };
    size_t nblocks;
    if (!lim_.minimise) {  // every raw state its own block (DEAD and QUIT included)
      for (int s = 0; s < n; ++s) block[s] = (uint32_t)s;
      nblocks = (size_t)n;
    } else {
      std::unordered_map<std::string, uint32_t> m;
      for (int s = 0; s < n; ++s) {
        auto it = m.emplace(out_key(s), (uint32_t)m.size()).first;
        block[s] = it->second;
      }
      nblocks = m.size();
    }
    while (lim_.minimise) {
      std::unordered_map<std::string, uint32_t> m;
      m.reserve(n * 2);
      for (int s = 0; s < n; ++s) {
        std::string sig((const char *)&block[s], 4);
        for (int j = 0; j < ncol; ++j) sig.append((const char *)&block[t[(size_t)s * ncol + j]], 4);
        if (strip_) sig.append((const char *)&block[strip_of(s)], 4);
        auto it = m.emplace(sig, (uint32_t)m.size()).first;
        nb[s] = it->second;
      }
      bool done = m.size() == nblocks;
      nblocks = m.size();
      block.swap(nb);
      if (done) break;
    }
    // representative per block and categories
    std::vector<int> rep(nblocks, -1);
    for (int s = 0; s < n; ++s) if (rep[block[s]] < 0) rep[block[s]] = s;
    const uint32_t dead_b = block[0];
    const bool quit_used = quit_ && true;
    const uint32_t quit_b = block[1];
    auto is_special = [&](uint32_t b) {
      int s = rep[b];
      if (b == dead_b || (quit_used && b == quit_b)) return false;
      if (is_set_) return now_of(keys_[s]) != 0;  // entering it reports matches
      return (keys_[s][0] & SF_MATCH) != 0;
    };
    // order: normal states reachable from the start states through ASCII
    // bytes first (the LDS-resident "hot" set of the kernels), then the
    // remaining normal states, all in BFS order.
    std::vector<int32_t> newid(nblocks, -1);
    std::vector<uint32_t> order_normal, order_special;
    auto is_ordinary = [&](uint32_t b) {
      return b != dead_b && !(quit_used && b == quit_b) && !is_special(b);
    };
    {
      std::vector<char> seen(nblocks, 0);
      std::deque<uint32_t> dq;
      for (int i = 0; i < 128; ++i) {
        uint32_t b = block[start_raw_[i]];
        if (start_used_[i] && !seen[b] && is_ordinary(b)) { seen[b] = 1; dq.push_back(b); }
      }
      while (!dq.empty()) {
        uint32_t b = dq.front(); dq.pop_front();
        order_normal.push_back(b);
        int s = rep[b];
        for (int j = 0; j < ncol; ++j) {
          if (colbyte[j] >= 0x80) continue;   // columns of ASCII bytes
          uint32_t nb2 = block[t[(size_t)s * ncol + j]];
          if (!seen[nb2] && is_ordinary(nb2)) { seen[nb2] = 1; dq.push_back(nb2); }
        }
      }
      out->n_ascii = (int)order_normal.size();
      std::vector<char> seen2(nblocks, 0);
      auto push = [&](uint32_t b) { if (!seen2[b]) { seen2[b] = 1; dq.push_back(b); } };
      for (int i = 0; i < 128; ++i) if (start_used_[i]) push(block[start_raw_[i]]);
      for (uint32_t b = 0; b < nblocks; ++b) push(b);  // unreachable blocks last
      while (!dq.empty()) {
        uint32_t b = dq.front(); dq.pop_front();
        if (b != dead_b && !(quit_used && b == quit_b)) {
          if (is_special(b)) order_special.push_back(b);
          else if (!seen[b]) order_normal.push_back(b);
        }
        int s = rep[b];
        for (int j = 0; j < ncol; ++j) push(block[t[(size_t)s * ncol + j]]);
      }
    }
    int next = 0;
    for (uint32_t b : order_normal) newid[b] = next++;
    out->n_normal = next;
    for (uint32_t b : order_special) newid[b] = next++;
    out->n_match_end = next;
    out->dead = next;
    newid[dead_b] = next++;
    out->quit = -1;
    if (quit_used && quit_b != dead_b) { out->quit = next; newid[quit_b] = next++; }
    out->nstates = next;
    out->is_set = is_set_;
    out->reverse = p_.is_reverse;
    out->ncol = (uint32_t)ncol;
    out->eof_match.assign(next, 0);
    out->eof_mask.assign(next, 0);
    out->now_mask.assign(next, 0);
    if (lim_.columns) {
      out->trans.clear();
      out->ctrans.assign((size_t)next * ncol, 0);
    } else {
      out->trans.assign((size_t)next * 256, 0);
      out->ctrans.clear();
    }
    for (uint32_t b = 0; b < nblocks; ++b) {
      int s = rep[b], id = newid[b];
      if (lim_.columns) {
        for (int j = 0; j < ncol; ++j) out->ctrans[(size_t)id * ncol + j] = newid[block[t[(size_t)s * ncol + j]]];
      } else {
        for (int c = 0; c < 256; ++c)
          out->trans[(size_t)id * 256 + c] = newid[block[t[(size_t)s * ncol + out->colmap[c]]]];
      }
      out->eof_match[id] = eof_match_[s];
      out->eof_mask[id] = eof_mask_[s];
      if (is_set_) out->now_mask[id] = now_of(keys_[s]);
    }
    for (int i = 0; i < 128; ++i) out->start[i] = (uint32_t)(start_used_[i] ? newid[block[start_raw_[i]]] : out->dead);
    out->strip.clear();
    if (strip_) {
      out->strip.assign(next, 0);
      for (uint32_t b = 0; b < nblocks; ++b) out->strip[newid[b]] = newid[block[strip_of(rep[b])]];
    }
  }
};

}  // namespace

bool build_dense_dfa(const Program &prog, const DfaBuildLimits &lim, DenseDfa *out, std::string *err) {
  Builder b(prog, lim);
  return b.build(out, err);
}

struct LazyDfa::Impl {
  Builder b;
  Impl(const Program &p, const DfaBuildLimits &lim) : b(p, lim) {}
};

LazyDfa::LazyDfa(const Program &prog, size_t max_bytes) : max_bytes_(max_bytes) {
  DfaBuildLimits lim;
  lim.max_raw_states = 0x7FFFFFF0;
  impl_ = new Impl(prog, lim);
  impl_->b.lazy_init(colmap, &ncol);
  for (int i = 0; i < 128; ++i) start[i] = impl_->b.lazy_start(i);
  sync_new();
  for (int i = 0; i < 128; ++i) start[i] = entry_of(start[i]);
}

LazyDfa::~LazyDfa() { delete impl_; }

uint32_t LazyDfa::entry_of(uint32_t s) const {
  return s | (impl_->b.lazy_match(s) ? kLazyMatch : 0u);
}

// rows (unknown) and EOF flags for the states interned since the last call
void LazyDfa::sync_new() {
  const uint32_t n = impl_->b.lazy_states();
  for (uint32_t s = (uint32_t)eof.size(); s < n; ++s) {
    eof.push_back(impl_->b.lazy_eof(s) ? 1 : 0);
    built.push_back(s < 2 ? 1 : 0);
    trans.resize((size_t)(s + 1) * ncol, s < 2 ? s : kLazyUnknown);
    if (s >= 2) todo_.push_back(s);
  }
}

bool LazyDfa::build_row(uint32_t s) {
  if (s >= built.size() || built[s]) return true;
  if (max_bytes_ && impl_->b.lazy_bytes() + trans.size() * 4 > max_bytes_) return false;
  std::vector<uint32_t> row(ncol);
  impl_->b.lazy_row(s, row.data());
  sync_new();
  for (uint32_t c = 0; c < ncol; ++c) trans[(size_t)s * ncol + c] = entry_of(row[c]);
  built[s] = 1;
  ++nbuilt_;
  return true;
}

bool LazyDfa::expand(size_t rows) {
  for (size_t k = 0; k < rows && todo_head_ < todo_.size(); ++todo_head_) {
    const uint32_t s = todo_[todo_head_];
    if (built[s]) continue;
    if (!build_row(s)) return false;
    ++k;
  }
  return true;
}

int start_flag_index_fwd(const uint8_t *text, size_t len, size_t at) {  // dfa.rs:1415-1434
  bool start = at == 0, end = len == 0;
  bool start_line = at == 0 || text[at - 1] == '\n';
  bool word_last = at > 0 && is_word_byte(text[at - 1]);
  bool word = at < len && is_word_byte(text[at]);
  bool wb = word_last != word;
  return (start ? 1 : 0) | (end ? 2 : 0) | (start_line ? 4 : 0) | (end ? 8 : 0) |
         (wb ? 16 : 32) | (word_last ? 64 : 0);
}

int start_flag_index_rev(const uint8_t *text, size_t len, size_t at) {  // dfa.rs:1440-1464
  bool start = at == len, end = len == 0;
  bool start_line = at == len || text[at] == '\n';
  bool word_last = at < len && is_word_byte(text[at]);
  bool word = at > 0 && is_word_byte(text[at - 1]);
  bool wb = word_last != word;
  return (start ? 1 : 0) | (end ? 2 : 0) | (start_line ? 4 : 0) | (end ? 8 : 0) |
         (wb ? 16 : 32) | (word_last ? 64 : 0);
}

void prune_unreachable(DenseDfa *d) {
  const int n = d->nstates;
  if (n == 0 || d->trans.empty() || d->is_set) return;
  std::vector<char> keep(n, 0);
  std::vector<int> st;
  auto mark = [&](uint32_t s) {
    if (s < (uint32_t)n && !keep[s]) { keep[s] = 1; st.push_back((int)s); }
  };
  for (int i = 0; i < 128; ++i) mark(d->start[i]);
  mark((uint32_t)d->dead);
  if (d->quit >= 0) mark((uint32_t)d->quit);
  while (!st.empty()) {
    const int s = st.back();
    st.pop_back();
    for (int b = 0; b < 256; ++b) mark(d->trans[(size_t)s * 256 + b]);
    if (!d->strip.empty()) mark(d->strip[s]);
  }
  std::vector<uint32_t> id(n, 0);
  int next = 0, n_normal = 0, n_match_end = 0, n_ascii = 0;
  for (int s = 0; s < n; ++s) {
    if (!keep[s]) continue;
    id[s] = (uint32_t)next++;
    if (s < d->n_normal) ++n_normal;
    if (s < d->n_match_end) ++n_match_end;
    if (s < d->n_ascii) ++n_ascii;
  }
  if (next == n) return;
  std::vector<uint32_t> trans((size_t)next * 256);
  std::vector<uint8_t> eof_match(next);
  std::vector<uint64_t> eof_mask(next), now_mask(next);
  std::vector<uint32_t> strip(d->strip.empty() ? 0 : next);
  for (int s = 0; s < n; ++s) {
    if (!keep[s]) continue;
    const uint32_t t = id[s];
    for (int b = 0; b < 256; ++b) trans[(size_t)t * 256 + b] = id[d->trans[(size_t)s * 256 + b]];
    eof_match[t] = d->eof_match[s];
    eof_mask[t] = d->eof_mask[s];
    now_mask[t] = d->now_mask[s];
    if (!strip.empty()) strip[t] = id[d->strip[s]];
  }
  for (int i = 0; i < 128; ++i) d->start[i] = id[d->start[i]];
  d->dead = (int)id[d->dead];
  if (d->quit >= 0) d->quit = (int)id[d->quit];
  d->n_normal = n_normal;
  d->n_match_end = n_match_end;
  d->n_ascii = n_ascii;
  d->nstates = next;
  d->trans.swap(trans);
  d->eof_match.swap(eof_match);
  d->eof_mask.swap(eof_mask);
  d->now_mask.swap(now_mask);
  d->strip.swap(strip);
}

}  // namespace rure_amd
