// Expression tree -> byte Program.  Restates the reference compiler
// src/compile.rs (patch/hole back-patching 208-766, UTF-8 class compilation
// with the bounded suffix cache 875-1049, byte equivalence classes
// 1051-1102) and the `utf8-ranges` 1.x crate's Utf8Sequences algorithm it
// calls (compile.rs:20,62,885-917; the crate is not vendored in the
// reference, its published algorithm is restated below).
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "program.hpp"

namespace rure_amd {
namespace {

// ------------------------------------------------------------ utf8-ranges
struct Utf8Range { uint8_t lo, hi; };
struct Utf8Seq { int n; Utf8Range r[4]; };

static int encode_utf8(uint32_t c, uint8_t *dst) {
  if (c < 0x80) { dst[0] = (uint8_t)c; return 1; }
  if (c < 0x800) { dst[0] = 0xC0 | (c >> 6); dst[1] = 0x80 | (c & 0x3F); return 2; }
  if (c < 0x10000) {
    dst[0] = 0xE0 | (c >> 12); dst[1] = 0x80 | ((c >> 6) & 0x3F); dst[2] = 0x80 | (c & 0x3F);
    return 3;
  }
  dst[0] = 0xF0 | (c >> 18); dst[1] = 0x80 | ((c >> 12) & 0x3F);
  dst[2] = 0x80 | ((c >> 6) & 0x3F); dst[3] = 0x80 | (c & 0x3F);
  return 4;
}

// Splits a scalar range into UTF-8 byte-range sequences that together match
// exactly the UTF-8 encodings of the scalars in the range (surrogates
// excluded), in ascending order.
class Utf8Sequences {
 public:
  void reset(uint32_t lo, uint32_t hi) { stack_.clear(); stack_.push_back({lo, hi}); }
  bool next(Utf8Seq *out) {
    static const uint32_t kMax[4] = {0x7F, 0x7FF, 0xFFFF, 0x10FFFF};
    while (!stack_.empty()) {
      SR r = stack_.back();
      stack_.pop_back();
      while (true) {
        if (r.lo < 0xE000 && r.hi > 0xD7FF) {       // split around surrogates
          stack_.push_back({0xE000, r.hi});
          r.hi = 0xD7FF;
          continue;
        }
        if (r.lo > r.hi) break;                      // invalid: next on stack
        bool again = false;
        for (int i = 0; i < 3; ++i) {                // split at encoded-length edges
          uint32_t m = kMax[i];
          if (r.lo <= m && m < r.hi) {
            stack_.push_back({m + 1, r.hi});
            r.hi = m;
            again = true;
            break;
          }
        }
        if (again) continue;
        if (r.hi <= 0x7F) {
          out->n = 1; out->r[0] = {(uint8_t)r.lo, (uint8_t)r.hi};
          return true;
        }
        for (int i = 1; i < 4; ++i) {                // align to continuation-byte blocks
          uint32_t m = (1u << (6 * i)) - 1;
          if ((r.lo & ~m) != (r.hi & ~m)) {
            if ((r.lo & m) != 0) {
              stack_.push_back({(r.lo | m) + 1, r.hi});
              r.hi = r.lo | m;
              again = true;
              break;
            }
            if ((r.hi & m) != m) {
              stack_.push_back({r.hi & ~m, r.hi});
              r.hi = (r.hi & ~m) - 1;
              again = true;
              break;
            }
          }
        }
        if (again) continue;
        uint8_t s[4], e[4];
        int n = encode_utf8(r.lo, s);
        int m = encode_utf8(r.hi, e);
        if (n != m) throw std::runtime_error("utf8 sequence length mismatch");
        out->n = n;
        for (int k = 0; k < n; ++k) out->r[k] = {s[k], e[k]};
        return true;
      }
    }
    return false;
  }

 private:
  struct SR { uint32_t lo, hi; };
  std::vector<SR> stack_;
};

// ------------------------------------------------------------- compiler
enum MState : uint8_t { M_COMPILED, M_HOLE, M_SPLIT, M_SPLIT1, M_SPLIT2 };
struct MaybeInst { Inst inst; MState st; };

typedef std::vector<uint32_t> Hole;   // flattened Hole::{None,One,Many}
struct Patch { Hole hole; uint32_t entry; };

struct CompileError { std::string msg; };

class Compiler {
 public:
  explicit Compiler(const CompileOptions &o) : opt_(o) {
    prog_.is_dfa = o.dfa;
    prog_.is_reverse = o.reverse;
    prog_.only_utf8 = o.only_utf8;
    memset(bcset_, 0, sizeof(bcset_));
    for (auto &e : sc_) e = SCEntry{};
  }

  Program compile(const std::vector<Expr> &exprs) {  // compile.rs:124-135
    num_exprs_ = exprs.size();
    if (exprs.size() == 1) compile_one(exprs[0]);
    else compile_many(exprs);
    finish();
    return std::move(prog_);
  }

 private:
  CompileOptions opt_;
  Program prog_;
  std::vector<MaybeInst> insts_;
  size_t num_exprs_ = 0;
  bool bcset_[256];
  Utf8Sequences seqs_;
  // Bounded suffix cache (compile.rs:989-1049), 1000 entries, FNV-1a.
  struct SCKey { uint64_t from; uint8_t lo, hi; };
  struct SCEntry { SCKey key{0, 0, 0}; uint32_t pc = 0; uint64_t version = 0; };
  SCEntry sc_[1000];
  uint64_t sc_version_ = 0;

  bool needs_dotstar() const { return prog_.is_dfa && !prog_.is_reverse && !prog_.anchored_start; }
  uint32_t len() const { return (uint32_t)insts_.size(); }

  void check_size() {  // compile.rs:757-765 (size_of::<Inst>() == 40)
    if (insts_.size() * 40 > opt_.size_limit)
      throw CompileError{"Compiled regex exceeds size limit of " + std::to_string(opt_.size_limit) + " bytes."};
  }

  void set_range(uint8_t lo, uint8_t hi) {  // compile.rs:1058-1064
    if (lo > 0) bcset_[lo - 1] = true;
    bcset_[hi] = true;
  }
  void set_word_boundary() {  // compile.rs:1066-1080
    int b1 = 0;
    while (b1 <= 255) {
      int b2 = b1 + 1;
      while (b2 <= 255 && is_word_byte((uint8_t)b1) == is_word_byte((uint8_t)b2)) ++b2;
      set_range((uint8_t)b1, (uint8_t)(b2 - 1));
      b1 = b2;
    }
  }

  Hole push_hole(Inst partial) {
    insts_.push_back({partial, M_HOLE});
    return Hole{len() - 1};
  }
  Hole push_split_hole() {
    Inst i{}; i.op = OP_SPLIT;
    insts_.push_back({i, M_SPLIT});
    return Hole{len() - 1};
  }
  void push_compiled(Inst i) { insts_.push_back({i, M_COMPILED}); }

  void fill(const Hole &h, uint32_t go) {  // compile.rs:680-692, 785-798
    for (uint32_t pc : h) {
      MaybeInst &m = insts_[pc];
      switch (m.st) {
        case M_HOLE: m.inst.x = go; m.st = M_COMPILED; break;
        case M_SPLIT1: m.inst.y = go; m.st = M_COMPILED; break;      // Split(goto1, go)
        case M_SPLIT2: m.inst.x = go; m.st = M_COMPILED; break;      // Split(go, goto2)
        default: throw std::runtime_error("fill on compiled instruction");
      }
    }
  }
  void fill_to_next(const Hole &h) { fill(h, len()); }
  // compile.rs:699-739; g1/g2 < 0 means "not given".
  Hole fill_split(const Hole &h, int64_t g1, int64_t g2) {
    Hole out;
    for (uint32_t pc : h) {
      MaybeInst &m = insts_[pc];
      if (m.st != M_SPLIT) throw std::runtime_error("fill_split on non-split");
      if (g1 >= 0 && g2 >= 0) { m.inst.x = (uint32_t)g1; m.inst.y = (uint32_t)g2; m.st = M_COMPILED; }
      else if (g1 >= 0) { m.inst.x = (uint32_t)g1; m.st = M_SPLIT1; out.push_back(pc); }
      else { m.inst.y = (uint32_t)g2; m.st = M_SPLIT2; out.push_back(pc); }
    }
    return out;
  }
  static Hole cat(Hole a, const Hole &b) { a.insert(a.end(), b.begin(), b.end()); return a; }

  void compile_one(const Expr &e) {  // compile.rs:137-160
    Patch dot{{}, 0};
    prog_.anchored_start = e.is_anchored_start();
    prog_.anchored_end = e.is_anchored_end();
    if (needs_dotstar()) { dot = c_dotstar(); prog_.start = dot.entry; prog_.dotstar_end = (uint32_t)len(); }
    prog_.capture_names = {""};
    prog_.capture_has_name = {false};
    Patch p = c_capture(0, e);
    if (needs_dotstar()) fill(dot.hole, p.entry);
    else prog_.start = p.entry;
    fill_to_next(p.hole);
    prog_.matches = {len()};
    Inst m{}; m.op = OP_MATCH; m.x = 0;
    push_compiled(m);
  }

  void compile_many(const std::vector<Expr> &es) {  // compile.rs:162-198
    bool as = true, ae = true;
    for (const Expr &e : es) { as = as && e.is_anchored_start(); ae = ae && e.is_anchored_end(); }
    prog_.anchored_start = as;
    prog_.anchored_end = ae;
    Patch dot{{}, 0};
    if (needs_dotstar()) { dot = c_dotstar(); prog_.start = dot.entry; prog_.dotstar_end = (uint32_t)len(); }
    else prog_.start = 0;
    fill_to_next(dot.hole);
    Hole prev;
    for (size_t i = 0; i + 1 < es.size(); ++i) {
      fill_to_next(prev);
      Hole split = push_split_hole();
      Patch p = c_capture(0, es[i]);
      fill_to_next(p.hole);
      prog_.matches.push_back(len());
      Inst m{}; m.op = OP_MATCH; m.x = (uint32_t)i;
      push_compiled(m);
      prev = fill_split(split, p.entry, -1);
    }
    size_t i = es.size() - 1;
    Patch p = c_capture(0, es[i]);
    fill(prev, p.entry);
    fill_to_next(p.hole);
    prog_.matches.push_back(len());
    Inst m{}; m.op = OP_MATCH; m.x = (uint32_t)i;
    push_compiled(m);
  }

  void finish() {  // compile.rs:200-206, 1082-1101
    prog_.insts.reserve(insts_.size());
    for (const MaybeInst &m : insts_) {
      if (m.st != M_COMPILED) throw std::runtime_error("uncompiled instruction left");
      prog_.insts.push_back(m.inst);
    }
    uint8_t cls = 0;
    for (int i = 0; i < 256; ++i) {
      prog_.byte_classes[i] = cls;
      if (i < 255 && bcset_[i]) ++cls;
    }
  }

  Patch c(const Expr &e) {  // compile.rs:260-362
    check_size();
    switch (e.kind) {
      case EK::Empty: return Patch{{}, len()};
      case EK::Literal: return c_literal(e.chars, e.casei);
      case EK::LiteralBytes: return c_bytes(e.bytes, e.casei);
      case EK::AnyChar: return c_class({{0, 0x10FFFF}});
      case EK::AnyCharNoNL: return c_class({{0, 0x09}, {0x0B, 0x10FFFF}});
      case EK::AnyByte: return c_class_bytes({{0, 0xFF}});
      case EK::AnyByteNoNL: return c_class_bytes({{0, 0x09}, {0x0B, 0xFF}});
      case EK::Class: return c_class(e.cls);
      case EK::ClassBytes: return c_class_bytes(e.bcls);
      case EK::StartLine:
        set_range('\n', '\n');
        return c_empty(prog_.is_reverse ? LOOK_END_LINE : LOOK_START_LINE);
      case EK::EndLine:
        set_range('\n', '\n');
        return c_empty(prog_.is_reverse ? LOOK_START_LINE : LOOK_END_LINE);
      case EK::StartText: return c_empty(prog_.is_reverse ? LOOK_END_TEXT : LOOK_START_TEXT);
      case EK::EndText: return c_empty(prog_.is_reverse ? LOOK_START_TEXT : LOOK_END_TEXT);
      case EK::WordBoundary:
        prog_.has_unicode_word_boundary = true;
        set_word_boundary();
        return c_empty(LOOK_WORD_BOUNDARY);
      case EK::NotWordBoundary:
        prog_.has_unicode_word_boundary = true;
        set_word_boundary();
        return c_empty(LOOK_NOT_WORD_BOUNDARY);
      case EK::WordBoundaryAscii:
        set_word_boundary();
        return c_empty(LOOK_WORD_BOUNDARY_ASCII);
      case EK::NotWordBoundaryAscii:
        set_word_boundary();
        return c_empty(LOOK_NOT_WORD_BOUNDARY_ASCII);
      case EK::Group: {
        if (e.cap < 0 && !e.has_name) return c(e.subs[0]);
        size_t i = (size_t)e.cap;
        if (i >= prog_.capture_names.size()) {
          prog_.capture_names.push_back(e.has_name ? e.name : "");
          prog_.capture_has_name.push_back(e.has_name);
        }
        return c_capture((uint32_t)(2 * i), e.subs[0]);
      }
      case EK::Concat: {
        std::vector<const Expr *> v;
        for (const Expr &s : e.subs) v.push_back(&s);
        if (prog_.is_reverse) std::reverse(v.begin(), v.end());
        return c_concat(v);
      }
      case EK::Alternate: return c_alternate(e.subs);
      case EK::Repeat: return c_repeat(e);
    }
    throw std::runtime_error("bad expr");
  }

  Patch c_capture(uint32_t first_slot, const Expr &e) {  // compile.rs:364-379
    if (num_exprs_ > 1 || prog_.is_dfa) return c(e);
    uint32_t entry = len();
    Inst s{}; s.op = OP_SAVE; s.y = first_slot;
    Hole h = push_hole(s);
    Patch p = c(e);
    fill(h, p.entry);
    fill_to_next(p.hole);
    Inst s2{}; s2.op = OP_SAVE; s2.y = first_slot + 1;
    Hole h2 = push_hole(s2);
    return Patch{h2, entry};
  }

  Patch c_dotstar() {  // compile.rs:381-395
    Expr any; any.kind = prog_.only_utf8 ? EK::AnyChar : EK::AnyByte;
    Expr r; r.kind = EK::Repeat; r.rep = Rep::ZeroOrMore; r.greedy = false;
    r.subs.push_back(any);
    return c(r);
  }

  Patch c_literal(const std::vector<uint32_t> &chars, bool casei) {  // compile.rs:397-413
    std::vector<uint32_t> v = chars;
    if (prog_.is_reverse) std::reverse(v.begin(), v.end());
    Patch p = c_char(v[0], casei);
    Hole hole = p.hole;
    for (size_t k = 1; k < v.size(); ++k) {
      Patch q = c_char(v[k], casei);
      fill(hole, q.entry);
      hole = q.hole;
    }
    return Patch{hole, p.entry};
  }
  Patch c_char(uint32_t ch, bool casei) {  // compile.rs:415-423
    if (casei) return c_class(class_case_fold({{ch, ch}}));
    return c_class({{ch, ch}});
  }
  Patch c_bytes(const std::vector<uint8_t> &bytes, bool casei) {  // compile.rs:444-460
    std::vector<uint8_t> v = bytes;
    if (prog_.is_reverse) std::reverse(v.begin(), v.end());
    Patch p = c_byte(v[0], casei);
    Hole hole = p.hole;
    for (size_t k = 1; k < v.size(); ++k) {
      Patch q = c_byte(v[k], casei);
      fill(hole, q.entry);
      hole = q.hole;
    }
    return Patch{hole, p.entry};
  }
  Patch c_byte(uint8_t b, bool casei) {  // compile.rs:462-470
    if (casei) return c_class_bytes(bclass_case_fold({{b, b}}));
    return c_class_bytes({{b, b}});
  }

  Patch c_class_bytes(const std::vector<BRange> &r) {  // compile.rs:472-496
    uint32_t first = len();
    Hole holes, prev;
    for (size_t k = 0; k + 1 < r.size(); ++k) {
      fill_to_next(prev);
      Hole split = push_split_hole();
      uint32_t next = len();
      set_range(r[k].lo, r[k].hi);
      Inst b{}; b.op = OP_BYTES; b.lo = r[k].lo; b.hi = r[k].hi;
      holes = cat(holes, push_hole(b));
      prev = fill_split(split, next, -1);
    }
    uint32_t next = len();
    set_range(r.back().lo, r.back().hi);
    Inst b{}; b.op = OP_BYTES; b.lo = r.back().lo; b.hi = r.back().hi;
    holes = cat(holes, push_hole(b));
    fill(prev, next);
    return Patch{holes, first};
  }

  Patch c_empty(Look look) {  // compile.rs:498-501
    Inst e{}; e.op = OP_EMPTY; e.look = look;
    Hole h = push_hole(e);
    return Patch{h, len() - 1};
  }

  Patch c_concat(const std::vector<const Expr *> &v) {  // compile.rs:503-519
    if (v.empty()) return Patch{{}, len()};
    Patch p = c(*v[0]);
    Hole hole = p.hole;
    for (size_t k = 1; k < v.size(); ++k) {
      Patch q = c(*v[k]);
      fill(hole, q.entry);
      hole = q.hole;
    }
    return Patch{hole, p.entry};
  }

  Patch c_alternate(const std::vector<Expr> &es) {  // compile.rs:521-544
    uint32_t first = len();
    Hole holes, prev;
    for (size_t k = 0; k + 1 < es.size(); ++k) {
      fill_to_next(prev);
      Hole split = push_split_hole();
      Patch p = c(es[k]);
      holes = cat(holes, p.hole);
      prev = fill_split(split, p.entry, -1);
    }
    Patch p = c(es.back());
    holes = cat(holes, p.hole);
    fill(prev, p.entry);
    return Patch{holes, first};
  }

  Patch c_repeat(const Expr &e) {  // compile.rs:546-678
    const Expr &x = e.subs[0];
    switch (e.rep) {
      case Rep::ZeroOrOne: {
        uint32_t entry = len();
        Hole split = push_split_hole();
        Patch r = c(x);
        Hole sh = e.greedy ? fill_split(split, r.entry, -1) : fill_split(split, -1, r.entry);
        return Patch{cat(r.hole, sh), entry};
      }
      case Rep::ZeroOrMore: return c_zero_or_more(x, e.greedy);
      case Rep::OneOrMore: {
        Patch r = c(x);
        fill_to_next(r.hole);
        Hole split = push_split_hole();
        Hole sh = e.greedy ? fill_split(split, r.entry, -1) : fill_split(split, -1, r.entry);
        return Patch{sh, r.entry};
      }
      case Rep::Range: {
        std::vector<const Expr *> v(e.rmin, &x);
        if (!e.has_max) {
          Patch pc = c_concat(v);
          Patch pr = c_zero_or_more(x, e.greedy);
          fill(pc.hole, pr.entry);
          return Patch{pr.hole, pc.entry};
        }
        Patch pc = c_concat(v);
        uint32_t initial = pc.entry;
        if (e.rmin == e.rmax) return pc;
        Hole holes, prev = pc.hole;
        for (uint32_t k = e.rmin; k < e.rmax; ++k) {
          fill_to_next(prev);
          Hole split = push_split_hole();
          Patch r = c(x);
          prev = r.hole;
          holes = cat(holes, e.greedy ? fill_split(split, r.entry, -1) : fill_split(split, -1, r.entry));
        }
        holes = cat(holes, prev);
        return Patch{holes, initial};
      }
    }
    throw std::runtime_error("bad repeat");
  }
  Patch c_zero_or_more(const Expr &x, bool greedy) {  // compile.rs:583-599
    uint32_t entry = len();
    Hole split = push_split_hole();
    Patch r = c(x);
    fill(r.hole, entry);
    Hole sh = greedy ? fill_split(split, r.entry, -1) : fill_split(split, -1, r.entry);
    return Patch{sh, entry};
  }

  // ------------------------------------------------- UTF-8 class compile
  uint32_t sc_get(SCKey k, uint32_t pc, bool *hit) {  // compile.rs:1020-1048
    const uint64_t P = 1099511628211ull;
    uint64_t h = 14695981039346656037ull;
    h = (h ^ k.from) * P;
    h = (h ^ (uint64_t)k.lo) * P;
    h = (h ^ (uint64_t)k.hi) * P;
    SCEntry &e = sc_[h % 1000];
    if (e.key.from == k.from && e.key.lo == k.lo && e.key.hi == k.hi && e.version == sc_version_) {
      *hit = true;
      return e.pc;
    }
    e.key = k; e.pc = pc; e.version = sc_version_;
    *hit = false;
    return 0;
  }

  Patch c_utf8_seq(const Utf8Seq &s) {  // compile.rs:924-968
    const uint64_t NONE = ~0ull;
    uint64_t from = NONE;
    Hole last;
    for (int k = 0; k < s.n; ++k) {
      // forward programs compile the sequence last byte first
      const Utf8Range &br = prog_.is_reverse ? s.r[k] : s.r[s.n - 1 - k];
      bool hit;
      uint32_t cached = sc_get(SCKey{from, br.lo, br.hi}, len(), &hit);
      if (hit) { from = cached; continue; }
      set_range(br.lo, br.hi);
      Inst b{}; b.op = OP_BYTES; b.lo = br.lo; b.hi = br.hi;
      if (from == NONE) last = push_hole(b);
      else { b.x = (uint32_t)from; push_compiled(b); }
      from = len() - 1;
    }
    return Patch{last, (uint32_t)from};
  }

  Patch c_class(const std::vector<CRange> &ranges) {  // compile.rs:425-442, 881-922
    if (ranges.empty()) throw std::runtime_error("empty class");
    Hole holes, last_split;
    int64_t initial = -1;
    sc_version_++;  // suffix_cache.clear()
    for (size_t i = 0; i < ranges.size(); ++i) {
      bool last_range = i + 1 == ranges.size();
      seqs_.reset(ranges[i].lo, ranges[i].hi);
      Utf8Seq cur, nxt;
      bool have = seqs_.next(&cur);
      while (have) {
        bool have_next = seqs_.next(&nxt);
        if (last_range && !have_next) {
          Patch p = c_utf8_seq(cur);
          holes = cat(holes, p.hole);
          fill(last_split, p.entry);
          last_split.clear();
          if (initial < 0) initial = p.entry;
        } else {
          if (initial < 0) initial = len();
          fill_to_next(last_split);
          last_split = push_split_hole();
          Patch p = c_utf8_seq(cur);
          holes = cat(holes, p.hole);
          last_split = fill_split(last_split, p.entry, -1);
        }
        cur = nxt;
        have = have_next;
      }
    }
    return Patch{holes, (uint32_t)initial};
  }
};

}  // namespace

bool compile_program(const std::vector<Expr> &exprs, const CompileOptions &opt,
                     Program *out, std::string *err) {
  try {
    Compiler c(opt);
    *out = c.compile(exprs);
    return true;
  } catch (const CompileError &e) {
    if (err) *err = e.msg;
    return false;
  } catch (const std::exception &e) {
    if (err) *err = std::string("internal compiler error: ") + e.what();
    return false;
  }
}

}  // namespace rure_amd
