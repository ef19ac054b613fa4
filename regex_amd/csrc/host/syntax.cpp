// Host-side regex parser.  See syntax.hpp for the reference behaviour this
// restates (regex-syntax/src/parser.rs, regex-syntax/src/lib.rs).
#include "syntax.hpp"

#include <algorithm>
#include <cstring>

#include "unicode_tables.h"

namespace rure_amd {
namespace U = rure_amd_unicode;

static const uint32_t kMaxChar = 0x10FFFF;

// ---------------------------------------------------------------- helpers
static uint32_t inc_char(uint32_t c) {            // lib.rs:1711-1717
  if (c == kMaxChar) return kMaxChar;
  if (c == 0xD7FF) return 0xE000;
  return c + 1;
}
static uint32_t dec_char(uint32_t c) {            // lib.rs:1719-1725
  if (c == 0) return 0;
  if (c == 0xE000) return 0xD7FF;
  return c - 1;
}

static bool in_table(U::Span s, uint32_t c) {
  const uint32_t *p = U::kPairs + 2 * s.first;
  size_t lo = 0, hi = s.count;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (c < p[2 * mid]) hi = mid;
    else if (c > p[2 * mid + 1]) lo = mid + 1;
    else return true;
  }
  return false;
}

static std::vector<CRange> table_class(U::Span s) {
  std::vector<CRange> out;
  out.reserve(s.count);
  for (uint32_t i = 0; i < s.count; ++i)
    out.push_back({U::kPairs[2 * (s.first + i)], U::kPairs[2 * (s.first + i) + 1]});
  return out;
}

bool is_word_byte(uint8_t b) {
  return b == '_' || (b >= '0' && b <= '9') || (b >= 'a' && b <= 'z') ||
         (b >= 'A' && b <= 'Z');
}

bool is_word_char(uint32_t c) {
  if (c < 0x80) return is_word_byte((uint8_t)c);
  return in_table(U::kPerlW, c);
}

static bool is_whitespace(uint32_t c) { return in_table(U::kPerlS, c); }

bool decode_utf8(const uint8_t *p, size_t n, uint32_t *cp, size_t *len) {
  // Strict decoding (rejects overlong, surrogates, > U+10FFFF), as Rust's
  // str::from_utf8 and the reference's utf8.rs:decode_utf8 (utf8.rs:24-81).
  if (n == 0) return false;
  uint8_t b0 = p[0];
  if (b0 < 0x80) { *cp = b0; *len = 1; return true; }
  if (b0 < 0xC2) return false;
  if (b0 < 0xE0) {
    if (n < 2 || (p[1] & 0xC0) != 0x80) return false;
    *cp = ((b0 & 0x1F) << 6) | (p[1] & 0x3F); *len = 2; return true;
  }
  if (b0 < 0xF0) {
    if (n < 3 || (p[1] & 0xC0) != 0x80 || (p[2] & 0xC0) != 0x80) return false;
    uint32_t c = ((b0 & 0x0F) << 12) | ((p[1] & 0x3F) << 6) | (p[2] & 0x3F);
    if (c < 0x800 || (c >= 0xD800 && c <= 0xDFFF)) return false;
    *cp = c; *len = 3; return true;
  }
  if (b0 < 0xF5) {
    if (n < 4 || (p[1] & 0xC0) != 0x80 || (p[2] & 0xC0) != 0x80 ||
        (p[3] & 0xC0) != 0x80) return false;
    uint32_t c = ((b0 & 0x07) << 18) | ((p[1] & 0x3F) << 12) |
                 ((p[2] & 0x3F) << 6) | (p[3] & 0x3F);
    if (c < 0x10000 || c > kMaxChar) return false;
    *cp = c; *len = 4; return true;
  }
  return false;
}

// ------------------------------------------------------- class algebra
std::vector<CRange> class_canonicalize(std::vector<CRange> r) {  // lib.rs:687-704
  std::sort(r.begin(), r.end(), [](const CRange &a, const CRange &b) {
    return a.lo != b.lo ? a.lo < b.lo : a.hi < b.hi;
  });
  std::vector<CRange> out;
  for (const CRange &c : r) {
    if (!out.empty()) {
      CRange &o = out.back();
      // overlapping(): max(start) <= inc_char(min(end))  (lib.rs:835-837)
      if (std::max(o.lo, c.lo) <= inc_char(std::min(o.hi, c.hi))) {
        o.lo = std::min(o.lo, c.lo);
        o.hi = std::max(o.hi, c.hi);
        continue;
      }
    }
    out.push_back(c);
  }
  return out;
}

std::vector<CRange> class_negate(std::vector<CRange> r) {  // lib.rs:745-768
  if (r.empty()) return {{0, kMaxChar}};
  r = class_canonicalize(std::move(r));
  std::vector<CRange> inv;
  if (r[0].lo > 0) inv.push_back({0, dec_char(r[0].lo)});
  for (size_t i = 1; i < r.size(); ++i)
    inv.push_back({inc_char(r[i - 1].hi), dec_char(r[i].lo)});
  if (r.back().hi < kMaxChar) inv.push_back({inc_char(r.back().hi), kMaxChar});
  return inv;
}

static std::vector<CRange> class_intersect(const std::vector<CRange> &a,
                                           const std::vector<CRange> &b) {
  // lib.rs:709-739
  std::vector<CRange> out;
  if (a.empty() || b.empty()) return out;
  size_t i = 0, j = 0;
  while (true) {
    uint32_t lo = std::max(a[i].lo, b[j].lo), hi = std::min(a[i].hi, b[j].hi);
    if (lo <= hi) out.push_back({lo, hi});
    if (a[i].hi < b[j].hi) { if (++i == a.size()) break; }
    else { if (++j == b.size()) break; }
  }
  return class_canonicalize(std::move(out));
}

// Simple case folding: each scalar maps to every partner listed in the
// C+S "both" table (lib.rs:776-915, unicode.rs:4994).  The result is the
// same set the reference builds; we canonicalize it.
static const uint32_t *fold_pairs() { return U::kPairs + 2 * U::kCaseFold.first; }

static size_t fold_lower_bound(uint32_t c) {
  const uint32_t *p = fold_pairs();
  size_t lo = 0, hi = U::kCaseFold.count;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (p[2 * mid] < c) lo = mid + 1; else hi = mid;
  }
  return lo;
}

std::vector<CRange> class_case_fold(const std::vector<CRange> &r) {
  const uint32_t *p = fold_pairs();
  const size_t n = U::kCaseFold.count;
  std::vector<CRange> out;
  for (const CRange &rg : r) {
    out.push_back(rg);
    size_t i = fold_lower_bound(rg.lo);
    for (; i < n && p[2 * i] <= rg.hi; ++i) {
      uint32_t c2 = p[2 * i + 1];
      out.push_back({c2, c2});
    }
  }
  return class_canonicalize(std::move(out));
}

std::vector<BRange> bclass_canonicalize(std::vector<BRange> r) {  // lib.rs:1006-1023
  std::sort(r.begin(), r.end(), [](const BRange &a, const BRange &b) {
    return a.lo != b.lo ? a.lo < b.lo : a.hi < b.hi;
  });
  std::vector<BRange> out;
  for (const BRange &c : r) {
    if (!out.empty()) {
      BRange &o = out.back();
      int mn = std::min(o.hi, c.hi);
      if ((int)std::max(o.lo, c.lo) <= std::min(mn + 1, 255)) {
        o.lo = std::min(o.lo, c.lo);
        o.hi = std::max(o.hi, c.hi);
        continue;
      }
    }
    out.push_back(c);
  }
  return out;
}

std::vector<BRange> bclass_case_fold(const std::vector<BRange> &r) {  // lib.rs:1062-1133
  std::vector<BRange> out;
  for (const BRange &b : r) {
    out.push_back(b);
    if (!(std::max<int>(b.lo, 'a') > std::min<int>(b.hi, 'z'))) {
      int lo = std::max<int>(b.lo, 'a'), hi = std::min<int>(b.hi, 'z');
      out.push_back({(uint8_t)(lo - 32), (uint8_t)(hi - 32)});
    }
    if (!(std::max<int>(b.lo, 'A') > std::min<int>(b.hi, 'Z'))) {
      int lo = std::max<int>(b.lo, 'A'), hi = std::min<int>(b.hi, 'Z');
      out.push_back({(uint8_t)(lo + 32), (uint8_t)(hi + 32)});
    }
  }
  return bclass_canonicalize(std::move(out));
}

static std::vector<BRange> to_byte_class(const std::vector<CRange> &r) {  // lib.rs:669-674
  std::vector<BRange> out;
  for (const CRange &c : r) {
    if (c.lo > 0xFF) continue;
    out.push_back({(uint8_t)c.lo, (uint8_t)std::min<uint32_t>(c.hi, 0xFF)});
  }
  return bclass_canonicalize(std::move(out));
}

// ------------------------------------------------------- Expr predicates
static bool rep_matches_empty(const Expr &e) {
  switch (e.rep) {
    case Rep::ZeroOrOne: case Rep::ZeroOrMore: return true;
    case Rep::OneOrMore: return false;
    case Rep::Range: return e.rmin == 0;
  }
  return false;
}

bool Expr::can_repeat() const {  // lib.rs:411-423
  switch (kind) {
    case EK::Empty: case EK::Repeat: case EK::Concat: case EK::Alternate:
      return false;
    default: return true;
  }
}
bool Expr::is_anchored_start() const {  // lib.rs:518-529
  switch (kind) {
    case EK::Repeat: return !rep_matches_empty(*this) && subs[0].is_anchored_start();
    case EK::Group: return subs[0].is_anchored_start();
    case EK::Concat: return subs[0].is_anchored_start();
    case EK::Alternate:
      for (const Expr &e : subs) if (!e.is_anchored_start()) return false;
      return true;
    case EK::StartText: return true;
    default: return false;
  }
}
bool Expr::has_anchored_start() const {  // lib.rs:533-544
  switch (kind) {
    case EK::Repeat: return !rep_matches_empty(*this) && subs[0].has_anchored_start();
    case EK::Group: return subs[0].has_anchored_start();
    case EK::Concat: return subs[0].has_anchored_start();
    case EK::Alternate:
      for (const Expr &e : subs) if (e.has_anchored_start()) return true;
      return false;
    case EK::StartText: return true;
    default: return false;
  }
}
bool Expr::is_anchored_end() const {  // lib.rs:548-559
  switch (kind) {
    case EK::Repeat: return !rep_matches_empty(*this) && subs[0].is_anchored_end();
    case EK::Group: return subs[0].is_anchored_end();
    case EK::Concat: return subs.back().is_anchored_end();
    case EK::Alternate:
      for (const Expr &e : subs) if (!e.is_anchored_end()) return false;
      return true;
    case EK::EndText: return true;
    default: return false;
  }
}
bool Expr::has_anchored_end() const {  // lib.rs:563-574
  switch (kind) {
    case EK::Repeat: return !rep_matches_empty(*this) && subs[0].has_anchored_end();
    case EK::Group: return subs[0].has_anchored_end();
    case EK::Concat: return subs.back().has_anchored_end();
    case EK::Alternate:
      for (const Expr &e : subs) if (e.has_anchored_end()) return true;
      return false;
    case EK::EndText: return true;
    default: return false;
  }
}
bool Expr::has_bytes() const {  // lib.rs:578-590
  switch (kind) {
    case EK::Repeat: case EK::Group: return subs[0].has_bytes();
    case EK::Concat: case EK::Alternate:
      for (const Expr &e : subs) if (e.has_bytes()) return true;
      return false;
    case EK::LiteralBytes: case EK::AnyByte: case EK::AnyByteNoNL:
    case EK::ClassBytes: case EK::WordBoundaryAscii: case EK::NotWordBoundaryAscii:
      return true;
    default: return false;
  }
}

// ------------------------------------------------------------- parser
namespace {

struct ParseError { std::string msg; };

static bool is_punct(uint32_t c) {  // parser.rs:1378-1384
  switch (c) {
    case '\\': case '.': case '+': case '*': case '?': case '(': case ')':
    case '|': case '[': case ']': case '{': case '}': case '^': case '$':
    case '#': case '&': case '-': case '~': return true;
    default: return false;
  }
}
static bool is_ascii_word(uint32_t c) {
  return c < 0x80 && is_word_byte((uint8_t)c);
}

struct AsciiClass { const char *name; std::vector<CRange> r; };
static const std::vector<AsciiClass> &ascii_classes() {  // parser.rs:1410-1458
  static const std::vector<AsciiClass> k = {
      {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
      {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
      {"ascii", {{0x00, 0x7F}}},
      {"blank", {{' ', ' '}, {'\t', '\t'}}},
      {"cntrl", {{0x00, 0x1F}, {0x7F, 0x7F}}},
      {"digit", {{'0', '9'}}},
      {"graph", {{'!', '~'}}},
      {"lower", {{'a', 'z'}}},
      {"print", {{' ', '~'}}},
      {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
      {"space", {{'\t', '\t'}, {'\n', '\n'}, {0x0B, 0x0B}, {0x0C, 0x0C}, {'\r', '\r'}, {' ', ' '}}},
      {"upper", {{'A', 'Z'}}},
      {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
      {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
  };
  return k;
}
static bool ascii_class(const std::string &name, std::vector<CRange> *out) {
  for (const AsciiClass &a : ascii_classes())
    if (name == a.name) { *out = a.r; return true; }
  return false;
}
static bool unicode_class(const std::string &name, std::vector<CRange> *out) {
  for (unsigned i = 0; i < U::kNumClasses; ++i)
    if (name == U::kClasses[i].name) { *out = table_class(U::kClasses[i].span); return true; }
  return false;
}

struct Build {
  bool is_paren = false;
  Expr e;
  int cap = -1;
  bool has_name = false;
  std::string name;
  size_t chari = 0;
  SyntaxFlags old_flags;
};

struct Bracket {
  enum K { Left, Set, Inter } k;
  bool negated = false;
  std::vector<CRange> cls;
};

class Parser {
 public:
  Parser(std::vector<uint32_t> chars, SyntaxFlags f) : c_(std::move(chars)), flags_(f) {}

  Expr parse_expr() {  // parser.rs:122-188
    while (true) {
      ignore_space();
      if (eof()) break;
      Build b;
      uint32_t ch = cur();
      switch (ch) {
        case '\\': b = parse_escape(); break;
        case '|': b = alternate(); bump(); break;
        case '?': b = parse_simple_repeat(Rep::ZeroOrOne); break;
        case '*': b = parse_simple_repeat(Rep::ZeroOrMore); break;
        case '+': b = parse_simple_repeat(Rep::OneOrMore); break;
        case '{': b = parse_counted_repeat(); break;
        case '[': b = parse_class(); break;
        case '^': b = one(flags_.multi ? EK::StartLine : EK::StartText); break;
        case '$': b = one(flags_.multi ? EK::EndLine : EK::EndText); break;
        case '.':
          if (flags_.dotnl) {
            if (flags_.unicode) b = one(EK::AnyChar);
            else { if (!flags_.allow_bytes) fail("invalid UTF-8"); b = one(EK::AnyByte); }
          } else {
            if (flags_.unicode) b = one(EK::AnyCharNoNL);
            else { if (!flags_.allow_bytes) fail("invalid UTF-8"); b = one(EK::AnyByteNoNL); }
          }
          break;
        case '(': b = parse_group(); break;
        case ')': {
          SyntaxFlags old;
          b = close_paren(&old);
          bump();
          flags_ = old;
          break;
        }
        default: { uint32_t c = bump(); b = lit(c); break; }
      }
      if (b.is_paren || b.e.kind != EK::Empty) stack_.push_back(std::move(b));
    }
    return finish_concat();
  }

 private:
  std::vector<uint32_t> c_;
  size_t i_ = 0;
  std::vector<Build> stack_;
  int caps_ = 0;
  std::vector<std::string> names_;
  SyntaxFlags flags_;

  [[noreturn]] void fail(const std::string &m) {
    throw ParseError{"regex parse error at position " + std::to_string(i_) + ": " + m};
  }
  bool eof() const { return i_ >= c_.size(); }
  uint32_t cur() const { return c_[i_]; }
  uint32_t bump() { return c_[i_++]; }
  bool peek_is(uint32_t ch) const { return !eof() && c_[i_] == ch; }
  bool peek_str(const char *s) const {
    size_t n = strlen(s);
    if (i_ + n > c_.size()) return false;
    for (size_t k = 0; k < n; ++k) if (c_[i_ + k] != (uint8_t)s[k]) return false;
    return true;
  }
  bool bump_if(uint32_t ch) { if (peek_is(ch)) { ++i_; return true; } return false; }
  bool bump_if_str(const char *s) { if (peek_str(s)) { i_ += strlen(s); return true; } return false; }
  template <class F> std::vector<uint32_t> bump_get(F f) {
    size_t s = i_;
    while (i_ < c_.size() && f(c_[i_])) ++i_;
    return std::vector<uint32_t>(c_.begin() + s, c_.begin() + i_);
  }
  static std::string to_ascii(const std::vector<uint32_t> &v) {
    std::string s;
    for (uint32_t x : v) {
      if (x < 0x80) s.push_back((char)x);
      else s.push_back('\x01');  // never valid in names or numbers
    }
    return s;
  }

  void ignore_space() {  // parser.rs:894-916
    if (!flags_.ignore_space) return;
    while (!eof()) {
      uint32_t ch = cur();
      if (ch == '#') {
        bump();
        while (!eof()) { if (bump() == '\n') break; }
      } else if (is_whitespace(ch)) {
        bump();
      } else {
        return;
      }
    }
  }

  Build one(EK k) { bump(); Build b; b.e.kind = k; return b; }
  Build expr_build(Expr e) { Build b; b.e = std::move(e); return b; }

  Build lit(uint32_t ch) {  // parser.rs:1025-1037
    Expr e;
    if (flags_.unicode) {
      e.kind = EK::Literal; e.chars = {ch}; e.casei = flags_.casei;
    } else {
      e.kind = EK::LiteralBytes; e.bytes = {codepoint_to_one_byte(ch)}; e.casei = flags_.casei;
    }
    return expr_build(std::move(e));
  }
  uint8_t codepoint_to_one_byte(uint32_t ch) {  // parser.rs:993-1000
    if (ch > 0x7F) fail("Unicode not allowed here");
    return (uint8_t)ch;
  }
  Build u32_to_one_byte(uint32_t b) {  // parser.rs:1008-1020
    if (b > 0xFF) fail("Unicode not allowed here");
    if (!flags_.allow_bytes && b > 0x7F) fail("invalid UTF-8");
    Expr e;
    e.kind = EK::LiteralBytes; e.bytes = {(uint8_t)b}; e.casei = flags_.casei;
    return expr_build(std::move(e));
  }

  std::vector<CRange> class_transform(bool negate, std::vector<CRange> cls) {  // parser.rs:979-987
    if (flags_.casei) cls = class_case_fold(cls);
    if (negate) cls = class_negate(std::move(cls));
    return cls;
  }

  Build class_expr(std::vector<CRange> cls) {
    Expr e; e.kind = EK::Class; e.cls = std::move(cls);
    return expr_build(std::move(e));
  }

  Build parse_escape() {  // parser.rs:194-242
    bump();
    if (eof()) fail("unexpected end of escape sequence");
    uint32_t ch = cur();
    if (is_punct(ch) || (flags_.ignore_space && is_whitespace(ch))) {
      uint32_t c2 = bump();
      return lit(c2);
    }
    switch (ch) {
      case 'a': bump(); return lit(0x07);
      case 'f': bump(); return lit(0x0C);
      case 't': bump(); return lit('\t');
      case 'n': bump(); return lit('\n');
      case 'r': bump(); return lit('\r');
      case 'v': bump(); return lit(0x0B);
      case 'A': { bump(); Expr e; e.kind = EK::StartText; return expr_build(e); }
      case 'z': { bump(); Expr e; e.kind = EK::EndText; return expr_build(e); }
      case 'b': { bump(); Expr e; e.kind = flags_.unicode ? EK::WordBoundary : EK::WordBoundaryAscii; return expr_build(e); }
      case 'B': { bump(); Expr e; e.kind = flags_.unicode ? EK::NotWordBoundary : EK::NotWordBoundaryAscii; return expr_build(e); }
      case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7':
        return parse_octal();
      case 'x': bump(); return parse_hex();
      case 'p': case 'P': bump(); return class_expr(parse_unicode_class(ch == 'P'));
      case 'd': case 's': case 'w': case 'D': case 'S': case 'W':
        bump(); return class_expr(parse_perl_class(ch));
      default: fail("unrecognized escape sequence");
    }
  }

  Build parse_group() {  // parser.rs:253-280
    size_t chari = i_;
    bool has_name = false;
    std::string name;
    bump();
    ignore_space();
    if (bump_if_str("?P<")) {
      name = parse_group_name();
      for (const std::string &n : names_) if (n == name) fail("duplicate capture group name");
      names_.push_back(name);
      has_name = true;
    } else if (bump_if('?')) {
      return parse_group_flags(chari);
    }
    caps_ += 1;
    Build b;
    b.is_paren = true; b.cap = caps_; b.has_name = has_name; b.name = name;
    b.chari = chari; b.old_flags = flags_;
    return b;
  }

  Build parse_group_flags(size_t opening) {  // parser.rs:291-352
    SyntaxFlags old = flags_;
    bool sign = true, saw = false;
    while (true) {
      if (eof()) fail("unexpected end of flags");
      uint32_t ch = cur();
      switch (ch) {
        case 'i': flags_.casei = sign; saw = true; break;
        case 'm': flags_.multi = sign; saw = true; break;
        case 's': flags_.dotnl = sign; saw = true; break;
        case 'U': flags_.swap_greed = sign; saw = true; break;
        case 'x': flags_.ignore_space = sign; saw = true; break;
        case 'u': flags_.unicode = sign; saw = true;
          break;
        case '-':
          if (!sign) fail("double flag negation");
          sign = false; saw = false; break;
        case ')': {
          if (!saw) fail("empty flag negation");
          bump();
          Build b; b.e.kind = EK::Empty; return b;
        }
        case ':': {
          if (!sign && !saw) fail("empty flag negation");
          bump();
          Build b; b.is_paren = true; b.cap = -1; b.chari = opening; b.old_flags = old;
          return b;
        }
        default: fail("unrecognized flag");
      }
      bump();
    }
  }

  std::string parse_group_name() {  // parser.rs:358-381
    std::vector<uint32_t> v;
    while (!eof() && !peek_is('>')) v.push_back(bump());
    if (eof()) fail("unclosed capture group name");
    if (v.empty()) fail("empty capture group name");
    bool valid = true;
    for (uint32_t x : v) if (!is_ascii_word(x)) valid = false;
    if ((v[0] >= '0' && v[0] <= '9') || !valid) fail("invalid capture group name");
    bump();
    return to_ascii(v);
  }

  Expr pop_expr() {
    if (stack_.empty() || stack_.back().is_paren) fail("repetition operator missing expression");
    Expr e = std::move(stack_.back().e);
    stack_.pop_back();
    return e;
  }

  uint32_t parse_decimal() {  // parser.rs:451-463
    std::vector<uint32_t> v = bump_get([](uint32_t x) { return is_ascii_word(x) || is_whitespace(x); });
    if (v.empty()) fail("missing base 10 number");
    // trim (Unicode whitespace)
    size_t a = 0, b = v.size();
    while (a < b && is_whitespace(v[a])) ++a;
    while (b > a && is_whitespace(v[b - 1])) --b;
    if (a == b) fail("invalid base 10 number");
    size_t k = a;
    if (v[k] == '+') ++k;  // Rust from_str_radix accepts a leading '+'
    if (k == b) fail("invalid base 10 number");
    uint64_t n = 0;
    for (; k < b; ++k) {
      if (v[k] < '0' || v[k] > '9') fail("invalid base 10 number");
      n = n * 10 + (v[k] - '0');
      if (n > 0xFFFFFFFFull) fail("invalid base 10 number");
    }
    return (uint32_t)n;
  }

  Build parse_counted_repeat() {  // parser.rs:387-424
    Expr e = pop_expr();
    if (!e.can_repeat()) fail("repetition operator applied to a non-repeatable expression");
    bump();
    ignore_space();
    uint32_t mn = parse_decimal();
    uint32_t mx = mn;
    bool has_max = true;
    ignore_space();
    if (bump_if(',')) {
      ignore_space();
      if (peek_is('}')) {
        has_max = false;
      } else {
        mx = parse_decimal();
        if (mn > mx) fail("invalid repeat range");
      }
    }
    ignore_space();
    if (!bump_if('}')) fail("unclosed counted repetition");
    Expr r;
    r.kind = EK::Repeat; r.rep = Rep::Range; r.rmin = mn; r.rmax = mx; r.has_max = has_max;
    r.greedy = (!bump_if('?')) ^ flags_.swap_greed;
    r.subs.push_back(std::move(e));
    return expr_build(std::move(r));
  }

  Build parse_simple_repeat(Rep rep) {  // parser.rs:433-445
    Expr e = pop_expr();
    if (!e.can_repeat()) fail("repetition operator applied to a non-repeatable expression");
    bump();
    Expr r;
    r.kind = EK::Repeat; r.rep = rep;
    r.greedy = (!bump_if('?')) ^ flags_.swap_greed;
    r.subs.push_back(std::move(e));
    return expr_build(std::move(r));
  }

  Build parse_octal() {  // parser.rs:469-488
    int k = 0;
    std::vector<uint32_t> v = bump_get([&k](uint32_t x) { ++k; return k <= 3 && x >= '0' && x <= '7'; });
    uint32_t n = 0;
    for (uint32_t x : v) n = n * 8 + (x - '0');
    if (!flags_.unicode) return u32_to_one_byte(n);
    return lit(n);
  }

  static bool hex_value(const std::vector<uint32_t> &v, uint32_t *out) {
    if (v.empty()) return false;
    size_t k = 0;
    if (v[0] == '+') k = 1;
    if (k == v.size()) return false;
    uint64_t n = 0;
    for (; k < v.size(); ++k) {
      uint32_t x = v[k], d;
      if (x >= '0' && x <= '9') d = x - '0';
      else if (x >= 'a' && x <= 'f') d = x - 'a' + 10;
      else if (x >= 'A' && x <= 'F') d = x - 'A' + 10;
      else return false;
      n = n * 16 + d;
      if (n > 0xFFFFFFFFull) return false;
    }
    *out = (uint32_t)n;
    return true;
  }

  Build parse_hex() {  // parser.rs:499-553
    ignore_space();
    if (bump_if('{')) {
      ignore_space();
      std::vector<uint32_t> s = bump_get(is_ascii_word);
      uint32_t n;
      if (!hex_value(s, &n)) fail("invalid base 16 number");
      ignore_space();
      if (!bump_if('}')) fail("unclosed hexadecimal literal");
      if (!flags_.unicode) return u32_to_one_byte(n);
      if (n > kMaxChar || (n >= 0xD800 && n <= 0xDFFF)) fail("invalid Unicode scalar value");
      return lit(n);
    }
    int k = 0;
    std::vector<uint32_t> s = bump_get([&k](uint32_t) { ++k; return k <= 2; });
    if (s.size() < 2) fail("unexpected end of two-digit hex");
    uint32_t n;
    if (!hex_value(s, &n)) fail("invalid base 16 number");
    if (!flags_.unicode) return u32_to_one_byte(n);
    return lit(n);
  }

  Build parse_class() {  // parser.rs:562-580
    std::vector<CRange> cls = parse_class_as_chars();
    if (flags_.unicode) return class_expr(std::move(cls));
    std::vector<BRange> bc = to_byte_class(cls);
    if (bc.empty()) fail("empty class");
    Expr e; e.kind = EK::ClassBytes; e.bcls = std::move(bc);
    return expr_build(std::move(e));
  }

  std::vector<Bracket> parse_open_bracket() {  // parser.rs:653-677
    bump();
    ignore_space();
    bool neg = bump_if('^');
    ignore_space();
    std::vector<CRange> cls;
    while (bump_if('-')) { cls.push_back({'-', '-'}); ignore_space(); }
    if (cls.empty()) {
      if (bump_if(']')) { cls.push_back({']', ']'}); ignore_space(); }
    }
    std::vector<Bracket> out;
    Bracket l; l.k = Bracket::Left; l.negated = neg;
    out.push_back(l);
    if (!cls.empty()) { Bracket s; s.k = Bracket::Set; s.cls = cls; out.push_back(s); }
    return out;
  }

  std::vector<CRange> parse_class_as_chars() {  // parser.rs:586-643
    std::vector<Bracket> st;
    for (Bracket &b : parse_open_bracket()) st.push_back(std::move(b));
    while (true) {
      ignore_space();
      if (eof()) fail("unexpected end of character class");
      uint32_t ch = cur();
      if (ch == '[') {
        std::vector<CRange> a;
        if (maybe_parse_ascii(&a)) {
          Bracket s; s.k = Bracket::Set; s.cls = std::move(a); st.push_back(std::move(s));
        } else {
          for (Bracket &b : parse_open_bracket()) st.push_back(std::move(b));
        }
      } else if (ch == ']') {
        bump();
        std::vector<CRange> cls = close_bracket(&st);
        if (st.empty()) return cls;
        Bracket s; s.k = Bracket::Set; s.cls = std::move(cls); st.push_back(std::move(s));
      } else if (ch == '\\') {
        Bracket s; s.k = Bracket::Set; s.cls = parse_class_escape(); st.push_back(std::move(s));
      } else if (ch == '&' && peek_str("&&")) {
        bump(); bump();
        Bracket s; s.k = Bracket::Inter; st.push_back(std::move(s));
      } else {
        uint32_t start = ch;
        if (!flags_.unicode) codepoint_to_one_byte(start);
        bump();
        if ((start == '~' || start == '-') && peek_is(start)) fail("unsupported class character");
        Bracket s; s.k = Bracket::Set; s.cls = parse_class_range(start); st.push_back(std::move(s));
      }
    }
  }

  std::vector<CRange> parse_class_escape() {  // parser.rs:688-716
    Build b = parse_escape();
    Expr &e = b.e;
    switch (e.kind) {
      case EK::Class: return e.cls;
      case EK::ClassBytes: {
        std::vector<CRange> out;
        for (const BRange &r : e.bcls) out.push_back({r.lo, r.hi});
        return out;
      }
      case EK::Literal: return parse_class_range(e.chars[0]);
      case EK::LiteralBytes: return parse_class_range(e.bytes[0]);
      default: fail("invalid escape sequence in character class");
    }
  }

  std::vector<CRange> parse_class_range(uint32_t start) {  // parser.rs:724-776
    ignore_space();
    if (!bump_if('-')) return {{start, start}};
    ignore_space();
    if (eof()) fail("unexpected end of character class");
    if (peek_is(']')) return {{start, start}, {'-', '-'}};
    uint32_t end;
    if (cur() == '\\') {
      Build b = parse_escape();
      if (b.e.kind == EK::Literal) end = b.e.chars[0];
      else if (b.e.kind == EK::LiteralBytes) end = b.e.bytes[0];
      else fail("invalid escape sequence in character class");
    } else {
      uint32_t c2 = bump();
      if (c2 == '-') fail("unsupported class character");
      if (!flags_.unicode) codepoint_to_one_byte(c2);
      end = c2;
    }
    if (end < start) fail("invalid character class range");
    return {{start, end}};
  }

  bool maybe_parse_ascii(std::vector<CRange> *out) {  // parser.rs:791-808
    size_t start = i_;
    bump();
    if (bump_if(':')) {
      bool neg = bump_if('^');
      std::vector<uint32_t> name = bump_get([](uint32_t x) { return x != ':'; });
      if (!name.empty() && bump_if_str(":]")) {
        std::vector<CRange> c;
        if (ascii_class(to_ascii(name), &c)) { *out = class_transform(neg, c); return true; }
      }
    }
    i_ = start;
    return false;
  }

  std::vector<CRange> parse_unicode_class(bool neg) {  // parser.rs:821-850
    ignore_space();
    std::string name;
    if (bump_if('{')) {
      ignore_space();
      std::vector<uint32_t> n = bump_get(is_ascii_word);
      ignore_space();
      if (n.empty() || !bump_if('}')) fail("unclosed Unicode class name");
      name = to_ascii(n);
    } else {
      if (eof()) fail("unexpected end of escape sequence");
      uint32_t x = bump();
      name = to_ascii({x});
    }
    std::vector<CRange> c;
    if (!unicode_class(name, &c)) fail("unrecognized Unicode class name");
    if (!flags_.unicode) fail("Unicode not allowed here");
    return class_transform(neg, c);
  }

  std::vector<CRange> parse_perl_class(uint32_t name) {  // parser.rs:857-875
    std::vector<CRange> c;
    bool neg = (name == 'D' || name == 'S' || name == 'W');
    uint32_t lower = neg ? name + 32 : name;
    if (flags_.unicode) {
      if (lower == 'd') c = table_class(U::kPerlD);
      else if (lower == 's') c = table_class(U::kPerlS);
      else c = table_class(U::kPerlW);
    } else {
      ascii_class(lower == 'd' ? "digit" : lower == 's' ? "space" : "word", &c);
    }
    return class_transform(neg, c);
  }

  std::vector<CRange> class_union_transform(std::vector<CRange> c) {  // parser.rs:1285-1292
    if (flags_.casei) return class_case_fold(c);
    return class_canonicalize(std::move(c));
  }

  std::vector<CRange> close_bracket(std::vector<Bracket> *st) {  // parser.rs:1249-1281
    std::vector<CRange> uni;
    std::vector<std::vector<CRange>> inter;
    while (true) {
      Bracket b = std::move(st->back());
      st->pop_back();
      if (b.k == Bracket::Set) {
        uni.insert(uni.end(), b.cls.begin(), b.cls.end());
      } else if (b.k == Bracket::Inter) {
        inter.push_back(class_union_transform(std::move(uni)));
        uni.clear();
      } else {
        std::vector<CRange> cls = class_union_transform(std::move(uni));
        for (auto &c : inter) cls = class_intersect(cls, c);
        if (b.negated) cls = class_negate(std::move(cls));
        if (cls.empty()) fail("empty character class");
        return cls;
      }
    }
  }

  static Expr rev_concat(std::vector<Expr> v) {  // parser.rs:1352-1361
    Expr e;
    if (v.empty()) return e;
    if (v.size() == 1) return std::move(v[0]);
    std::reverse(v.begin(), v.end());
    e.kind = EK::Concat;
    e.subs = std::move(v);
    return e;
  }

  Build alternate() {  // parser.rs:1098-1129
    std::vector<Expr> concat;
    auto alts = [this](std::vector<Expr> es) {
      Expr e; e.kind = EK::Alternate; e.subs = std::move(es);
      return expr_build(std::move(e));
    };
    while (true) {
      if (stack_.empty()) {
        if (concat.empty()) fail("empty alternate");
        std::vector<Expr> es; es.push_back(rev_concat(std::move(concat)));
        return alts(std::move(es));
      }
      Build b = std::move(stack_.back());
      stack_.pop_back();
      if (b.is_paren) {
        if (concat.empty()) fail("empty alternate");
        stack_.push_back(std::move(b));
        std::vector<Expr> es; es.push_back(rev_concat(std::move(concat)));
        return alts(std::move(es));
      }
      if (b.e.kind == EK::Alternate) {
        if (concat.empty()) fail("empty alternate");
        b.e.subs.push_back(rev_concat(std::move(concat)));
        return alts(std::move(b.e.subs));
      }
      concat.push_back(std::move(b.e));
    }
  }

  Build close_paren(SyntaxFlags *old) {  // parser.rs:1153-1192
    std::vector<Expr> concat;
    while (true) {
      if (stack_.empty()) fail("unopened parenthesis");
      Build b = std::move(stack_.back());
      stack_.pop_back();
      if (b.is_paren) {
        if (concat.empty()) fail("empty group");
        *old = b.old_flags;
        Expr g; g.kind = EK::Group; g.cap = b.cap; g.has_name = b.has_name; g.name = b.name;
        g.subs.push_back(rev_concat(std::move(concat)));
        return expr_build(std::move(g));
      }
      if (b.e.kind == EK::Alternate) {
        if (concat.empty()) fail("empty alternate");
        b.e.subs.push_back(rev_concat(std::move(concat)));
        if (stack_.empty()) fail("unopened parenthesis");
        Build p = std::move(stack_.back());
        stack_.pop_back();
        *old = p.old_flags;
        Expr g; g.kind = EK::Group; g.cap = p.cap; g.has_name = p.has_name; g.name = p.name;
        g.subs.push_back(std::move(b.e));
        return expr_build(std::move(g));
      }
      concat.push_back(std::move(b.e));
    }
  }

  Expr finish_concat() {  // parser.rs:1207-1236
    std::vector<Expr> concat;
    while (true) {
      if (stack_.empty()) return rev_concat(std::move(concat));
      Build b = std::move(stack_.back());
      stack_.pop_back();
      if (b.is_paren) { i_ = b.chari; fail("unclosed parenthesis"); }
      if (b.e.kind == EK::Alternate) {
        if (concat.empty()) fail("empty alternate");
        b.e.subs.push_back(rev_concat(std::move(concat)));
        if (!stack_.empty()) { i_ = stack_.back().chari; fail("unclosed parenthesis"); }
        return std::move(b.e);
      }
      concat.push_back(std::move(b.e));
    }
  }
};

// lib.rs:425-500
static void combine_literals(std::vector<Expr> &es, Expr e) {
  if (!es.empty()) {
    Expr &last = es.back();
    if (last.kind == EK::Literal && e.kind == EK::Literal && last.casei == e.casei) {
      last.chars.insert(last.chars.end(), e.chars.begin(), e.chars.end());
      return;
    }
    if (last.kind == EK::LiteralBytes && e.kind == EK::LiteralBytes && last.casei == e.casei) {
      last.bytes.insert(last.bytes.end(), e.bytes.begin(), e.bytes.end());
      return;
    }
  }
  es.push_back(std::move(e));
}

static Expr simplify(Expr e, size_t depth, size_t limit) {
  if (depth > limit) throw ParseError{"regex parse error: exceeded the maximum nesting depth"};
  switch (e.kind) {
    case EK::Repeat: {
      e.subs[0] = simplify(std::move(e.subs[0]), depth + 1, limit);
      return e;
    }
    case EK::Group: {
      Expr in = simplify(std::move(e.subs[0]), depth + 1, limit);
      if (e.cap < 0 && !e.has_name && in.can_repeat()) return in;
      e.subs[0] = std::move(in);
      return e;
    }
    case EK::Concat: {
      std::vector<Expr> es;
      for (Expr &s : e.subs) combine_literals(es, simplify(std::move(s), depth + 1, limit));
      if (es.size() == 1) return std::move(es[0]);
      e.subs = std::move(es);
      return e;
    }
    case EK::Alternate: {
      for (Expr &s : e.subs) s = simplify(std::move(s), depth + 1, limit);
      return e;
    }
    default: return e;
  }
}

}  // namespace

bool parse_regex(const std::string &pat, SyntaxFlags flags, Expr *out, std::string *err) {
  std::vector<uint32_t> chars;
  const uint8_t *p = (const uint8_t *)pat.data();
  size_t n = pat.size(), i = 0;
  while (i < n) {
    uint32_t cp; size_t len;
    if (!decode_utf8(p + i, n - i, &cp, &len)) {
      if (err) *err = "pattern is not valid UTF-8";
      return false;
    }
    chars.push_back(cp);
    i += len;
  }
  try {
    Parser ps(std::move(chars), flags);
    Expr e = ps.parse_expr();
    *out = simplify(std::move(e), 0, 200);
    return true;
  } catch (const ParseError &pe) {
    if (err) *err = pe.msg;
    return false;
  }
}

}  // namespace rure_amd
