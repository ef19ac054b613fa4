// Host-side regex syntax: pattern text -> expression tree.
//
// Restates the behaviour of the reference parser `regex-syntax` 0.4.2
// (regex-syntax/src/parser.rs:107-1405, lib.rs:97-591, lib.rs:610-1134) for
// the byte-regex configuration used by `regex::bytes::Regex` and the `rure`
// C API (allow_bytes = true, Unicode on by default).  Unicode classes come
// from the reference's own Unicode 10 tables (unicode_tables.h).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace rure_amd {

struct CRange { uint32_t lo, hi; };   // inclusive Unicode scalar range
struct BRange { uint8_t lo, hi; };    // inclusive byte range

enum class EK : uint8_t {
  Empty, Literal, LiteralBytes, AnyChar, AnyCharNoNL, AnyByte, AnyByteNoNL,
  Class, ClassBytes, StartLine, EndLine, StartText, EndText,
  WordBoundary, NotWordBoundary, WordBoundaryAscii, NotWordBoundaryAscii,
  Group, Repeat, Concat, Alternate,
};

enum class Rep : uint8_t { ZeroOrOne, ZeroOrMore, OneOrMore, Range };

struct Expr {
  EK kind = EK::Empty;
  bool casei = false;
  std::vector<uint32_t> chars;   // Literal
  std::vector<uint8_t> bytes;    // LiteralBytes
  std::vector<CRange> cls;       // Class (canonical)
  std::vector<BRange> bcls;      // ClassBytes (canonical)
  int cap = -1;                  // Group capture index (-1: non-capturing)
  bool has_name = false;
  std::string name;
  Rep rep = Rep::ZeroOrOne;      // Repeat
  uint32_t rmin = 0, rmax = 0;
  bool has_max = false;
  bool greedy = true;
  std::vector<Expr> subs;        // Group/Repeat: 1; Concat/Alternate: n

  bool can_repeat() const;
  bool is_anchored_start() const;
  bool has_anchored_start() const;
  bool is_anchored_end() const;
  bool has_anchored_end() const;
  bool has_bytes() const;
};

struct SyntaxFlags {
  bool casei = false, multi = false, dotnl = false, swap_greed = false;
  bool ignore_space = false, unicode = true, allow_bytes = true;
};

// Parses and simplifies (lib.rs:395-397, 425-500).  On error returns false
// and fills `err`.
bool parse_regex(const std::string &pattern_utf8, SyntaxFlags flags,
                 Expr *out, std::string *err);

// Character-class algebra (lib.rs:687-915).
std::vector<CRange> class_canonicalize(std::vector<CRange> r);
std::vector<CRange> class_negate(std::vector<CRange> r);
std::vector<CRange> class_case_fold(const std::vector<CRange> &r);
std::vector<BRange> bclass_canonicalize(std::vector<BRange> r);
std::vector<BRange> bclass_case_fold(const std::vector<BRange> &r);

bool is_word_byte(uint8_t b);        // lib.rs:1746-1751
bool is_word_char(uint32_t c);       // lib.rs:1729-1744 (Unicode PERLW)
bool decode_utf8(const uint8_t *p, size_t n, uint32_t *cp, size_t *len);

}  // namespace rure_amd
