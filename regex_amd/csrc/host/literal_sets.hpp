// Literal prefix / suffix extraction and the engine choice that depends on it.
//
// Restates regex-syntax 0.4's `Literals` (regex-syntax/src/literals.rs:
// prefixes 573-642, suffixes 644-718, repeats 720-815, alternations 817-840,
// union / cross products 271-430, unambiguous_prefixes 206-257), the literal
// sets the reference builds per regex (src/exec.rs:209-271, 308-321), the
// searcher properties it reads off them (src/literals.rs:70-88, 145-170,
// 186-250: complete, len, lcp, lcs, char_len) and choose_match_type
// (src/exec.rs:1130-1210).
//
// The engine choice is observable: MatchType::Literal(AnchoredStart) tests
// the literals at the search start whatever it is (exec.rs:613-617,
// literals.rs:105-115: `^abc` finds (1, 4) in "xabc" from start 1 and
// iterates "abcabc" as two matches), and DfaSuffix (exec.rs:725-794)
// reports the first suffix occurrence whose reverse scan matches, which can
// start after the leftmost-first match when a longer match spans an earlier
// occurrence.  Both are reproduced on the GPU, so the match type is computed
// exactly as the reference computes it.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "syntax.hpp"

namespace rure_amd {

struct Lit {
  std::string v;
  bool cut = false;
};

struct Literals {
  std::vector<Lit> lits;
  size_t limit_size = 250, limit_class = 10;

  bool all_complete() const;
  bool any_complete() const;
  bool contains_empty() const;
  bool is_empty() const;
  size_t num_bytes() const;
  Literals to_empty() const;
  std::string longest_common_prefix() const;
  std::string longest_common_suffix() const;
  Literals unambiguous_prefixes() const;
  Literals unambiguous_suffixes() const;
  bool union_prefixes(const Expr &e);
  bool union_suffixes(const Expr &e);
  bool union_with(Literals other);
  bool cross_product(const Literals &other);
  bool cross_add(const std::string &bytes);
  bool add(const Lit &l);
  bool add_char_class(const std::vector<CRange> &cls, bool reverse);
  bool add_byte_class(const std::vector<BRange> &cls);
  void cut();
  void reverse();
  std::vector<Lit> remove_complete();
  bool class_exceeds_limits(size_t size) const;
};

// regex-syntax's `prefixes(expr, lits)` / `suffixes(expr, lits)` (the
// suffix literals come out reversed, as there).
void literal_prefixes(const Expr &e, Literals *lits);
void literal_suffixes(const Expr &e, Literals *lits);

// A LiteralSearcher's properties (src/literals.rs).
struct LitSearcher {
  Literals lits;          // the unambiguous set it was built from
  int matcher = 0;        // 0 Empty, 1 Bytes, 2 single literal, 3 several (Teddy / AC)
  size_t len = 0;         // len(): Bytes -> distinct bytes, single -> 1, several -> literals
  bool complete = false;  // complete(): all literals complete and len() > 0
  std::string lcp, lcs;
  size_t lcp_chars = 0, lcs_chars = 0;   // char_len (String::from_utf8_lossy)
};
LitSearcher make_searcher(const Literals &lits, bool suffix);

// MatchType (src/exec.rs:1213-1245) for one regex.
enum MatchTypeCode : int {
  MT_LITERAL_UNANCHORED = 0,
  MT_LITERAL_ANCHORED_START = 1,
  MT_LITERAL_ANCHORED_END = 2,
  MT_DFA = 3,
  MT_DFA_ANCHORED_REVERSE = 4,
  MT_DFA_SUFFIX = 5,
  MT_NFA = 6,
  MT_NOTHING = 7,
};

struct ExecLiterals {
  LitSearcher prefixes;   // nfa.prefixes == dfa.prefixes (exec.rs:308-311)
  LitSearcher suffixes;   // exec.rs:309, 320
  int match_type = MT_DFA;
};
// The literal sets and match type of a single regex (exec.rs:209-271 with
// one pattern, 308-321, 1130-1188); the DFA is assumed executable
// (dfa::can_exec holds for every program this compiler emits).
ExecLiterals exec_literals(const Expr &e);

size_t char_len_lossy(const std::string &bytes);

}  // namespace rure_amd
