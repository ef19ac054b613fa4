// Literal prefix / suffix sets and the match type.  See literal_sets.hpp.
#include "literal_sets.hpp"

#include <algorithm>
#include <cstring>

namespace rure_amd {
namespace {

// literals.rs:923-933: index of the first occurrence of needle in haystack
long position(const std::string &needle, const std::string &hay) {
  if (needle.size() > hay.size()) return -1;
  for (size_t i = 0; i + needle.size() <= hay.size(); ++i)
    if (memcmp(hay.data() + i, needle.data(), needle.size()) == 0) return (long)i;
  return -1;
}

std::string utf8_of(uint32_t c) {
  std::string s;
  if (c < 0x80) s.push_back((char)c);
  else if (c < 0x800) { s.push_back((char)(0xC0 | (c >> 6))); s.push_back((char)(0x80 | (c & 0x3F))); }
  else if (c < 0x10000) {
    s.push_back((char)(0xE0 | (c >> 12)));
    s.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
    s.push_back((char)(0x80 | (c & 0x3F)));
  } else {
    s.push_back((char)(0xF0 | (c >> 18)));
    s.push_back((char)(0x80 | ((c >> 12) & 0x3F)));
    s.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
    s.push_back((char)(0x80 | (c & 0x3F)));
  }
  return s;
}

bool valid_char(uint32_t c) { return c <= 0x10FFFF && !(c >= 0xD800 && c <= 0xDFFF); }

// Lit's derived Ord: bytes (unsigned, lexicographic), then cut
bool lit_less(const Lit &a, const Lit &b) {
  const size_t n = std::min(a.v.size(), b.v.size());
  const int c = n ? memcmp(a.v.data(), b.v.data(), n) : 0;
  if (c != 0) return c < 0;
  if (a.v.size() != b.v.size()) return a.v.size() < b.v.size();
  return !a.cut && b.cut;
}

void sort_dedup(std::vector<Lit> *v) {
  std::stable_sort(v->begin(), v->end(), lit_less);
  std::vector<Lit> out;
  for (Lit &l : *v)
    if (out.empty() || out.back().v != l.v) out.push_back(std::move(l));
  *v = std::move(out);
}

size_t num_chars(const std::vector<CRange> &cls) {  // lib.rs:792-797
  size_t n = 0;
  for (const CRange &r : cls) n += 1 + r.hi - r.lo;
  return n;
}
size_t num_bytes_cls(const std::vector<BRange> &cls) {  // lib.rs:1071-1076
  size_t n = 0;
  for (const BRange &r : cls) n += 1 + r.hi - r.lo;
  return n;
}

using Extract = void (*)(const Expr &, Literals *);

void repeat_zero_or_one(const Expr &e, Literals *lits, Extract f) {  // literals.rs:720-737
  Literals lits2 = *lits, lits3 = lits->to_empty();
  lits3.limit_size = lits->limit_size / 2;
  f(e, &lits3);
  if (lits3.is_empty() || !lits2.cross_product(lits3)) {
    lits->cut();
    return;
  }
  lits2.add(Lit{});
  if (!lits->union_with(lits2)) lits->cut();
}

void repeat_zero_or_more(const Expr &e, Literals *lits, Extract f) {  // literals.rs:739-757
  Literals lits2 = *lits, lits3 = lits->to_empty();
  lits3.limit_size = lits->limit_size / 2;
  f(e, &lits3);
  if (lits3.is_empty() || !lits2.cross_product(lits3)) {
    lits->cut();
    return;
  }
  lits2.cut();
  lits2.add(Lit{});
  if (!lits->union_with(lits2)) lits->cut();
}

void repeat_one_or_more(const Expr &e, Literals *lits, Extract f) {  // literals.rs:759-766
  f(e, lits);
  lits->cut();
}

void repeat_range(const Expr &e, uint32_t mn, bool has_max, uint32_t mx, bool greedy, Literals *lits,
                  Extract f) {  // literals.rs:768-802
  if (mn == 0) {
    Expr r;
    r.kind = EK::Repeat;
    r.rep = Rep::ZeroOrMore;
    r.greedy = greedy;
    r.subs.push_back(e);
    f(r, lits);
  } else {
    const size_t n = std::min(lits->limit_size, (size_t)mn);
    Expr c;
    c.kind = EK::Concat;
    c.subs.assign(n, e);
    f(c, lits);
    if (n < (size_t)mn || lits->contains_empty()) lits->cut();
    if (!has_max || mn < mx) lits->cut();
  }
}

void alternate(const std::vector<Expr> &es, Literals *lits, Extract f) {  // literals.rs:804-825
  Literals lits2 = lits->to_empty();
  for (const Expr &e : es) {
    Literals lits3 = lits->to_empty();
    lits3.limit_size = lits->limit_size / 5;
    f(e, &lits3);
    if (lits3.is_empty() || !lits2.union_with(lits3)) {
      lits->cut();
      return;
    }
  }
  if (!lits->cross_product(lits2)) lits->cut();
}

std::vector<BRange> fold_byte(uint8_t b) { return bclass_case_fold({BRange{b, b}}); }
std::vector<CRange> fold_char(uint32_t c) { return class_case_fold({CRange{c, c}}); }

void repeat_dispatch(const Expr &e, Literals *lits, Extract f) {
  const Expr &sub = e.subs[0];
  switch (e.rep) {
    case Rep::ZeroOrOne: repeat_zero_or_one(sub, lits, f); break;
    case Rep::ZeroOrMore: repeat_zero_or_more(sub, lits, f); break;
    case Rep::OneOrMore: repeat_one_or_more(sub, lits, f); break;
    case Rep::Range: repeat_range(sub, e.rmin, e.has_max, e.rmax, e.greedy, lits, f); break;
  }
}

}  // namespace

bool Literals::all_complete() const {  // literals.rs:118-120
  if (lits.empty()) return false;
  for (const Lit &l : lits) if (l.cut) return false;
  return true;
}
bool Literals::any_complete() const {
  for (const Lit &l : lits) if (!l.cut) return true;
  return false;
}
bool Literals::contains_empty() const {
  for (const Lit &l : lits) if (l.v.empty()) return true;
  return false;
}
bool Literals::is_empty() const {  // literals.rs:133-135
  for (const Lit &l : lits) if (!l.v.empty()) return false;
  return true;
}
size_t Literals::num_bytes() const {
  size_t n = 0;
  for (const Lit &l : lits) n += l.v.size();
  return n;
}
Literals Literals::to_empty() const {
  Literals o;
  o.limit_size = limit_size;
  o.limit_class = limit_class;
  return o;
}

std::string Literals::longest_common_prefix() const {  // literals.rs:145-160
  if (is_empty()) return std::string();
  const std::string &l0 = lits[0].v;
  size_t len = l0.size();
  for (size_t i = 1; i < lits.size(); ++i) {
    size_t k = 0;
    const std::string &l = lits[i].v;
    while (k < l.size() && k < l0.size() && l[k] == l0[k]) ++k;
    len = std::min(len, k);
  }
  return l0.substr(0, len);
}

std::string Literals::longest_common_suffix() const {  // literals.rs:163-178
  if (is_empty()) return std::string();
  const std::string &l0 = lits[0].v;
  size_t len = l0.size();
  for (size_t i = 1; i < lits.size(); ++i) {
    size_t k = 0;
    const std::string &l = lits[i].v;
    while (k < l.size() && k < l0.size() && l[l.size() - 1 - k] == l0[l0.size() - 1 - k]) ++k;
    len = std::min(len, k);
  }
  return l0.substr(l0.size() - len);
}

Literals Literals::unambiguous_prefixes() const {  // literals.rs:206-257
  if (lits.empty()) return to_empty();
  std::vector<Lit> old = lits;
  Literals nw = to_empty();
  while (!old.empty()) {
    Lit cand = old.back();
    old.pop_back();
    if (cand.v.empty()) continue;
    if (nw.lits.empty()) {
      nw.lits.push_back(cand);
      continue;
    }
    bool next_outer = false;
    for (Lit &lit2 : nw.lits) {
      if (lit2.v.empty()) continue;
      if (cand.v == lit2.v) {
        // duplicates: cut literals are infectious
        cand.cut = cand.cut || lit2.cut;
        lit2.cut = cand.cut;
        next_outer = true;
        break;
      }
      if (cand.v.size() < lit2.v.size()) {
        const long i = position(cand.v, lit2.v);
        if (i >= 0) {
          cand.cut = true;
          Lit lit3 = lit2;
          lit3.v.resize((size_t)i);
          lit3.cut = true;
          old.push_back(lit3);
          lit2.v.clear();
        }
      } else {
        const long i = position(lit2.v, cand.v);
        if (i >= 0) {
          lit2.cut = true;
          Lit nc = cand;
          nc.v.resize((size_t)i);
          nc.cut = true;
          old.push_back(nc);
          cand.v.clear();
        }
      }
      if (cand.v.empty()) {
        next_outer = true;
        break;
      }
    }
    if (next_outer) continue;
    nw.lits.push_back(cand);
  }
  std::vector<Lit> kept;
  for (Lit &l : nw.lits) if (!l.v.empty()) kept.push_back(l);
  sort_dedup(&kept);
  nw.lits = std::move(kept);
  return nw;
}

Literals Literals::unambiguous_suffixes() const {  // literals.rs:268-275
  Literals c = *this;
  c.reverse();
  Literals u = c.unambiguous_prefixes();
  u.reverse();
  return u;
}

bool Literals::union_prefixes(const Expr &e) {  // literals.rs:285-289
  Literals l = to_empty();
  literal_prefixes(e, &l);
  return !l.is_empty() && !l.contains_empty() && union_with(std::move(l));
}

bool Literals::union_suffixes(const Expr &e) {  // literals.rs:299-304
  Literals l = to_empty();
  literal_suffixes(e, &l);
  l.reverse();
  return !l.is_empty() && !l.contains_empty() && union_with(std::move(l));
}

bool Literals::union_with(Literals o) {  // literals.rs:311-322
  if (num_bytes() + o.num_bytes() > limit_size) return false;
  if (o.is_empty()) lits.push_back(Lit{});
  else for (Lit &l : o.lits) lits.push_back(std::move(l));
  return true;
}

bool Literals::cross_product(const Literals &o) {  // literals.rs:331-371
  if (o.is_empty()) return true;
  size_t after;
  if (is_empty() || !any_complete()) {
    after = num_bytes();
    for (const Lit &l : o.lits) after += l.v.size();
  } else {
    after = 0;
    for (const Lit &l : lits) if (l.cut) after += l.v.size();
    for (const Lit &ol : o.lits)
      for (const Lit &sl : lits)
        if (!sl.cut) after += sl.v.size() + ol.v.size();
  }
  if (after > limit_size) return false;
  std::vector<Lit> base = remove_complete();
  if (base.empty()) base.push_back(Lit{});
  for (const Lit &ol : o.lits)
    for (Lit sl : base) {
      sl.v += ol.v;
      sl.cut = ol.cut;
      lits.push_back(std::move(sl));
    }
  return true;
}

bool Literals::cross_add(const std::string &bytes) {  // literals.rs:381-411
  if (bytes.empty()) return true;
  if (lits.empty()) {
    const size_t i = std::min(limit_size, bytes.size());
    lits.push_back(Lit{bytes.substr(0, i), i < bytes.size()});
    return !lits[0].cut;
  }
  const size_t size = num_bytes();
  if (size + lits.size() >= limit_size) return false;
  size_t i = 1;
  while (size + i * lits.size() <= limit_size && i < bytes.size()) ++i;
  for (Lit &l : lits) {
    if (!l.cut) {
      l.v += bytes.substr(0, i);
      if (i < bytes.size()) l.cut = true;
    }
  }
  return true;
}

bool Literals::add(const Lit &l) {  // literals.rs:417-423
  if (num_bytes() + l.v.size() > limit_size) return false;
  lits.push_back(l);
  return true;
}

bool Literals::add_char_class(const std::vector<CRange> &cls, bool reverse) {  // literals.rs:443-470
  if (class_exceeds_limits(num_chars(cls))) return false;
  std::vector<Lit> base = remove_complete();
  if (base.empty()) base.push_back(Lit{});
  for (const CRange &r : cls)
    for (uint64_t c = r.lo; c <= r.hi; ++c) {
      if (!valid_char((uint32_t)c)) continue;
      std::string b = utf8_of((uint32_t)c);
      if (reverse) std::reverse(b.begin(), b.end());
      for (Lit l : base) {
        l.v += b;
        lits.push_back(std::move(l));
      }
    }
  return true;
}

bool Literals::add_byte_class(const std::vector<BRange> &cls) {  // literals.rs:475-493
  if (class_exceeds_limits(num_bytes_cls(cls))) return false;
  std::vector<Lit> base = remove_complete();
  if (base.empty()) base.push_back(Lit{});
  for (const BRange &r : cls)
    for (uint32_t b = r.lo; b <= r.hi; ++b)
      for (Lit l : base) {
        l.v.push_back((char)b);
        lits.push_back(std::move(l));
      }
  return true;
}

void Literals::cut() {
  for (Lit &l : lits) l.cut = true;
}
void Literals::reverse() {
  for (Lit &l : lits) std::reverse(l.v.begin(), l.v.end());
}
std::vector<Lit> Literals::remove_complete() {  // literals.rs:516-527
  std::vector<Lit> base, keep;
  for (Lit &l : lits) (l.cut ? keep : base).push_back(std::move(l));
  lits = std::move(keep);
  return base;
}
bool Literals::class_exceeds_limits(size_t size) const {  // literals.rs:538-570
  if (size > limit_class) return true;
  size_t nb = 0;
  if (lits.empty()) nb = size;
  else for (const Lit &l : lits) nb += l.cut ? 0 : (l.v.size() + 1) * size;
  return nb > limit_size;
}

void literal_prefixes(const Expr &e, Literals *lits) {  // literals.rs:573-642
  switch (e.kind) {
    case EK::Literal:
      if (!e.casei) {
        std::string s;
        for (uint32_t c : e.chars) s += utf8_of(c);
        lits->cross_add(s);
      } else {
        for (uint32_t c : e.chars)
          if (!lits->add_char_class(fold_char(c), false)) {
            lits->cut();
            return;
          }
      }
      return;
    case EK::LiteralBytes:
      if (!e.casei) {
        lits->cross_add(std::string(e.bytes.begin(), e.bytes.end()));
      } else {
        for (uint8_t b : e.bytes)
          if (!lits->add_byte_class(fold_byte(b))) {
            lits->cut();
            return;
          }
      }
      return;
    case EK::Class:
      if (!lits->add_char_class(e.cls, false)) lits->cut();
      return;
    case EK::ClassBytes:
      if (!lits->add_byte_class(e.bcls)) lits->cut();
      return;
    case EK::Group:
      literal_prefixes(e.subs[0], lits);
      return;
    case EK::Repeat:
      repeat_dispatch(e, lits, literal_prefixes);
      return;
    case EK::Concat:
      if (e.subs.empty()) return;
      if (e.subs.size() == 1) { literal_prefixes(e.subs[0], lits); return; }
      for (const Expr &s : e.subs) {
        if (s.kind == EK::StartText) {
          if (!lits->is_empty()) {
            lits->cut();
            break;
          }
          lits->add(Lit{});
          continue;
        }
        Literals l2 = lits->to_empty();
        literal_prefixes(s, &l2);
        if (!lits->cross_product(l2) || !l2.any_complete()) {
          lits->cut();
          break;
        }
      }
      return;
    case EK::Alternate:
      alternate(e.subs, lits, literal_prefixes);
      return;
    default:
      lits->cut();
      return;
  }
}

void literal_suffixes(const Expr &e, Literals *lits) {  // literals.rs:644-718
  switch (e.kind) {
    case EK::Literal:
      if (!e.casei) {
        std::string s;
        for (uint32_t c : e.chars) s += utf8_of(c);
        std::reverse(s.begin(), s.end());
        lits->cross_add(s);
      } else {
        for (size_t k = e.chars.size(); k-- > 0;)
          if (!lits->add_char_class(fold_char(e.chars[k]), true)) {
            lits->cut();
            return;
          }
      }
      return;
    case EK::LiteralBytes:
      if (!e.casei) {
        std::string s(e.bytes.rbegin(), e.bytes.rend());
        lits->cross_add(s);
      } else {
        for (size_t k = e.bytes.size(); k-- > 0;)
          if (!lits->add_byte_class(fold_byte(e.bytes[k]))) {
            lits->cut();
            return;
          }
      }
      return;
    case EK::Class:
      if (!lits->add_char_class(e.cls, true)) lits->cut();
      return;
    case EK::ClassBytes:
      if (!lits->add_byte_class(e.bcls)) lits->cut();
      return;
    case EK::Group:
      literal_suffixes(e.subs[0], lits);
      return;
    case EK::Repeat:
      repeat_dispatch(e, lits, literal_suffixes);
      return;
    case EK::Concat:
      if (e.subs.empty()) return;
      if (e.subs.size() == 1) { literal_suffixes(e.subs[0], lits); return; }
      for (size_t k = e.subs.size(); k-- > 0;) {
        const Expr &s = e.subs[k];
        if (s.kind == EK::EndText) {
          if (!lits->is_empty()) {
            lits->cut();
            break;
          }
          lits->add(Lit{});
          continue;
        }
        Literals l2 = lits->to_empty();
        literal_suffixes(s, &l2);
        if (!lits->cross_product(l2) || !l2.any_complete()) {
          lits->cut();
          break;
        }
      }
      return;
    case EK::Alternate:
      alternate(e.subs, lits, literal_suffixes);
      return;
    default:
      lits->cut();
      return;
  }
}

size_t char_len_lossy(const std::string &s) {
  // String::from_utf8_lossy(..).chars().count(): one char per valid scalar,
  // one U+FFFD per maximal invalid subpart
  const uint8_t *p = (const uint8_t *)s.data();
  const size_t n = s.size();
  size_t i = 0, count = 0;
  while (i < n) {
    const uint8_t b = p[i];
    size_t need = 0;
    uint8_t lo = 0x80, hi = 0xBF;
    if (b < 0x80) { ++count; ++i; continue; }
    if (b >= 0xC2 && b <= 0xDF) need = 1;
    else if (b >= 0xE0 && b <= 0xEF) { need = 2; if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; }
    else if (b >= 0xF0 && b <= 0xF4) { need = 3; if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; }
    else { ++count; ++i; continue; }
    size_t k = 1;
    while (k <= need && i + k < n) {
      const uint8_t c = p[i + k];
      const uint8_t l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
      if (c < l || c > h) break;
      ++k;
    }
    ++count;   // a whole valid scalar or one replacement for the maximal subpart
    i += k;
  }
  return count;
}

LitSearcher make_searcher(const Literals &lits, bool suffix) {  // literals.rs:62-88, 186-250, 325-355
  LitSearcher s;
  s.lits = lits;
  std::vector<uint8_t> dense;
  bool seen[256] = {false};
  bool one_byte = true;
  for (const Lit &l : lits.lits) {
    one_byte = one_byte && l.v.size() == 1;
    if (l.v.empty()) continue;
    const uint8_t b = (uint8_t)(suffix ? l.v.back() : l.v[0]);
    if (!seen[b]) { seen[b] = true; dense.push_back(b); }
  }
  if (lits.lits.empty() || dense.size() >= 26) s.matcher = 0;
  else if (one_byte) s.matcher = 1;
  else if (lits.lits.size() == 1) s.matcher = 2;
  else s.matcher = 3;
  s.len = s.matcher == 0 ? 0 : s.matcher == 1 ? dense.size() : s.matcher == 2 ? 1 : lits.lits.size();
  s.complete = lits.all_complete() && s.len > 0;
  s.lcp = lits.longest_common_prefix();
  s.lcs = lits.longest_common_suffix();
  s.lcp_chars = char_len_lossy(s.lcp);
  s.lcs_chars = char_len_lossy(s.lcs);
  return s;
}

ExecLiterals exec_literals(const Expr &e) {  // exec.rs:209-271, 308-321, 1130-1210
  Literals pre, suf;
  bool pre_ok = true, suf_ok = true;
  if (!e.is_anchored_start() && e.has_anchored_start()) pre_ok = false;
  if (pre_ok && !pre.union_prefixes(e)) pre_ok = false;
  if (!pre_ok) pre = Literals{};
  if (!e.is_anchored_end() && e.has_anchored_end()) suf_ok = false;
  if (suf_ok && !suf.union_suffixes(e)) suf_ok = false;
  if (!suf_ok) suf = Literals{};
  ExecLiterals x;
  x.prefixes = make_searcher(pre.unambiguous_prefixes(), false);
  x.suffixes = make_searcher(suf.unambiguous_suffixes(), true);
  if (x.prefixes.complete)
    x.match_type = e.is_anchored_start() ? MT_LITERAL_ANCHORED_START : MT_LITERAL_UNANCHORED;
  else if (x.suffixes.complete)
    x.match_type = e.is_anchored_end() ? MT_LITERAL_ANCHORED_END : MT_LITERAL_UNANCHORED;
  else if (!e.is_anchored_start() && e.is_anchored_end())
    x.match_type = MT_DFA_ANCHORED_REVERSE;
  else if (x.suffixes.len > 0 && x.suffixes.lcs_chars >= 3 && x.suffixes.lcs_chars > x.prefixes.lcp_chars)
    x.match_type = MT_DFA_SUFFIX;  // should_suffix_scan (exec.rs:1204-1210)
  else
    x.match_type = MT_DFA;
  return x;
}

}  // namespace rure_amd
