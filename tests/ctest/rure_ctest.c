/*
 * C-ABI drop-in check: the calls a C program written against the
 * reference's regex-capi/include/rure.h makes (the same cases its
 * regex-capi/ctest/test.c covers: is_match, shortest_match, find, iter,
 * flags, compile errors, size limit, sets, set start offsets, captures,
 * iteration with captures, capture names), made against
 * include/rure_amd.h and librure_amd.so.  Exit status 0 = all passed.
 */
#include <stdio.h>
#include <string.h>

#include "rure_amd.h"

static int failures = 0;
#define CHECK(cond, what)                                        \
  do {                                                           \
    if (!(cond)) {                                               \
      fprintf(stderr, "FAIL %s (%s:%d)\n", what, __FILE__, __LINE__); \
      ++failures;                                                \
    }                                                            \
  } while (0)

static void is_match_and_find(void) {
  const char *hay = "snowman: \xE2\x98\x83";
  rure *re = rure_compile_must("\\p{So}$");
  CHECK(rure_is_match(re, (const uint8_t *)hay, strlen(hay), 0), "is_match \\p{So}$");
  rure_match m = {0, 0};
  CHECK(rure_find(re, (const uint8_t *)hay, strlen(hay), 0, &m), "find \\p{So}$");
  CHECK(m.start == 9 && m.end == 12, "find offsets (9, 12)");
  CHECK(rure_find(re, (const uint8_t *)hay, strlen(hay), 0, NULL), "find with NULL match");
  rure_free(re);
}

static void shortest(void) {
  rure *re = rure_compile_must("a+");
  size_t end = 0;
  CHECK(rure_shortest_match(re, (const uint8_t *)"aaaaa", 5, 0, &end), "shortest_match a+");
  CHECK(end == 1, "shortest_match end 1");
  rure_free(re);
}

static void iter(void) {
  rure *re = rure_compile_must("\\w+(\\w)");
  rure_iter *it = rure_iter_new(re);
  const uint8_t *hay = (const uint8_t *)"abc xyz";
  rure_match m;
  CHECK(rure_iter_next(it, hay, 7, &m) && m.start == 0 && m.end == 3, "iter first (0, 3)");
  CHECK(rure_iter_next(it, hay, 7, &m) && m.start == 4 && m.end == 7, "iter second (4, 7)");
  CHECK(!rure_iter_next(it, hay, 7, &m), "iter exhausted");
  rure_iter_free(it);
  rure_free(re);
  re = rure_compile_must("");
  it = rure_iter_new(re);
  size_t n = 0;
  while (rure_iter_next(it, (const uint8_t *)"ab", 2, &m)) ++n;
  CHECK(n == 3, "empty-pattern iter yields 3 empty matches");
  rure_iter_free(it);
  rure_free(re);
}

static void captures(void) {
  const char *hay = "snowman: \xE2\x98\x83";
  rure *re = rure_compile_must(".(.*(?P<snowman>\\p{So}))$");
  rure_captures *caps = rure_captures_new(re);
  CHECK(rure_find_captures(re, (const uint8_t *)hay, strlen(hay), 0, caps), "find_captures matches");
  CHECK(rure_captures_len(caps) == 3, "captures_len 3");
  CHECK(rure_capture_name_index(re, "snowman") == 2, "capture_name_index snowman = 2");
  CHECK(rure_capture_name_index(re, "nope") == -1, "capture_name_index unknown = -1");
  rure_match m = {0, 0};
  CHECK(rure_captures_at(caps, 2, &m) && m.start == 9 && m.end == 12, "capture 2 at (9, 12)");
  CHECK(rure_captures_at(caps, 0, &m) && m.start == 0 && m.end == 12, "capture 0 at (0, 12)");
  CHECK(!rure_captures_at(caps, 3, &m), "capture 3 out of range");
  CHECK(!rure_find_captures(re, (const uint8_t *)"x", 1, 0, caps), "find_captures no match");
  CHECK(!rure_captures_at(caps, 0, &m), "no groups after a failed search");
  rure_captures_free(caps);
  rure_free(re);

  re = rure_compile_must("\\w+(\\w)");
  caps = rure_captures_new(re);
  rure_iter *it = rure_iter_new(re);
  const uint8_t *h2 = (const uint8_t *)"abc xyz";
  CHECK(rure_iter_next(it, h2, 7, &m) && m.start == 0 && m.end == 3, "iter first (0, 3)");
  CHECK(rure_iter_next_captures(it, h2, 7, caps), "iter_next_captures second match");
  CHECK(rure_captures_at(caps, 1, &m) && m.start == 6 && m.end == 7, "second match group 1 at (6, 7)");
  CHECK(!rure_iter_next_captures(it, h2, 7, caps), "iter_next_captures exhausted");
  rure_iter_free(it);
  rure_captures_free(caps);
  rure_free(re);

  re = rure_compile_must("(?P<year>\\d{4})-(?P<month>\\d{2})-(?P<day>\\d{2})");
  rure_iter_capture_names *names = rure_iter_capture_names_new(re);
  char *name = NULL;
  const char *expect[] = {"", "year", "month", "day"};
  for (int i = 0; i < 4; ++i)
    CHECK(rure_iter_capture_names_next(names, &name) && strcmp(name, expect[i]) == 0, "capture name in order");
  CHECK(!rure_iter_capture_names_next(names, &name), "capture names exhausted");
  rure_iter_capture_names_free(names);
  rure_free(re);
}

static void flags(void) {
  /* without RURE_FLAG_UNICODE, '.' matches any byte but \n */
  rure *re = rure_compile((const uint8_t *)".", 1, 0, NULL, NULL);
  CHECK(re != NULL, "compile . without unicode");
  CHECK(rure_is_match(re, (const uint8_t *)"\xFF", 1, 0), ". matches \\xFF without unicode");
  rure_free(re);
  re = rure_compile((const uint8_t *)".", 1, RURE_FLAG_UNICODE, NULL, NULL);
  CHECK(!rure_is_match(re, (const uint8_t *)"\xFF", 1, 0), ". does not match \\xFF with unicode");
  rure_free(re);
  re = rure_compile((const uint8_t *)"abc", 3, RURE_FLAG_CASEI | RURE_FLAG_UNICODE, NULL, NULL);
  CHECK(rure_is_match(re, (const uint8_t *)"xABCx", 5, 0), "case-insensitive flag");
  rure_free(re);
}

static void compile_errors(void) {
  rure_error *err = rure_error_new();
  rure *re = rure_compile((const uint8_t *)"(", 1, 0, NULL, err);
  CHECK(re == NULL, "unclosed paren rejected");
  CHECK(strlen(rure_error_message(err)) > 0, "error message present");
  rure_options *opts = rure_options_new();
  rure_options_size_limit(opts, 0);
  re = rure_compile((const uint8_t *)"\\w{100}", 7, 0, opts, err);
  CHECK(re == NULL, "size limit 0 rejects \\w{100}");
  CHECK(strstr(rure_error_message(err), "size") != NULL, "size limit message");
  rure_options_free(opts);
  rure_error_free(err);
}

static void sets(void) {
  const char *pats[] = {"foo", "barfoo", "\\w+", "\\d+", "foobar", "bar"};
  size_t lens[] = {3, 6, 3, 3, 6, 3};
  rure_set *s = rure_compile_set((const uint8_t **)pats, lens, 6, 0, NULL, NULL);
  CHECK(s != NULL, "compile set");
  CHECK(rure_set_len(s) == 6, "set len");
  CHECK(rure_set_is_match(s, (const uint8_t *)"foobar", 6, 0), "set is_match foobar");
  CHECK(!rure_set_is_match(s, (const uint8_t *)"", 0, 0), "set no match on empty");
  bool matches[6];
  CHECK(rure_set_matches(s, (const uint8_t *)"foobar", 6, 0, matches), "set matches foobar");
  const bool want[6] = {true, false, true, false, true, true};
  for (int i = 0; i < 6; ++i) CHECK(matches[i] == want[i], "set match vector");
  rure_set_free(s);

  const char *p2[] = {"foo", "bar", "fooo"};
  size_t l2[] = {3, 3, 4};
  s = rure_compile_set((const uint8_t **)p2, l2, 3, 0, NULL, NULL);
  CHECK(!rure_set_is_match(s, (const uint8_t *)"foobiasdr", 9, 2), "set start offset skips foo");
  bool m2[3];
  CHECK(rure_set_matches(s, (const uint8_t *)"fooobar", 7, 0, m2) && m2[0] && m2[1] && m2[2], "set all three");
  CHECK(rure_set_matches(s, (const uint8_t *)"fooobar", 7, 1, m2) && !m2[0] && m2[1] && !m2[2], "set start 1");
  rure_set_free(s);
}

int main(void) {
  is_match_and_find();
  shortest();
  iter();
  captures();
  flags();
  compile_errors();
  sets();
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("rure_ctest: all checks passed\n");
  return 0;
}
