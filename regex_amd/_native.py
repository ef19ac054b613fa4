"""ctypes binding of the C ABI in include/rure_amd.h (librure_amd.so).

The library is built in-tree (`make` / `__graft_entry__.build()`) into
regex_amd/lib/.  There is no fallback: if the shared object is missing the
import fails loudly.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "librure_amd.so")
# A/B builds of the same library (tools/*: diagnostic variants under
# regex_amd/lib/); never set in product use
if os.environ.get("RURE_AMD_LIB_AB"):
    LIB_PATH = os.path.join(_HERE, "lib", os.path.basename(os.environ["RURE_AMD_LIB_AB"]))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "regex_amd: native library %s is missing; build it with `make` or "
        "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)

# Share the HIP runtime with PyTorch (the device-memory / stream plumbing):
# torch bundles its own libamdhip64.so.7; loading it first makes our library
# bind to the same runtime instead of pulling in a second copy from /opt/rocm.
try:
    import torch  # noqa: F401
except ImportError:  # pure C-ABI use without torch
    pass

lib = ctypes.CDLL(LIB_PATH)

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_size = ctypes.c_size_t


class RureMatch(ctypes.Structure):
    _fields_ = [("start", c_size), ("end", c_size)]


class RureBatch(ctypes.Structure):
    _fields_ = [("haystack", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("stride", c_size), ("length", c_size), ("count", c_size),
                ("start", c_size)]


class DfaInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "ok", "states", "raw_states", "normal", "match_end", "dead", "quit",
        "hot", "byte_classes", "insts", "fast_stride", "fast_classes")]


class ProgInfo(ctypes.Structure):
    _fields_ = [("ninsts", ctypes.c_uint32), ("start", ctypes.c_uint32),
                ("nmatches", ctypes.c_uint32), ("ncaptures", ctypes.c_uint32),
                ("anchored_start", ctypes.c_uint8), ("anchored_end", ctypes.c_uint8),
                ("has_unicode_word_boundary", ctypes.c_uint8), ("is_reverse", ctypes.c_uint8),
                ("byte_classes", ctypes.c_uint8 * 256)]


class Inst(ctypes.Structure):
    _fields_ = [("op", ctypes.c_uint8), ("look", ctypes.c_uint8), ("lo", ctypes.c_uint8),
                ("hi", ctypes.c_uint8), ("x", ctypes.c_uint32), ("y", ctypes.c_uint32)]


class NfaInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "leaves", "closures", "entries", "root", "nmatch", "anchored", "looks", "unicode_wb")]


class CoreInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("K", "ncores", "hot", "dead", "quit", "lds_bytes")]


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


VP = ctypes.c_void_p
rure_error_new = _sig("rure_error_new", VP)
rure_error_free = _sig("rure_error_free", None, VP)
rure_error_message = _sig("rure_error_message", ctypes.c_char_p, VP)
rure_options_new = _sig("rure_options_new", VP)
rure_options_free = _sig("rure_options_free", None, VP)
rure_options_size_limit = _sig("rure_options_size_limit", None, VP, c_size)
rure_options_dfa_size_limit = _sig("rure_options_dfa_size_limit", None, VP, c_size)
rure_compile = _sig("rure_compile", VP, ctypes.c_char_p, c_size, ctypes.c_uint32, VP, VP)
rure_free = _sig("rure_free", None, VP)
rure_is_match = _sig("rure_is_match", ctypes.c_bool, VP, ctypes.c_char_p, c_size, c_size)
rure_find = _sig("rure_find", ctypes.c_bool, VP, ctypes.c_char_p, c_size, c_size,
                 ctypes.POINTER(RureMatch))
rure_shortest_match = _sig("rure_shortest_match", ctypes.c_bool, VP, ctypes.c_char_p, c_size, c_size,
                           ctypes.POINTER(c_size))
rure_iter_new = _sig("rure_iter_new", VP, VP)
rure_iter_free = _sig("rure_iter_free", None, VP)
rure_iter_next = _sig("rure_iter_next", ctypes.c_bool, VP, ctypes.c_char_p, c_size,
                      ctypes.POINTER(RureMatch))
rure_captures_new = _sig("rure_captures_new", VP, VP)
rure_captures_free = _sig("rure_captures_free", None, VP)
rure_captures_len = _sig("rure_captures_len", c_size, VP)
rure_captures_at = _sig("rure_captures_at", ctypes.c_bool, VP, c_size, ctypes.POINTER(RureMatch))
rure_find_captures = _sig("rure_find_captures", ctypes.c_bool, VP, ctypes.c_char_p, c_size, c_size, VP)
rure_iter_next_captures = _sig("rure_iter_next_captures", ctypes.c_bool, VP, ctypes.c_char_p, c_size, VP)
rure_capture_name_index = _sig("rure_capture_name_index", ctypes.c_int32, VP, ctypes.c_char_p)
rure_iter_capture_names_new = _sig("rure_iter_capture_names_new", VP, VP)
rure_iter_capture_names_free = _sig("rure_iter_capture_names_free", None, VP)
rure_iter_capture_names_next = _sig("rure_iter_capture_names_next", ctypes.c_bool, VP,
                                    ctypes.POINTER(ctypes.c_char_p))
rure_compile_set = _sig("rure_compile_set", VP, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_size),
                        c_size, ctypes.c_uint32, VP, VP)
rure_set_free = _sig("rure_set_free", None, VP)
rure_set_is_match = _sig("rure_set_is_match", ctypes.c_bool, VP, ctypes.c_char_p, c_size, c_size)
rure_set_matches = _sig("rure_set_matches", ctypes.c_bool, VP, ctypes.c_char_p, c_size, c_size,
                        ctypes.POINTER(ctypes.c_bool))
rure_set_len = _sig("rure_set_len", c_size, VP)
rure_amd_find_batch = _sig("rure_amd_find_batch", ctypes.c_int, VP, ctypes.POINTER(RureBatch), VP, VP)
rure_amd_is_match_batch = _sig("rure_amd_is_match_batch", ctypes.c_int, VP, ctypes.POINTER(RureBatch), VP, VP)
rure_amd_shortest_match_batch = _sig("rure_amd_shortest_match_batch", ctypes.c_int, VP,
                                     ctypes.POINTER(RureBatch), VP, VP)
rure_amd_set_matches_batch = _sig("rure_amd_set_matches_batch", ctypes.c_int, VP, ctypes.POINTER(RureBatch),
                                  VP, VP)
rure_amd_replace_batch = _sig("rure_amd_replace_batch", ctypes.c_int, VP, ctypes.POINTER(RureBatch), ctypes.c_char_p,
                              c_size, c_size, VP, VP, c_size, VP, VP)
rure_amd_replace_all_chain = _sig("rure_amd_replace_all_chain", ctypes.c_int, VP, VP, VP, c_size, VP, c_size, VP, VP,
                                  c_size, VP, VP)
rure_amd_split_batch = _sig("rure_amd_split_batch", ctypes.c_int, VP, ctypes.POINTER(RureBatch), c_size, VP, VP,
                            c_size, VP, VP)
rure_amd_captures_batch = _sig("rure_amd_captures_batch", ctypes.c_int, VP, ctypes.POINTER(RureBatch), VP, VP)
rure_amd_captures_len = _sig("rure_amd_captures_len", c_size, VP)
rure_amd_nfa_saves_export = _sig("rure_amd_nfa_saves_export", ctypes.c_int, VP, VP, VP, ctypes.POINTER(c_size))
rure_amd_dfa_info_get = _sig("rure_amd_dfa_info_get", ctypes.c_int, VP, ctypes.c_int, ctypes.POINTER(DfaInfo))
rure_amd_set_dfa_info_get = _sig("rure_amd_set_dfa_info_get", ctypes.c_int, VP, ctypes.POINTER(DfaInfo))
rure_amd_program_export = _sig("rure_amd_program_export", ctypes.c_int64, VP, ctypes.c_int,
                               ctypes.POINTER(ProgInfo), VP, c_size)
rure_amd_set_program_export = _sig("rure_amd_set_program_export", ctypes.c_int64, VP, ctypes.c_int,
                                   ctypes.POINTER(ProgInfo), VP, c_size)
rure_amd_dfa_export = _sig("rure_amd_dfa_export", ctypes.c_int, VP, ctypes.c_int, VP, VP, VP)
rure_amd_nfa_export = _sig("rure_amd_nfa_export", ctypes.c_int, VP, ctypes.POINTER(NfaInfo), VP, VP, VP)
rure_amd_set_nfa_export = _sig("rure_amd_set_nfa_export", ctypes.c_int, VP, ctypes.POINTER(NfaInfo), VP, VP, VP)
rure_amd_set_dfa_export = _sig("rure_amd_set_dfa_export", ctypes.c_int, VP, VP, VP, VP, VP)
rure_amd_set_core_export = _sig("rure_amd_set_core_export", ctypes.c_int, VP, ctypes.POINTER(CoreInfo), VP, VP,
                                VP, VP, VP)
rure_amd_dfa_strip_export = _sig("rure_amd_dfa_strip_export", ctypes.c_int, VP, VP)
rure_amd_find_iter_batch = _sig("rure_amd_find_iter_batch", ctypes.c_int, VP, ctypes.POINTER(RureBatch), VP, VP,
                                c_size, VP, VP)
rure_amd_find_iter_span = _sig("rure_amd_find_iter_span", ctypes.c_int, VP, VP, c_size, c_size, c_size, VP, VP,
                               VP, c_size, VP, VP)
rure_amd_find_iter_span_multi = _sig("rure_amd_find_iter_span_multi", ctypes.c_int, VP, c_size, VP, c_size, c_size,
                                     c_size, VP, VP, VP, VP, VP, VP)
rure_amd_literals_export = _sig("rure_amd_literals_export", ctypes.c_int64, VP, VP, VP, c_size)
rure_amd_shiftand_export = _sig("rure_amd_shiftand_export", ctypes.c_int64, VP, VP, VP, VP, VP)
rure_amd_uses_dfa = _sig("rure_amd_uses_dfa", ctypes.c_int, VP)
rure_amd_set_uses_dfa = _sig("rure_amd_set_uses_dfa", ctypes.c_int, VP)
rure_amd_last_fwd_path = _sig("rure_amd_last_fwd_path", ctypes.c_int)
rure_amd_debug_set = _sig("rure_amd_debug_set", ctypes.c_int, ctypes.c_char_p)
rure_amd_first_byte_export = _sig("rure_amd_first_byte_export", ctypes.c_int, VP, VP)
rure_amd_lex_export = _sig("rure_amd_lex_export", ctypes.c_int64, VP, VP, c_size, VP)
rure_amd_lex4_export = _sig("rure_amd_lex4_export", ctypes.c_int64, VP, VP, c_size, VP)
rure_amd_run_class_export = _sig("rure_amd_run_class_export", ctypes.c_int, VP, ctypes.c_int, VP)
rure_amd_run_cp_export = _sig("rure_amd_run_cp_export", ctypes.c_int, VP, VP, c_size)
rure_amd_class_one_export = _sig("rure_amd_class_one_export", ctypes.c_int, VP, VP)
rure_amd_lex_ascii_export = _sig("rure_amd_lex_ascii_export", ctypes.c_int64, VP, ctypes.c_int, VP, c_size, VP)
rure_amd_set_matches_batch_words = _sig("rure_amd_set_matches_batch_words", ctypes.c_int, VP,
                                        ctypes.POINTER(RureBatch), VP, c_size, VP)
class MatchInfo(ctypes.Structure):
    _fields_ = [("match_type", ctypes.c_int32), ("prefix_matcher", ctypes.c_int32),
                ("suffix_matcher", ctypes.c_int32), ("prefix_len", ctypes.c_uint32),
                ("suffix_len", ctypes.c_uint32), ("prefix_complete", ctypes.c_uint8),
                ("suffix_complete", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 2),
                ("lcp_chars", ctypes.c_uint32), ("lcs_chars", ctypes.c_uint32),
                ("lcs_bytes", ctypes.c_uint32), ("lcs", ctypes.c_uint8 * 256)]


rure_amd_literals_syntax = _sig("rure_amd_literals_syntax", ctypes.c_int64, ctypes.c_char_p, c_size, ctypes.c_uint32,
                                ctypes.c_int, c_size, c_size, VP, c_size)
rure_amd_literals_op = _sig("rure_amd_literals_op", ctypes.c_int64, ctypes.c_int, ctypes.c_char_p, c_size, VP, c_size)
rure_amd_exec_literals_export = _sig("rure_amd_exec_literals_export", ctypes.c_int64, VP, ctypes.c_int, VP, c_size)
rure_amd_match_info_get = _sig("rure_amd_match_info_get", ctypes.c_int, VP, VP)
rure_amd_release_scratch = _sig("rure_amd_release_scratch", None)
rure_amd_scratch_stats = _sig("rure_amd_scratch_stats", None, ctypes.POINTER(c_size), ctypes.POINTER(c_size),
                              ctypes.POINTER(ctypes.c_long))
rure_amd_kernel_timer = _sig("rure_amd_kernel_timer", ctypes.c_int, ctypes.c_int)
rure_amd_kernel_timer_read = _sig("rure_amd_kernel_timer_read", ctypes.c_double, VP)
rure_amd_compact_matches = _sig("rure_amd_compact_matches", ctypes.c_int, VP, c_size, ctypes.c_uint64, VP, c_size,
                                VP, VP)

FLAG_CASEI = 1 << 0
FLAG_MULTI = 1 << 1
FLAG_DOTNL = 1 << 2
FLAG_SWAP_GREED = 1 << 3
FLAG_SPACE = 1 << 4
FLAG_UNICODE = 1 << 5
DEFAULT_FLAGS = FLAG_UNICODE

OK = 0
ERR_ARG = -1
ERR_HIP = -2
ERR_DFA = -3
NONE = (1 << 64) - 1
QUIT = (1 << 64) - 2
