"""The regex-dna shootout (examples/shootout-regex-dna-bytes.rs) end to end
on the device, through the C ABI only:

  1. strip: `>[^\\n]*\\n|\\n` replace_all with "" (:21) — rure_amd_replace_batch
  2. the 9 variant find_iter counts (:24-42) — rure_amd_find_iter_span_multi
     (one fused pass over the stripped stream)
  3. the 11 IUB substitutions (:44-60), each a replace_all of one byte by its
     alternation text — rure_amd_replace_all_chain: the 11 steps enqueued
     at once, each step's kernel counting the next step's byte as it writes
  4. the three lengths the program prints (:65): input, stripped, substituted

The sequence stays in HBM from the input to the last substitution; only the
counts and lengths are read back.
"""
import ctypes

from . import _native as N
from . import Regex, _check, _stream_ptr, find_iter_span_multi, replace_all_chain

STRIP = b">[^\n]*\n|\n"
VARIANTS = [
    b"agggtaaa|tttaccct",
    b"[cgt]gggtaaa|tttaccc[acg]",
    b"a[act]ggtaaa|tttacc[agt]t",
    b"ag[act]gtaaa|tttac[agt]ct",
    b"agg[act]taaa|ttta[agt]cct",
    b"aggg[acg]aaa|ttt[cgt]ccct",
    b"agggt[cgt]aa|tt[acg]accct",
    b"agggta[cgt]a|t[acg]taccct",
    b"agggtaa[cgt]|[acg]ttaccct",
]
SUBSTS = [(b"B", b"(c|g|t)"), (b"D", b"(a|g|t)"), (b"H", b"(a|c|t)"), (b"K", b"(g|t)"), (b"M", b"(a|c)"),
          (b"N", b"(a|c|g|t)"), (b"R", b"(a|g)"), (b"S", b"(c|g)"), (b"V", b"(a|c|g)"), (b"W", b"(a|t)"),
          (b"Y", b"(c|t)")]


class RegexDna(object):
    """Compiled once; run() many times (bench.py times run() as the C3 line's
    pipeline_ms field, with its known-answer check)."""

    def __init__(self):
        self.strip = Regex(STRIP)
        self.variants = [Regex(v) for v in VARIANTS]
        self.substs = [(Regex(p), r) for p, r in SUBSTS]

    def _replace(self, re_, buf, n, rep, stream, out_cap):
        """replace_all over one haystack buf[0..n) -> (out tensor, length)."""
        import torch
        b = N.RureBatch()
        b.haystack = buf.data_ptr()
        b.offsets = None
        b.stride = n
        b.length = n
        b.count = 1
        b.start = 0
        dev = buf.device
        ooff = torch.empty((2,), dtype=torch.int64, device=dev)
        total = torch.zeros((1,), dtype=torch.int64, device=dev)
        cap = out_cap
        while True:
            out = torch.empty((cap + 16,), dtype=torch.uint8, device=dev)
            _check(N.rure_amd_replace_batch(re_._re, ctypes.byref(b), rep, len(rep), 0, ctypes.c_void_p(out.data_ptr()),
                                            ctypes.c_void_p(ooff.data_ptr()), cap, ctypes.c_void_p(total.data_ptr()),
                                            _stream_ptr(stream)), "replace_batch")
            t = int(total.item())   # one sync per replacement (sizes the next buffer)
            if t <= cap:
                out[t:t + 16].zero_()
                return out, t
            cap = t

    def run(self, seq, n, stream=None):
        """seq: device uint8 tensor holding the input in [0, n) (readable to
        n rounded up to 16).  Returns {"counts": [9], "ilen", "clen", "slen"}."""
        stripped, clen = self._replace(self.strip, seq, n, b"", stream, n)
        # counts only: small match buffers (a count above its capacity is still exact)
        res = find_iter_span_multi(self.variants, stripped, 0, clen, length=clen, capacities=[1 << 16] * 9,
                                   stream=stream)
        counts = [int(c.item()) for c, _, _ in res]
        # the 11 substitutions in one enqueue; the final length is the one
        # read-back (a cut output, lengths[-1] > capacity, reruns sized
        # exactly; the IUB codes grow the stream by a third, so twice its
        # length is never cut)
        cap = 2 * clen + 4096
        while True:
            _, lengths = replace_all_chain([r for r, _ in self.substs], [t for _, t in self.substs], stripped,
                                           length=clen, capacity=cap, stream=stream)
            sl = int(lengths[-1].item())
            if sl <= cap:
                break
            cap = sl
        return {"counts": counts, "ilen": n, "clen": clen, "slen": sl}
