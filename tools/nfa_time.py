"""Times the Pike VM paths: Unicode word boundaries on text with non-ASCII
bytes (DFA quits -> wavefront Pike VM) and an automaton too large for a DFA."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import regex_amd as R
dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
n, L = 1 << 16, 1024
words = [w.encode() for w in "the quick brown fox jumps over lazy dog héllo wörld naïve café".split()]
parts = []
total = n * L
buf = bytearray()
while len(buf) < total:
    buf += words[int(rng.integers(len(words)))] + b" "
hay = torch.from_numpy(np.frombuffer(bytes(buf[:total]) + b"\0" * 16, dtype=np.uint8).copy()).to(dev)
for pat in [r"\bfox\b", r"\b\w+\b", r"(?-u:[ab])*a(?-u:[ab]){17}"]:
    re = R.Regex(pat)
    out = re.find_batch(hay, stride=L, length=L, count=n)
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(3):
        re.find_batch(hay, stride=L, length=L, count=n, out=out)
    torch.cuda.synchronize()
    ms = (time.time() - t) / 3 * 1e3
    print("%-32s uses_dfa=%s  %8.2f ms  %8.2f GB/s" % (pat, re.uses_dfa(), ms, total / ms / 1e6), flush=True)
