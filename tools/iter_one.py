"""One find_iter workload for profiling: regex-dna strip pattern over N copies."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch
import regex_amd as R
from golden_data import corpus, known_counts
copies = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
pat = sys.argv[2] if len(sys.argv) > 2 else known_counts()["regexdna"]["strip"]
raw = corpus("regexdna")
dev = torch.device("cuda", 0)
one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(dev)
N = copies * len(raw)
big = torch.zeros(N + 16, dtype=torch.uint8, device=dev)
big[:N].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
re = R.Regex(pat)
for _ in range(3):
    c, m = re.find_iter_batch(big, stride=N, length=N, count=1, capacity=copies * 2000)
torch.cuda.synchronize()
print("matches", int(c[0]))
