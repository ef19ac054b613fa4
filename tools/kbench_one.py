"""Runs one scan configuration a few times (for rocprofv3 counter passes)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import regex_amd as R
from regex_amd.workloads import date_haystacks_device

ap = argparse.ArgumentParser()
ap.add_argument("--pattern", default=r"\d{4}-\d{2}-\d{2}")
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--L", type=int, default=4096)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda:0")
hay, _ = date_haystacks_device(a.n, a.L, 123, dev)
re = R.Regex(a.pattern)
out = re.find_batch(hay, stride=a.L, length=a.L, count=a.n)
for _ in range(a.reps):
    re.find_batch(hay, stride=a.L, length=a.L, count=a.n, out=out)
torch.cuda.synchronize()
print("done")
