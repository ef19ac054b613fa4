"""Micro-benchmarks of the scan kernel across regimes (diagnostics only)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import regex_amd as R
from regex_amd.workloads import date_haystacks_device

dev = torch.device("cuda:0")
def bench(pat, n, L, mode="find", reps=10):
    hay, _ = date_haystacks_device(n, L, 123, dev)
    re = R.Regex(pat)
    fn = {"find": re.find_batch, "is_match": re.is_match_batch}[mode]
    out = fn(hay, stride=L, length=L, count=n)
    torch.cuda.synchronize()
    t0 = time.time()
    while time.time() - t0 < 0.3:  # let the clocks ramp up before timing
        fn(hay, stride=L, length=L, count=n, out=out)
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn(hay, stride=L, length=L, count=n, out=out)
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print("%-28s %-8s n=%-8d L=%-6d %8.3f ms  %8.1f GB/s" % (pat, mode, n, L, ms, n * L / ms / 1e6), flush=True)
    del hay

for args in [(r"\d{4}-\d{2}-\d{2}", 1 << 20, 4096), ("a", 1 << 20, 4096), ("zqzq", 1 << 20, 4096),
             (r"\d{4}-\d{2}-\d{2}", 1 << 15, 4096), ("zqzq", 1 << 15, 4096),
             (r"\d{4}-\d{2}-\d{2}", 1 << 22, 1024), (r"\w+@\w+\.\w+", 1 << 20, 4096)]:
    bench(*args)
bench(r"\d{4}-\d{2}-\d{2}", 1 << 20, 4096, "is_match")
