"""Times the C4 set scan (10M log lines x 64 patterns) on one GPU."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import regex_amd as R
from regex_amd.workloads import C4_PATTERNS, log_lines_device
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dev = torch.device("cuda", 0)
t = time.time()
buf, offs = log_lines_device(n, dev)
torch.cuda.synchronize()
print("gen %.2fs, %d bytes" % (time.time() - t, buf.numel()), flush=True)
t = time.time()
rs = R.RegexSet(C4_PATTERNS)
out = torch.empty(n, dtype=torch.int64, device=dev)
rs.matches_batch(buf, offsets=offs, out=out)
torch.cuda.synchronize()
print("compile+first %.2fs" % (time.time() - t), flush=True)
st = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(st)
for _ in range(5):
    rs.matches_batch(buf, offsets=offs, out=out, stream=st)
ev[1].record(st)
torch.cuda.synchronize()
ms = ev[0].elapsed_time(ev[1]) / 5
nb = int(offs[-1])
print("C4: %.3f ms per pass, %.1f GB/s, %.1f M lines/s" % (ms, nb / ms / 1e6, n / ms / 1e3), flush=True)
