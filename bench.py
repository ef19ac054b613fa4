#!/usr/bin/env python3
"""Headline benchmark: batched `bytes::Regex::find` (BASELINE.json configs[1], C2).

  python bench.py [--gpus N] [--steps K] [--warmup W]

A step = one pass of the hot path over one batch: the date regex
`\\d{4}-\\d{2}-\\d{2}` `find` over 1,048,576 synthetic haystacks x 4 KiB
(4 GiB, fixed stride, resident in HBM) on every rank (weak scaling: each
rank owns its own shard of haystacks), followed, for N > 1, by an RCCL
all-gather of the compacted match records (haystack id, start, end) — the
only exchange step the path has.  One process per GPU (torch.distributed,
backend "nccl" = RCCL).

Prints ONE JSON line (rank 0) with the roofline of the scan kernel (HIP
events on the launch stream, algorithmic bytes per launch) and the CPU
baseline (the oracle = restated reference lazy DFA, timed on a bounded
sample of the same haystacks, multi-threaded).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PATTERN = r"\d{4}-\d{2}-\d{2}"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--haystacks", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=4096)
    ap.add_argument("--match-frac", type=float, default=0.01)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def cpu_threads(req):
    if req > 0:
        return req
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import regex_amd as R
    from regex_amd.workloads import date_haystacks_device

    n, L = args.haystacks, args.length
    seed = 0x5EED0002 ^ rank
    hay, planted = date_haystacks_device(n, L, seed, dev, frac=args.match_frac)
    re = R.Regex(PATTERN)
    out = torch.empty((n, 2), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def scan():
        re.find_batch(hay, stride=L, length=L, count=n, out=out, stream=stream)

    max_rec = max(1024, int(n * args.match_frac * 2) + 1024)

    def step():
        scan()
        if world > 1:
            # compact (haystack id, start, end) records and gather them to all ranks
            hit = (out[:, 0] >= 0).nonzero().squeeze(1)
            k = min(hit.numel(), max_rec)
            rec = torch.full((max_rec, 3), -1, dtype=torch.int64, device=dev)
            rec[:k, 0] = hit[:k] + rank * n
            rec[:k, 1:] = out[hit[:k]]
            gathered = torch.empty((world * max_rec, 3), dtype=torch.int64, device=dev)
            dist.all_gather_into_tensor(gathered, rec)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # kernel-only timing with HIP events on the launch stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for a, b in ev:
        a.record(stream)
        scan()
        b.record(stream)
    torch.cuda.synchronize()
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # timed steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt * 1000.0 / args.steps

    res = out.cpu().numpy()
    matched = int((res[:, 0] >= 0).sum())
    # algorithmic bytes per launch: forward bytes to the DFA's stop
    # (whole haystack when there is no match; e+1 when the DFA dies after a
    # match), reverse span, 16-byte result records.
    m = res[:, 0] >= 0
    fwd = np.where(m, np.minimum(res[:, 1] + 1, L), L).sum()
    rev = (res[m, 1] - res[m, 0]).sum()
    b_alg = float(fwd + rev + 16 * n)
    achieved = b_alg / (kernel_ms * 1e-3) / 1e9

    total_bytes = float(n) * L * world
    value = total_bytes / (ms_per_step * 1e-3) / 1e9
    matches_per_s = matched * world / (ms_per_step * 1e-3)

    line = {
        "metric": "haystack GB/s scanned + matches/s, batched bytes::Regex::find, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded printable ASCII, 20% digits, 1% planted dates)",
        "config": {"workload": "C2: find %s over %d x %d B haystacks per GPU" % (PATTERN, n, L),
                   "haystacks_per_gpu": n, "haystack_bytes": L, "parallelism": "dp%d" % world},
        "matches_per_s": round(matches_per_s, 1),
        "matched_haystacks": matched,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": int(b_alg)},
    }

    tr = profiled_traffic(line["config"], b_alg)
    if tr is not None:
        line["roofline"]["traffic"] = tr["bytes"]
        line["roofline"]["traffic_source"] = tr["source"]

    if rank == 0 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(re, hay, res, n, L, args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def profiled_traffic(config, b_alg):
    """HBM bytes per launch of the scan kernel from the committed rocprofv3
    PMC pass of this same command (profiles/<tag>_summary.json, written by
    tools/gpu_profile.sh + tools/summarize_profile.py: FETCH_SIZE KB x 1024 x 2,
    MI355X_MICROARCH.md HBM section).  PMC counters cannot be read from inside
    the timed process, so the newest summary whose workload matches is used."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        strip = lambda c: {k: v for k, v in (c or {}).items() if k != "parallelism"}
        if strip(d.get("bench_config")) != strip(config) or not d.get("hbm_read_bytes_per_launch"):
            continue
        if best is None or os.path.getmtime(p) >= best[0]:
            best = (os.path.getmtime(p), p, d)
    if best is None:
        return None
    d = best[2]
    return {"bytes": int(d["hbm_read_bytes_per_launch"]),
            "source": "%s (rocprofv3 --pmc FETCH_SIZE, kernel %s, %.3fx algorithmic)" %
                      (os.path.relpath(best[1], ROOT), d["kernel"].split("(")[0].replace("void ", ""),
                       d["hbm_read_bytes_per_launch"] / b_alg)}


def cpu_baseline(re, hay, res, n, L, args):
    """The oracle (restated reference lazy DFA, oracle/) on a bounded sample of
    the same haystacks, one private DFA cache per thread; also re-checks the
    GPU results for the sample bit-exactly."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    threads = cpu_threads(args.cpu_threads)
    o = OracleRegex(re)
    # sample: first S haystacks, sized so one pass is ~1 s of CPU time
    S = min(n, 65536)
    buf = hay[: S * L].cpu().numpy()
    t0 = time.perf_counter()
    exp, st = o.find_batch(buf, L, L, S, nthreads=threads)
    t1 = time.perf_counter()
    passes, elapsed = 1, t1 - t0
    while elapsed < args.cpu_seconds and passes < 64:
        t0 = time.perf_counter()
        o.find_batch(buf, L, L, S, nthreads=threads)
        elapsed += time.perf_counter() - t0
        passes += 1
    gbps = S * L * passes / elapsed / 1e9
    parity = bool(np.array_equal(exp.astype(np.int64), res[:S]))
    return {"value": round(gbps, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "%d passes over the first %d haystacks x %d B (%.0f MiB) of the same batch" %
                      (passes, S, L, S * L / 2**20),
            "parity_on_sample": parity, "fwd_bytes_per_pass": int(st["fwd_bytes"])}


if __name__ == "__main__":
    main()
