#!/usr/bin/env python3
"""Headline benchmark: batched `bytes::Regex::find` (BASELINE.json configs[1], C2).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c4|c5]

With --gpus N > 1 and no torch.distributed environment (WORLD_SIZE unset),
this process starts N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT set, one per GPU), before anything touches
the GPU, and prints rank 0's line; under torchrun it is one of the ranks.

Default (the driver's line) = C2: a step is one pass of the hot path over one
batch — the date regex `\\d{4}-\\d{2}-\\d{2}` `find` over 1,048,576 synthetic
haystacks x 4 KiB (4 GiB, fixed stride, resident in HBM) on every rank (weak
scaling: each rank owns its own shard), followed, for N > 1, by the only
exchange the path has: an all-gather (RCCL) of the compacted match records.

Other configs (for DESIGN.md's table; same timing protocol):
  c1  the date regex `is_match` over 1K x 1 KiB ASCII buffers (BASELINE
      configs[0], the reference's CPU-runnable case): the batched GPU call
      and the oracle on the host, whole-batch parity
  c3  regex-dna: `>[^\\n]*\\n|\\n` find_iter over the input replicated to
      2 GiB, then the 9 variant patterns' find_iter over the stripped 2 GiB;
      for N > 1 each logical stream is cut into N contiguous spans (strong
      scaling) with one exit exchange (all-gather) per step
  c4  RegexSet of 64 patterns over 10M synthetic log lines (one mask per line)
  c5  `\\w+@\\w+\\.\\w+` find over one 16 GiB haystack per GPU, one planted
      match in its last MiB; records gathered across ranks
  big `[a-q][^u-z]{13}x` find over 256K x 4 KiB random a-w haystacks (an x
      planted per 2 KiB):
      a 73,725-state forward DFA (past the u16 tables) on the u32 big-DFA
      kernel, with the Pike VM it replaces timed beside it

Prints ONE JSON line (rank 0) with the roofline of the scan kernel (HIP
events on the launch stream, algorithmic bytes per launch; HBM traffic from
the committed rocprofv3 PMC pass of the same command) and, for C2, the CPU
baseline (the oracle = restated reference lazy DFA, timed on a bounded sample
of the same haystacks, multi-threaded).
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
METRIC = "haystack GB/s scanned + matches/s, batched bytes::Regex::find, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "big", "rehearsal"])
    ap.add_argument("--haystacks", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=4096)
    ap.add_argument("--match-frac", type=float, default=0.01)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive measurement (C2)")
    ap.add_argument("--no-parity", action="store_true", help="skip the whole-batch oracle check (C2)")
    ap.add_argument("--c3-separate", action="store_true",
                    help="C3: one find_iter pass per variant instead of the fused multi-regex pass")
    return ap.parse_args()


def host_cpus():
    """(CPUs this process may run on, the cgroup CPU quota in CPUs or None)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    quota = None
    for path, split in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), open(
                            "/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()])):
        try:
            q, per = split(open(path).read())
            if q not in ("max", "-1"):
                quota = int(q) / int(per)
            break
        except (OSError, ValueError):
            continue
    return n, quota


def cpu_threads(req):
    """Threads for the CPU baseline: every CPU the process may use, bounded
    by the cgroup quota and by OMP_NUM_THREADS (the GPU box grants 16 CPUs
    per GPU and says so there) — the host's full count is reported beside."""
    if req > 0:
        return req
    n, quota = host_cpus()
    if quota:
        n = min(n, max(1, int(quota)))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_info(threads):
    n, quota = host_cpus()
    return {"cores": threads, "host_cpus": os.cpu_count(), "affinity_cpus": n,
            "cgroup_cpu_quota": quota, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


class Ctx(object):
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.args = torch, dist, args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, self.world))
        # REGEX_AMD_BENCH_BACKEND=gloo rehearses the N > 1 paths with several
        # ranks sharing one GPU (RCCL refuses duplicate devices); the driver's
        # multi-GPU runs use the default, nccl (= RCCL over xGMI)
        backend = os.environ.get("REGEX_AMD_BENCH_BACKEND", "nccl")
        if args.config == "rehearsal":   # CPU-only protocol check (tests/test_bench_launch.py)
            self.dev, self.stream = torch.device("cpu"), None
            if self.world > 1:
                dist.init_process_group("gloo")
            return
        if backend != "nccl":
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        if self.world > 1:
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(backend)
        self.stream = torch.cuda.current_stream(self.dev)

    def kernel_ms(self, fn):
        """Mean duration of fn() over --steps launches, HIP events on the launch stream."""
        torch = self.torch
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(self.args.steps)]
        for a, b in ev:
            a.record(self.stream)
            fn()
            b.record(self.stream)
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in ev]))

    def ramp(self, fn, seconds=0.25):
        """Untimed launches until the GPU clocks have left their ramp (the first
        ~10-50 ms of launches after idle run up to 15 % slower); reported in
        the JSON line as clock_ramp_s."""
        torch = self.torch
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            fn()
            torch.cuda.synchronize()
        self.ramp_s = round(time.perf_counter() - t0, 3)

    def sync(self):
        if self.dev.type == "cuda":
            self.torch.cuda.synchronize()

    def timed(self, step):
        """Warmup, then EXACTLY --steps steps between barrier + synchronize;
        max over ranks (seconds per step)."""
        dist = self.dist
        for _ in range(self.args.warmup):
            step()
        self.sync()
        if self.world > 1:
            dist.barrier()
        self.sync()
        t0 = time.perf_counter()
        for _ in range(self.args.steps):
            step()
        self.sync()
        if self.world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if self.world > 1:
            from regex_amd.dist import max_over_ranks
            dt = max_over_ranks(dt, self.dev)
        return dt / self.args.steps

    def line(self, metric, value, unit, ms, dtype, data, config, **extra):
        d = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": self.world,
             "steps": self.args.steps, "warmup": self.args.warmup, "ms_per_step": round(ms, 4),
             "clock_ramp_s": getattr(self, "ramp_s", 0.0),
             "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
             "data": data, "config": config}
        d.update(extra)
        return d

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def roofline(achieved_gbs, kernel_ms, b_alg, config):
    r = {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": None,
         "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": int(b_alg)}
    tr = profiled_traffic(config, b_alg)
    if tr is not None:
        r["traffic"] = tr["bytes"]
        r["traffic_source"] = tr["source"]
    return r


def _short_kernel(name):
    import re
    return re.sub(r"\((rure_amd::BatchDev|unsigned|int|long|void\*).*$", "", name).replace("void ", "")


def profiled_traffic(config, b_alg, kernel=None):
    """HBM bytes per launch of the scan kernel from the committed rocprofv3
    PMC pass of this same command (profiles/<tag>_summary.json, written by
    tools/gpu_profile.sh + tools/summarize_profile.py: FETCH_SIZE KB x 1024 x 2,
    MI355X_MICROARCH.md HBM section).  PMC counters cannot be read from inside
    the timed process, so the newest summary whose workload matches is used
    (by its `generated_utc` stamp: file times do not survive a checkout)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        strip = lambda c: {k: v for k, v in (c or {}).items() if k != "parallelism"}
        if strip(d.get("bench_config")) != strip(config):
            continue
        # the summary's dominant kernel, or one of its per-roofline entries
        # (launches of the workload's grid only: C3's strip lexer)
        cands = [d] + list((d.get("rooflines") or {}).values())
        for e in cands:
            if not e.get("hbm_read_bytes_per_launch"):
                continue
            if kernel is not None and kernel not in (e.get("kernel") or ""):
                continue
            key = (d.get("generated_utc", ""), os.path.basename(p))
            if best is None or key >= best[0]:
                best = (key, p, e)
            break
    if best is None:
        return None
    d = best[2]
    return {"bytes": int(d["hbm_read_bytes_per_launch"]),
            "source": "%s (rocprofv3 --pmc FETCH_SIZE, kernel %s, %.3fx algorithmic)" %
                      (os.path.relpath(best[1], ROOT), _short_kernel(d["kernel"]),
                       d["hbm_read_bytes_per_launch"] / b_alg)}


# ------------------------------------------------------------------ C2
def run_c2(ctx):
    import regex_amd as R
    from regex_amd.dist import RecordGather
    from regex_amd.workloads import date_haystacks_device
    torch, args = ctx.torch, ctx.args
    n, L = args.haystacks, args.length
    hay, planted = date_haystacks_device(n, L, 0x5EED0002 ^ ctx.rank, ctx.dev, frac=args.match_frac)
    re = R.Regex(PATTERN)
    out = torch.empty((n, 2), dtype=torch.int64, device=ctx.dev)

    def scan():
        re.find_batch(hay, stride=L, length=L, count=n, out=out, stream=ctx.stream)

    gather = None
    if ctx.world > 1:
        # fixed-capacity record exchange sized from an untimed first scan
        scan()
        torch.cuda.synchronize()
        hits = int((out[:, 0] >= 0).sum().item())
        cap = torch.tensor([hits], dtype=torch.int64, device=ctx.dev)
        ctx.dist.all_reduce(cap, op=ctx.dist.ReduceOp.MAX)
        gather = RecordGather(int(cap.item()) + 1024, ctx.dev)

    def step():
        scan()
        if gather is not None:
            gather.step(out, ctx.rank * n, ctx.stream)

    ctx.ramp(scan)
    sec = ctx.timed(step)
    # kernel-only time with HIP events, measured after the timed steps so the
    # clocks have left their ramp (the first ~10 ms of launches run slower)
    kernel_ms = ctx.kernel_ms(scan)

    res = out.cpu().numpy()
    matched = int((res[:, 0] >= 0).sum())
    extra = {}
    if gather is not None:
        recs, counts = gather.result()
        mine = recs[sum(counts[:ctx.rank]):sum(counts[:ctx.rank + 1])].cpu().numpy()
        hit = np.nonzero(res[:, 0] >= 0)[0]
        extra["gathered_records"] = int(recs.shape[0])
        extra["gather_ok"] = bool(counts[ctx.rank] == matched and np.array_equal(mine[:, 0], hit + ctx.rank * n)
                                  and np.array_equal(mine[:, 1:], res[hit]))
    if not args.no_parity:
        extra["parity"] = full_parity(re, hay, res, n, L, args)
    # algorithmic bytes per launch: forward bytes to the DFA's stop
    # (whole haystack when there is no match; e+1 when the DFA dies after a
    # match), reverse span, 16-byte result records.
    m = res[:, 0] >= 0
    fwd = np.where(m, np.minimum(res[:, 1] + 1, L), L).sum()
    rev = (res[m, 1] - res[m, 0]).sum()
    b_alg = float(fwd + rev + 16 * n)
    achieved = b_alg / (kernel_ms * 1e-3) / 1e9
    value = float(n) * L * ctx.world / sec / 1e9
    config = {"workload": "C2: find %s over %d x %d B haystacks per GPU" % (PATTERN, n, L),
              "haystacks_per_gpu": n, "haystack_bytes": L, "parallelism": "dp%d" % ctx.world}
    line = ctx.line(METRIC, value, "GB/s", sec * 1e3, "u8",
                    "synthetic (seeded printable ASCII, 20% digits, 1% planted dates)", config,
                    matches_per_s=round(matched * ctx.world / sec, 1), matched_haystacks=matched,
                    roofline=roofline(achieved, kernel_ms, b_alg, config), **extra)
    if ctx.rank == 0 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(re, hay, res, n, L, args)
    if ctx.rank == 0 and not args.no_pcie:
        line["pcie_inclusive"] = pcie_inclusive(ctx, hay, scan)
    return line


def pcie_inclusive(ctx, hay, scan):
    """End-to-end rate when the batch starts in (pinned) host memory: one
    host->HBM copy of the whole batch plus the find launch, on the launch
    stream (never the headline `value`)."""
    torch = ctx.torch
    host = hay.cpu().pin_memory()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for rep in range(2):  # the second repetition is reported
        ev[0].record(ctx.stream)
        with torch.cuda.stream(ctx.stream):
            hay.copy_(host, non_blocking=True)
        ev[1].record(ctx.stream)
        scan()
        ev[2].record(ctx.stream)
        torch.cuda.synchronize()
    h2d = ev[0].elapsed_time(ev[1])
    tot = ev[0].elapsed_time(ev[2])
    nbytes = hay.numel()
    return {"GBps": round(nbytes / (tot * 1e-3) / 1e9, 2), "h2d_ms": round(h2d, 3), "find_ms": round(tot - h2d, 3),
            "h2d_GBps": round(nbytes / (h2d * 1e-3) / 1e9, 2), "note": "pinned host -> HBM copy + find, per batch"}


def full_parity(re, hay, res, n, L, args):
    """Whole-batch bit-exact check of this rank's GPU find results against the
    oracle (the restated reference lazy DFA, dfa.rs:576-764 + exec.rs:632-662),
    multi-threaded on the host.  A mismatch ends the run with a non-zero exit
    status before any metric line is printed."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    t0 = time.perf_counter()
    buf = hay[: n * L].cpu().numpy()
    exp, _ = OracleRegex(re).find_batch(buf, L, L, n, nthreads=cpu_threads(args.cpu_threads))
    bad = np.nonzero((exp.astype(np.int64) != res).any(axis=1))[0]
    if bad.size:
        i = int(bad[0])
        sys.stderr.write("PARITY FAILURE: %d of %d haystacks differ from the oracle; first %d: gpu %s oracle %s\n"
                         % (bad.size, n, i, res[i].tolist(), exp[i].astype(np.int64).tolist()))
        sys.exit(3)
    return {"haystacks_checked": n, "mismatches": 0, "check_s": round(time.perf_counter() - t0, 2),
            "against": "oracle (restated reference lazy DFA), whole batch"}


def cpu_baseline(re, hay, res, n, L, args):
    """The oracle (restated reference lazy DFA, oracle/) on a bounded sample of
    the same haystacks, one private DFA cache per thread; also re-checks the
    GPU results for the sample bit-exactly."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    threads = cpu_threads(args.cpu_threads)
    o = OracleRegex(re)
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
    # a measured one-thread rate, on the first 4096 haystacks
    S1 = min(S, 4096)
    p1, e1 = 0, 0.0
    while e1 < max(2.0, args.cpu_seconds / 4) and p1 < 256:
        t0 = time.perf_counter()
        o.find_batch(buf, L, L, S1, nthreads=1)
        e1 += time.perf_counter() - t0
        p1 += 1
    one = S1 * L * p1 / e1 / 1e9
    d = {"value": round(gbps, 3), "unit": "GB/s", "kind": "port",
         "sample": "%d passes over the first %d haystacks x %d B (%.0f MiB) of the same batch" %
                   (passes, S, L, S * L / 2**20),
         "engine_path": "lazy DFA forward + reverse (dfa.rs:576-866 via exec.rs:632-662; the date regex has no "
                        "literal prefixes: MatchType::Dfa)",
         "per_core_GBps": round(one, 3),
         "one_thread": {"value": round(one, 3), "unit": "GB/s",
                        "sample": "%d passes over the first %d haystacks (%.0f MiB), 1 thread" %
                                  (p1, S1, S1 * L / 2**20)},
         "parity_on_sample": parity, "fwd_bytes_per_pass": int(st["fwd_bytes"])}
    d.update(cpu_info(threads))
    return d


# ------------------------------------------------------------------ C3
def run_c3(ctx):
    import ctypes

    import regex_amd as R
    from regex_amd import _native as NN
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_data import corpus, known_counts
    from oracle_py import OracleRegex
    torch = ctx.torch
    kc = known_counts()["regexdna"]
    raw = corpus("regexdna")
    copies = (1 << 31) // len(raw)            # 21106 copies, 2,147,429,970 B
    N = copies * len(raw)
    one = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(ctx.dev)
    big = torch.empty(N + 16, dtype=torch.uint8, device=ctx.dev)
    big[:N].view(copies, len(raw)).copy_(one.expand(copies, len(raw)))
    big[N:] = 0
    strip = R.Regex(kc["strip"])
    cap = 40_000_000
    spans = torch.empty((cap, 2), dtype=torch.int64, device=ctx.dev)
    cnt = torch.empty(1, dtype=torch.int64, device=ctx.dev)
    tot = torch.empty(1, dtype=torch.int64, device=ctx.dev)

    def find_iter_raw(re_, buf, n, out, counts, total):
        b = R._batch(buf, None, n, n, 1, 0)
        rc = NN.rure_amd_find_iter_batch(re_._re, ctypes.byref(b), ctypes.c_void_p(counts.data_ptr()),
                                         ctypes.c_void_p(out.data_ptr()), out.shape[0],
                                         ctypes.c_void_p(total.data_ptr()), R._stream_ptr(ctx.stream))
        assert rc == 0

    find_iter_raw(strip, big, N, spans, cnt, tot)
    torch.cuda.synchronize()
    nsp = int(tot.item())
    assert nsp <= cap
    # replace_all(strip, "") on the device: keep mask from the match spans
    d = torch.zeros(N + 1, dtype=torch.int32, device=ctx.dev)
    sp = spans[:nsp]
    d.index_add_(0, sp[:, 0], torch.ones(nsp, dtype=torch.int32, device=ctx.dev))
    d.index_add_(0, sp[:, 1], torch.full((nsp,), -1, dtype=torch.int32, device=ctx.dev))
    keep = torch.cumsum(d[:N], 0) == 0
    del d
    seq = torch.cat([big[:N][keep], torch.zeros(16, dtype=torch.uint8, device=ctx.dev)])
    del keep
    M = seq.numel() - 16
    assert M == kc["stripped_len"] * copies, (M, kc["stripped_len"] * copies)
    variants = [R.Regex(v["re"]) for v in kc["variants"]]
    vout = torch.empty((1 << 20, 2), dtype=torch.int64, device=ctx.dev)
    # one pass = one find_iter over the rank's span of one logical haystack
    # (the whole haystack at N = 1); SURVEY §8e: contiguous spans, one exit
    # exchange per step, recomputation only where a match crosses a cut
    from regex_amd.dist import _entry_key, iterate_spans, span_bounds
    passes = [(strip, big, N, spans)] + [(v, seq, M, vout) for v in variants]
    P, W, rk = len(passes), ctx.world, ctx.rank
    pcount = torch.zeros((P,), dtype=torch.int64, device=ctx.dev)
    pexit = torch.zeros((P, 3), dtype=torch.int64, device=ctx.dev)
    spv = [R._stream_ptr(ctx.stream)]
    stats = {"recomputed": 0}

    def span_raw(j, i, entry):
        re_, buf, L, out = passes[j]
        lo, hi = span_bounds(L, W, i)
        ent = ctypes.c_void_p(entry.data_ptr()) if entry is not None else None
        rc = NN.rure_amd_find_iter_span(re_._re, ctypes.c_void_p(buf.data_ptr()), L, lo, hi, ent,
                                        ctypes.c_void_p(pcount[j:].data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                        out.shape[0], ctypes.c_void_p(pexit[j].data_ptr()), spv[0])
        assert rc == 0

    def repair(j):
        # rare: a match crosses a cut of pass j; the generic exchange loop
        stats["recomputed"] += 1

        def run(i, entry):
            e = None if entry is None else torch.tensor(entry, dtype=torch.int64, device=ctx.dev)
            span_raw(j, i, e)
            return pcount[j:j + 1], None, pexit[j]

        def gather(mine):
            parts = [torch.empty(3, dtype=torch.int64, device=ctx.dev) for _ in range(W)]
            ctx.dist.all_gather(parts, mine[rk].clone())
            return [q.tolist() for q in parts]

        iterate_spans(run, W, [rk], gather)

    def exchange():
        parts = [torch.empty_like(pexit) for _ in range(W)]
        ctx.dist.all_gather(parts, pexit)
        ex = torch.stack(parts).cpu().tolist()     # (W, P, 3): one sync per step
        for j in range(P):
            if any(_entry_key(ex[i - 1][j]) != ("fresh",) for i in range(1, W)):
                repair(j)

    def strip_pass():
        span_raw(0, rk, None)

    # the 9 variants over the rank's span in one call: they are all finite
    # sets of 8-byte strings, so rure_amd_find_iter_span_multi reads the
    # stream once for all of them (each variant's matches, count and exit are
    # exactly its own find_iter_span's: tests/test_gpu_multi.py)
    VP = ctypes.c_void_p
    nv = P - 1
    m_res = (VP * nv)(*[passes[j][0]._re for j in range(1, P)])
    m_cnt = (VP * nv)(*[VP(pcount[j:].data_ptr()) for j in range(1, P)])
    m_out = (VP * nv)(*[VP(passes[j][3].data_ptr()) for j in range(1, P)])
    m_cap = (ctypes.c_size_t * nv)(*[passes[j][3].shape[0] for j in range(1, P)])
    m_exit = (VP * nv)(*[VP(pexit[j].data_ptr()) for j in range(1, P)])
    v_lo, v_hi = span_bounds(M, W, rk)

    def variant_pass():
        if ctx.args.c3_separate:
            for j in range(1, P):
                span_raw(j, rk, None)
            return
        rc = NN.rure_amd_find_iter_span_multi(m_res, nv, VP(seq.data_ptr()), M, v_lo, v_hi, None, m_cnt, m_out,
                                              m_cap, m_exit, spv[0])
        assert rc == 0

    def step():
        strip_pass()
        variant_pass()
        if W > 1:
            exchange()

    for _ in range(ctx.args.warmup):
        step()
    torch.cuda.synchronize()
    tot = pcount.clone()
    if W > 1:
        ctx.dist.all_reduce(tot)
    got_all = [int(x) for x in tot.tolist()]
    nsp_sharded, got = got_all[0], got_all[1:]
    # known answers: per-copy counts x copies + matches across copy seams
    stripped_one = bytes(seq[: kc["stripped_len"]].cpu().numpy())
    ok = nsp_sharded == nsp
    for v, g in zip(kc["variants"], got):
        o = OracleRegex(R.Regex(v["re"]))
        seam = len(o.find_iter(stripped_one * 2)) - 2 * v["count"]
        ok = ok and g == v["count"] * copies + seam * (copies - 1)
    ctx.ramp(variant_pass)
    sec = ctx.timed(step)
    # host time to enqueue one variant phase (no sync inside): the phase is
    # ~100 launches and stream-ordered allocations behind one long kernel
    torch.cuda.synchronize()
    hts = []
    for _ in range(ctx.args.steps):
        t0 = time.perf_counter()
        variant_pass()
        hts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    strip_ms = ctx.kernel_ms(strip_pass)
    var_ms = ctx.kernel_ms(variant_pass)
    pipe = shootout_pipeline(ctx, big, N, copies, kc, variants) if W == 1 else None
    # the dominant kernel of each phase timed live (HIP events the library
    # records around the speculative kernel on the launch stream)
    lex_ms, lex_n = kernel_timer_ms(strip_pass, ctx.args.steps)
    spec_ms, spec_n = kernel_timer_ms(variant_pass, ctx.args.steps)
    fused = not ctx.args.c3_separate
    strip_bytes = (N + W - 1) // W
    scanned = N + len(variants) * M   # regex-bytes: the stripped stream once per variant
    var_bytes = v_hi - v_lo      # the rank's span of the stripped stream
    extra = {"variant_host_enqueue_ms": round(float(np.median(hts)) * 1e3, 3)}
    if ctx.rank == 0 and not ctx.args.no_cpu:
        extra["cpu_baseline"] = cpu_baseline_c3(strip, raw, variants, seq, M, got, ctx.args)
    # bytes the step must move: the raw text read by the strip pass, the
    # stripped stream read once by the fused variant pass (9 times when
    # separate), and the match records written (16 B each)
    var_matches = sum(got) // W
    # the fused pass runs the k-mer probe engine when every variant is a set
    # of 8-byte strings (all 9 are) unless the debug knob kmer=0 is set
    kmer = "kmer=0" not in os.environ.get("RURE_AMD_DEBUG", "")
    var_kernel = ("iter_spec_kmer_multi_tile" if kmer else "iter_spec_sa_multi_tile") if fused else "iter_spec_sa_tile"
    step_bytes = strip_bytes + var_bytes * (1 if fused else len(variants)) + 16 * (nsp_sharded // W + var_matches)
    config = {"workload": "C3: regex-dna x%d (%d B raw, %d B stripped): strip find_iter + 9 variant find_iter"
                          % (copies, N, M),
              "parallelism": "span%d (one logical stream cut into %d contiguous spans, exit exchange per step)"
                             % (W, W)}
    # value: haystack bytes per second, each haystack (raw text, stripped
    # stream) counted once; regex_bytes_GBps counts the stripped stream once
    # per variant (the 9 find_iter the reference runs)
    return ctx.line("haystack GB/s scanned, batched bytes::Regex::find_iter (regex-dna)",
                    (N + M) / sec / 1e9, "GB/s", sec * 1e3, "u8",
                    "examples/regexdna-input.txt replicated", config, scaling="strong",
                    regex_bytes_GBps=round(scanned / sec / 1e9, 1),
                    strip_pass_ms=round(strip_ms, 3), strip_GBps=round(strip_bytes / strip_ms / 1e6, 1),
                    variant_phase_ms=round(var_ms, 3),
                    variant_phase_GBps=round(var_bytes / var_ms / 1e6, 1),
                    strip_matches=nsp_sharded, variant_counts=got, known_answers_ok=ok,
                    variant_engine="separate passes" if ctx.args.c3_separate else "one fused pass",
                    cut_recomputations=stats["recomputed"],
                    **({} if pipe is None else pipe),
                    roofline=roofline_kernel(var_bytes, spec_ms, spec_n, config, var_kernel,
                                             "variant speculative kernel (%s)" %
                                             ("%s_kernel: one read of the stripped span for all 9 variants"
                                              % var_kernel if fused else
                                              "iter_spec_sa_tile_kernel, one launch per variant")),
                    roofline_strip=roofline_kernel(strip_bytes, lex_ms, lex_n, config,
                                                   "iter_spec_lex_tile",
                                                   "strip speculative kernel (iter_spec_lex_tile_kernel: one read "
                                                   "of the raw text)"),
                    roofline_variant_phase={"bound": "hbm", "achieved": round(var_bytes / var_ms / 1e6, 1),
                                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                            "frac": round(var_bytes / var_ms / 1e6 / HBM_PEAK_GBS, 4),
                                            "ms": round(var_ms, 4), "alg_bytes": int(var_bytes),
                                            "what": "whole variant phase (speculative kernel + each variant's "
                                                    "fix/walk/emit/count kernels), HIP events"},
                    roofline_step={"bound": "hbm", "achieved": round(step_bytes / sec / 1e9, 1),
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": round(step_bytes / sec / 1e9 / HBM_PEAK_GBS, 4),
                                   "ms": round(sec * 1e3, 4), "alg_bytes_per_step": int(step_bytes),
                                   "what": "whole step: raw text read once (strip), stripped stream read %s, "
                                           "match records written; driver-visible time incl. launch gaps"
                                           % ("once (fused variant pass)" if fused else "once per variant")},
                    **extra)


def shootout_pipeline(ctx, big, N, copies, kc, variants):
    """The whole regex-dna program (examples/shootout-regex-dna-bytes.rs:16-66)
    on the device through the C ABI (regex_amd/shootout.py): strip
    replace_all, the 9 variant counts in one fused pass, the 11 IUB
    substitutions chained; timed end to end (host syncs included: each
    replacement reads its output length back to size the next buffer).
    Known answers: the lengths of examples/regexdna-output.txt x copies, and
    each variant's count x copies plus the matches across copy seams."""
    import regex_amd as R
    from regex_amd.shootout import RegexDna
    from oracle_py import OracleRegex
    torch = ctx.torch
    dna = RegexDna()
    out = dna.run(big, N, stream=ctx.stream)
    one = R.Regex(kc["strip"]).replace_all(corpus_regexdna(), b"")
    ok = out["ilen"] == kc["input_len"] * copies and out["clen"] == kc["stripped_len"] * copies and \
        out["slen"] == kc["substituted_len"] * copies
    for v, got in zip(kc["variants"], out["counts"]):
        seam = len(OracleRegex(R.Regex(v["re"])).find_iter(one * 2)) - 2 * v["count"]
        ok = ok and got == v["count"] * copies + seam * (copies - 1)
    times = []
    for _ in range(max(1, ctx.args.steps)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dna.run(big, N, stream=ctx.stream)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ms = float(np.median(times)) * 1e3
    return {"pipeline_ms": round(ms, 3), "pipeline_GBps": round(N / ms / 1e6, 1),
            "pipeline_known_answers_ok": bool(ok),
            "pipeline": {"what": "shootout-regex-dna-bytes.rs end to end on the device (regex_amd/shootout.py): "
                                 "strip replace_all + 9 variant counts (one fused pass) + 11 IUB replace_all, "
                                 "median of %d runs, host syncs included" % len(times),
                         "lengths": [out["ilen"], out["clen"], out["slen"]], "counts": out["counts"]}}


def corpus_regexdna():
    from golden_data import corpus
    return corpus("regexdna")


def kernel_timer_ms(fn, steps):
    """Average duration of the find_iter speculative kernel of fn() over
    `steps` calls (rure_amd_kernel_timer: HIP events on the launch stream)."""
    import ctypes
    from regex_amd import _native as NN
    NN.rure_amd_kernel_timer(1)
    for _ in range(steps):
        fn()
    n = ctypes.c_uint64(0)
    ms = NN.rure_amd_kernel_timer_read(ctypes.byref(n))
    NN.rure_amd_kernel_timer(0)
    return float(ms), int(n.value)


def roofline_kernel(alg_bytes, ms, launches, config, kernel, what):
    """Roofline of one kernel: algorithmic bytes per launch / its average
    launch duration (live HIP events); traffic = HBM bytes per launch from the
    committed PMC pass of this command (profiles/*_summary.json)."""
    a = alg_bytes / ms / 1e6 if ms > 0 else 0.0
    r = {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(a / HBM_PEAK_GBS, 4), "traffic": None, "kernel_ms": round(ms, 4),
         "launches_timed": launches, "alg_bytes_per_launch": int(alg_bytes), "kernel": what}
    tr = profiled_traffic(config, alg_bytes, kernel=kernel)
    if tr is not None:
        r["traffic"] = tr["bytes"]
        r["traffic_source"] = tr["source"]
    return r


def cpu_baseline_c3(strip, raw, variants, seq, M, gpu_counts, args):
    """The C3 step on the CPU the way the reference's shootout runs it
    (examples/shootout-regex-dna-bytes.rs): the strip replace_all on one
    thread (:21), then the 9 variant find_iter counts on one thread each
    (:37-42), with the oracle (restated lazy DFA + re_trait.rs:197-221
    iteration) as the engine.  Sample: the first `copies` whole copies of the
    input (about 32 MiB raw), repeated for --cpu-seconds; its stripped output
    and variant counts are checked against the GPU's."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    copies = max(1, (32 << 20) // len(raw))
    text = raw * copies
    R_ = len(text)
    o_strip = OracleRegex(strip)
    os_ = [OracleRegex(v) for v in variants]

    def strip_once(cap=None):
        sp = o_strip.find_iter_array(text, cap=cap)
        # replace_all(.., "") = the bytes outside the matches
        a = np.frombuffer(text, dtype=np.uint8)
        d = np.zeros(R_ + 1, dtype=np.int32)
        # the spans are disjoint and non-empty here: starts (and ends) are
        # distinct, so plain fancy-index updates (np.add.at is ~10x slower)
        d[sp[:, 0].astype(np.int64)] += 1
        d[sp[:, 1].astype(np.int64)] -= 1
        keep = np.cumsum(d[:R_]) == 0
        return sp.shape[0], a[keep].tobytes()

    nstrip, stripped = strip_once()
    S = len(stripped)
    res = [None] * len(os_)

    def var_thread(i, cap):
        res[i] = os_[i].find_iter_array(stripped, cap=cap).shape[0]

    def variants_once(caps):
        th = [threading.Thread(target=var_thread, args=(i, caps[i])) for i in range(len(os_))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return list(res)

    exp = variants_once([None] * len(os_))
    caps = [c + 16 for c in exp]
    t_strip = t_var = 0.0
    passes = 0
    while (t_strip + t_var) < args.cpu_seconds and passes < 64:
        t0 = time.perf_counter()
        strip_once(nstrip + 16)
        t1 = time.perf_counter()
        variants_once(caps)
        t2 = time.perf_counter()
        t_strip += t1 - t0
        t_var += t2 - t1
        passes += 1
    gpu_strip = bytes(seq[:S].cpu().numpy())
    got = [int(v.find_iter_batch(seq[:S + 16], stride=S, length=S, count=1)[0][0]) for v in variants]
    sec = (t_strip + t_var) / passes
    return {"value": round((R_ + S) / sec / 1e9, 3), "unit": "GB/s", "cores": len(os_),
            "kind": "port",
            "regex_bytes_GBps": round((R_ + len(os_) * S) / sec / 1e9, 3),
            "strip_GBps_1thread": round(R_ * passes / t_strip / 1e9, 3),
            "variants_GBps_9threads": round(len(os_) * S * passes / t_var / 1e9, 3),
            "sample": "%d passes over %d copies of the input (%.1f MiB raw -> %.1f MiB stripped): strip "
                      "replace_all on 1 thread, then the 9 variant find_iter on 9 threads (one per variant, "
                      "shootout-regex-dna-bytes.rs:37-42)" % (passes, copies, R_ / 2**20, S / 2**20),
            "engine_path": {"strip": "MatchType::Dfa with the start-state prefix skip: SingleByteSet {'>', '\\n'} "
                                     "via memchr2 (dfa.rs:700-711, literals.rs:353-361), then a reverse DFA per "
                                     "match (exec.rs:632-662)",
                            "variants": "MatchType::Literal(Unanchored) (exec.rs:1148-1155): the literal searcher "
                                        "(Teddy / Aho-Corasick in the reference; here one forward pass with a "
                                        "4-byte hash prefilter, literals.rs:92-103), no DFA"},
            "reference_published": {"strip_MBps": 343, "source": "bench/log/05/rust:42 (regex-dna strip "
                                    "`>[^\\n]*\\n|\\n` on the reference's own machine)",
                                    "ratio_of_strip_1thread": round(R_ * passes / t_strip / 1e9 * 1e3 / 343, 3)},
            "parity_on_sample": bool(gpu_strip == stripped and exp == got)}


# ------------------------------------------------------------------ C4
def run_c4(ctx):
    import regex_amd as R
    from regex_amd.workloads import C4_PATTERNS, log_lines_device
    torch = ctx.torch
    n = 10_000_000
    buf, offs = log_lines_device(n, ctx.dev, seed=0x5EED0004 ^ ctx.rank)
    rs = R.RegexSet(C4_PATTERNS)
    out = torch.empty(n, dtype=torch.int64, device=ctx.dev)

    def scan():
        rs.matches_batch(buf, offsets=offs, out=out, stream=ctx.stream)

    ctx.ramp(scan)
    sec = ctx.timed(scan)
    kms = ctx.kernel_ms(scan)
    nb = int(offs[-1].item())
    config = {"workload": "C4: RegexSet of %d patterns over %d log lines (%d B) per GPU" % (len(C4_PATTERNS), n, nb),
              "parallelism": "dp%d" % ctx.world}
    extra = {}
    if ctx.rank == 0 and not ctx.args.no_cpu:
        extra["cpu_baseline"] = cpu_baseline_c4(rs, buf, offs, out, ctx.args)
    return ctx.line("haystack GB/s scanned, batched RegexSet::matches", nb * ctx.world / sec / 1e9, "GB/s",
                    sec * 1e3, "u8", "synthetic log lines (seeded token stream)", config,
                    lines_per_s=round(n * ctx.world / sec, 1),
                    roofline=roofline(nb / kms / 1e6, kms, nb, config), **extra)


def cpu_baseline_c4(rs, buf, offs, out, args):
    """Oracle set matcher (restated DfaMany lazy DFA, dfa.rs:525-570) on the
    first lines of the same batch; re-checks the GPU masks of the sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    threads = cpu_threads(args.cpu_threads)
    o = OracleRegex(rs)
    S = 500_000
    so = offs[: S + 1].cpu().numpy().astype(np.uint64)
    hb = buf[: int(so[-1])].cpu().numpy()
    t0 = time.perf_counter()
    exp = o.set_batch(hb, 0, 0, S, nthreads=threads, offsets=so)
    passes, elapsed = 1, time.perf_counter() - t0
    while elapsed < args.cpu_seconds and passes < 64:
        t0 = time.perf_counter()
        o.set_batch(hb, 0, 0, S, nthreads=threads, offsets=so)
        elapsed += time.perf_counter() - t0
        passes += 1
    got = out[:S].cpu().numpy().view(np.uint64)
    # the engine path the reference takes on these lines: its 2 MiB lazy-DFA
    # cache outgrows dfa_size_limit, and after three flushes clear_cache
    # refuses to flush again within 10 x (states) bytes of the last flush
    # (dfa.rs:1282-1293, flush_count never resets), so the DFA quits and the
    # line is answered by the Pike VM (exec.rs:1019-1030)
    _, st = o.set_batch(hb, 0, 0, S, nthreads=threads, offsets=so, stats=True)
    d = {"value": round(int(so[-1]) * passes / elapsed / 1e9, 3), "unit": "GB/s",
         "kind": "port", "lines_per_s": round(S * passes / elapsed, 1),
         "engine_path": {"lines": S, "dfa_quits_to_pike_vm": int(st["quits"]),
                         "lazy_dfa_cache_flushes": int(st["flushes"]),
                         "cached_states_at_end": int(st["states"]), "threads": threads,
                         "what": "DfaMany lazy DFA (dfa.rs:525-570) with the reference's 2 MiB cache and flush "
                                 "policy; a line whose DFA quits is re-run on the Pike VM (pikevm.rs)"},
         "sample": "%d passes over the first %d lines (%.0f MiB) of the same batch" % (passes, S, so[-1] / 2**20),
         "parity_on_sample": bool(np.array_equal(exp, got))}
    d.update(cpu_info(threads))
    return d


# ------------------------------------------------------------------ C5
def run_c5(ctx):
    import regex_amd as R
    from regex_amd.dist import RecordGather
    torch = ctx.torch
    L = 16 << 30
    g = torch.Generator(device=ctx.dev)
    g.manual_seed(0x5EED0005 ^ ctx.rank)
    hay = torch.empty(L + 16, dtype=torch.uint8, device=ctx.dev)
    chunk = 1 << 30
    for s in range(0, L, chunk):
        v = torch.randint(0, 94, (min(chunk, L - s),), generator=g, device=ctx.dev, dtype=torch.int32)
        v = v + 32
        v = torch.where(v >= 64, v + 1, v)         # printable ASCII without '@'
        hay[s:s + v.numel()] = v.to(torch.uint8)
        del v
    hay[L:] = 0
    pos = L - (1 << 20) + 4096 * (ctx.rank + 1)
    plant = b" user@example.org "
    hay[pos:pos + len(plant)] = torch.frombuffer(bytearray(plant), dtype=torch.uint8).to(ctx.dev)
    re = R.Regex(r"\w+@\w+\.\w+")
    out = torch.empty((1, 2), dtype=torch.int64, device=ctx.dev)
    gather = RecordGather(1, ctx.dev) if ctx.world > 1 else None

    def scan():
        re.find_batch(hay, stride=L, length=L, count=1, out=out, stream=ctx.stream)

    def step():
        scan()
        if gather is not None:
            gather.step(out, ctx.rank, ctx.stream)

    scan()
    torch.cuda.synchronize()
    got = [int(x) for x in out[0].cpu()]
    ctx.ramp(scan)
    sec = ctx.timed(step)
    kms = ctx.kernel_ms(scan)
    config = {"workload": "C5: find \\w+@\\w+\\.\\w+ over one 16 GiB haystack per GPU", "haystack_bytes": L,
              "parallelism": "dp%d" % ctx.world}
    extra = {}
    if gather is not None:
        recs, _ = gather.result()
        extra["gathered_records"] = recs.cpu().tolist()
    if ctx.rank == 0 and not ctx.args.no_cpu:
        extra["cpu_baseline"] = cpu_baseline_c5(re, hay, pos, plant, ctx)
    return ctx.line("haystack GB/s scanned, bytes::Regex::find over 16 GiB shards", L * ctx.world / sec / 1e9,
                    "GB/s", sec * 1e3, "u8", "synthetic (seeded printable ASCII without '@', one planted address)",
                    config, match=got, expected=[pos + 1, pos + len(plant) - 1],
                    roofline=roofline(L / kms / 1e6, kms, L, config), **extra)


def cpu_baseline_c5(re, hay, pos, plant, ctx):
    """One `find` over one haystack is one sequential lazy-DFA scan in the
    reference (exec.rs:473-514), so the oracle runs single-threaded on the
    shard's last 256 MiB (which holds the planted address); the GPU's answer
    on the same slice is re-checked."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    torch = ctx.torch
    S = 256 << 20
    L = hay.numel() - 16
    lo = L - S
    piece = hay[lo:L].cpu().numpy()
    o = OracleRegex(re)
    t0 = time.perf_counter()
    exp, _ = o.find_batch(piece, S, S, 1, nthreads=1)
    passes, elapsed = 1, time.perf_counter() - t0
    while elapsed < ctx.args.cpu_seconds and passes < 16:
        t0 = time.perf_counter()
        o.find_batch(piece, S, S, 1, nthreads=1)
        elapsed += time.perf_counter() - t0
        passes += 1
    sub = torch.empty((1, 2), dtype=torch.int64, device=ctx.dev)
    re.find_batch(hay[lo:], stride=S, length=S, count=1, out=sub, stream=ctx.stream)
    torch.cuda.synchronize()
    return {"value": round(S * passes / elapsed / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "%d passes of find over the shard's last %d MiB (one sequential scan, as the reference's "
                      "single-haystack find)" % (passes, S >> 20),
            "engine_path": "MatchType::Dfa (Unicode \\w: no literal prefixes or suffixes): lazy DFA forward + "
                           "reverse (exec.rs:632-662)",
            "parity_on_sample": [int(x) for x in exp[0]] == [int(x) for x in sub[0].cpu()] ==
                                [pos - lo + 1, pos - lo + len(plant) - 1]}


def launch_ranks(n):
    """Start n rank processes of this same command (one per GPU) and relay rank
    0's JSON line.  The parent never touches the GPU (no torch import) and does
    not exec: the ranks are children.  If a rank fails, the others are stopped
    and the exit status is non-zero."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None))
    out0 = procs[0].stdout
    lines = []
    rc = 0
    while any(p.poll() is None for p in procs):
        failed = [p for p in procs if p.poll() not in (None, 0)]
        if failed:
            rc = failed[0].returncode
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            break
        time.sleep(0.2)
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    lines = out0.read().decode().splitlines()
    rc = rc or max(abs(p.returncode) for p in procs)
    for ln in lines:
        print(ln, flush=True)
    return rc


def run_rehearsal(ctx):
    """CPU-only rehearsal of the N-rank protocol (launcher, barrier + max over
    ranks timing, fixed-capacity record gather) with synthetic find results;
    no kernel runs.  tests/test_bench_launch.py drives it with gloo."""
    import torch
    from regex_amd.dist import RecordGather
    n = 4096
    g = torch.Generator().manual_seed(1234 + ctx.rank)
    found = torch.full((n, 2), -1, dtype=torch.int64)
    hit = torch.randperm(n, generator=g)[: 100 + ctx.rank]
    found[hit, 0] = hit
    found[hit, 1] = hit + 10
    gather = RecordGather(512, ctx.dev)
    sec = ctx.timed(lambda: gather.step(found, ctx.rank * n))
    recs, counts = gather.result()
    exp = []
    for r in range(ctx.world):
        m = torch.full((n, 2), -1, dtype=torch.int64)
        h = torch.randperm(n, generator=torch.Generator().manual_seed(1234 + r))[: 100 + r]
        m[h, 0], m[h, 1] = h, h + 10
        idx = (m[:, 0] >= 0).nonzero().squeeze(1)
        exp.append(torch.stack([idx + r * n, m[idx, 0], m[idx, 1]], 1))
    ok = bool(torch.equal(recs, torch.cat(exp)))
    return ctx.line("rehearsal", n * ctx.world / sec, "haystacks/s", sec * 1e3, "int64", "synthetic find results",
                    {"workload": "rehearsal", "parallelism": "dp%d" % ctx.world}, gathered_records=int(recs.shape[0]),
                    gather_ok=ok, counts=counts)


BIG_PATTERN = r"[a-q][^u-z]{13}x"


def run_big(ctx):
    """A forward DFA past the u16 tables (SURVEY §8 a7 / VERDICT r2 item 7):
    `[a-q][^u-z]{13}x` builds 73,725 states, run by big_dfa.hip from u32
    column tables (hot rows in LDS, the rest from L2 / Infinity Cache).  The
    Pike VM that served such automata before is timed once beside it; parity
    against the oracle on a sample."""
    import regex_amd as R
    from regex_amd import _native as NN
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    torch, args = ctx.torch, ctx.args
    n, L = 1 << 18, 4096
    # letters a-w with an `x` planted about every 2 KiB: most haystacks are
    # scanned to their end (a match needs the 14 bytes before an `x` to fit)
    g = torch.Generator(device=ctx.dev).manual_seed(0xB16 + ctx.rank)
    hay = (torch.randint(0, 23, (n * L + 16,), generator=g, device=ctx.dev, dtype=torch.uint8) + ord("a"))
    xs = torch.randint(0, n * L, (n * L // 2048,), generator=g, device=ctx.dev)
    hay[xs] = ord("x")
    t0 = time.perf_counter()
    re = R.Regex(BIG_PATTERN)
    info = re.dfa_info(3)
    build_s = time.perf_counter() - t0
    out = torch.empty((n, 2), dtype=torch.int64, device=ctx.dev)

    def scan():
        re.find_batch(hay, stride=L, length=L, count=n, out=out, stream=ctx.stream)

    ctx.ramp(scan)
    assert NN.rure_amd_last_fwd_path() == -6, "big-DFA kernel not taken"
    sec = ctx.timed(scan)
    kms = ctx.kernel_ms(scan)
    res = out.cpu().numpy()
    # Pike VM on the same batch (debug knob big=0, read per call), untimed
    pk = out.clone()
    with R.debug(big=0):
        torch.cuda.synchronize()
        tp = time.perf_counter()
        re.find_batch(hay, stride=L, length=L, count=n, out=pk, stream=ctx.stream)
        torch.cuda.synchronize()
        pike_s = time.perf_counter() - tp
    same = bool(torch.equal(pk, out))
    # oracle parity on a sample of haystacks
    o = OracleRegex(re)
    sample = list(range(0, n, n // 512))
    buf = hay[: n * L].view(n, L)
    bad = 0
    for i in sample:
        e = o.find(bytes(buf[i].cpu().numpy()))
        gg = None if res[i, 0] < 0 else (int(res[i, 0]), int(res[i, 1]))
        bad += gg != e
    if bad:
        sys.stderr.write("PARITY FAILURE (big): %d of %d sampled haystacks differ\n" % (bad, len(sample)))
        sys.exit(3)
    m = res[:, 0] >= 0
    fwd = np.where(m, np.minimum(res[:, 1] + 1, L), L).sum()
    rev = (res[m, 1] - res[m, 0]).sum()
    b_alg = float(fwd + rev + 16 * n)
    config = {"workload": "big: find %s (%d-state forward DFA, u32 tables) over %d x %d B random lowercase "
                          "haystacks per GPU (a-w, an x per 2 KiB)" % (BIG_PATTERN, info["states"], n, L),
              "haystacks_per_gpu": n, "haystack_bytes": L, "parallelism": "dp%d" % ctx.world}
    extra = {}
    if ctx.rank == 0 and not args.no_cpu:
        reps, t1 = 0, time.perf_counter()
        cs = [bytes(buf[i].cpu().numpy()) for i in range(0, 2048)]
        while time.perf_counter() - t1 < min(args.cpu_seconds, 5.0):
            for h in cs:
                o.find(h)
            reps += 1
        el = time.perf_counter() - t1
        extra["cpu_baseline"] = {"value": round(len(cs) * L * reps / el / 1e9, 4), "unit": "GB/s", "cores": 1,
                                 "kind": "port", "sample": "%d passes over the first 2048 haystacks, one thread, "
                                                           "oracle lazy DFA" % reps}
    return ctx.line("haystack GB/s scanned, batched bytes::Regex::find (DFA > 65535 states)",
                    n * L * ctx.world / sec / 1e9, "GB/s", sec * 1e3, "u8", "synthetic (seeded random a-w, planted x)", config,
                    dfa_states=info["states"], dfa_columns=info["byte_classes"], dfa_build_s=round(build_s, 3),
                    matched_haystacks=int(m.sum()), kernel_ms=round(kms, 4),
                    pike_vm_GBps=round(n * L / pike_s / 1e9, 2), pike_vm_agrees=same,
                    parity={"haystacks_checked": len(sample), "mismatches": 0, "against": "oracle lazy DFA"},
                    roofline=roofline(b_alg / (kms * 1e-3) / 1e9, kms, b_alg, config), **extra)


def run_c1(ctx):
    """BASELINE configs[0]: the date regex `is_match` over 1K x 1 KiB ASCII
    buffers.  The batched GPU call (latency-bound at this size: one launch
    over 1 MiB) next to the oracle (restated reference lazy DFA) on the
    host, whole-batch parity."""
    import regex_amd as R
    from regex_amd.workloads import date_haystacks_host
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleRegex
    torch, args = ctx.torch, ctx.args
    n, L = 1024, 1024
    buf, planted = date_haystacks_host(n, L, seed=0x5EED0001 ^ ctx.rank, frac=0.5)
    hay = torch.from_numpy(buf).to(ctx.dev)
    re = R.Regex(PATTERN)
    out = torch.empty((n,), dtype=torch.uint8, device=ctx.dev)

    def scan():
        re.is_match_batch(hay, stride=L, length=L, count=n, out=out, stream=ctx.stream)

    ctx.ramp(scan)
    sec = ctx.timed(scan)
    kms = ctx.kernel_ms(scan)
    got = out.cpu().numpy().astype(bool)
    o = OracleRegex(re)
    exp = o.is_match_batch(buf, L, L, n, nthreads=1).astype(bool)
    if not np.array_equal(got, exp):
        sys.stderr.write("PARITY FAILURE (c1): %d haystacks differ\n" % int((got != exp).sum()))
        sys.exit(3)
    extra = {}
    if ctx.rank == 0 and not args.no_cpu:
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min(args.cpu_seconds, 5.0):
            o.is_match_batch(buf, L, L, n, nthreads=1)
            reps += 1
        el = time.perf_counter() - t0
        extra["cpu_baseline"] = {"value": round(n * L * reps / el / 1e9, 3), "unit": "GB/s", "cores": 1,
                                 "kind": "port", "sample": "%d passes of the whole 1K x 1 KiB batch, one thread (the "
                                                           "reference's is_match is one call per buffer)" % reps}
    config = {"workload": "C1: is_match %s over %d x %d B ASCII buffers" % (PATTERN, n, L),
              "haystacks_per_gpu": n, "haystack_bytes": L, "parallelism": "dp%d" % ctx.world}
    return ctx.line("haystack GB/s scanned, batched bytes::Regex::is_match", n * L * ctx.world / sec / 1e9, "GB/s",
                    sec * 1e3, "u8", "synthetic (seeded printable ASCII, 20% digits, 50% planted dates)", config,
                    matched_haystacks=int(got.sum()), parity={"haystacks_checked": n, "mismatches": 0},
                    kernel_ms=round(kms, 4), note="latency-bound: one launch over 1 MiB", **extra)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    ctx = Ctx(args)
    line = {"c1": run_c1, "c2": run_c2, "c3": run_c3, "c4": run_c4, "c5": run_c5, "big": run_big,
            "rehearsal": run_rehearsal}[args.config](ctx)
    if ctx.rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
