"""Synthetic, seeded haystack batches for the BASELINE.json configurations
(SURVEY.md §8d).  Generated on the device so the 4 GiB / 16 GiB batches never
cross PCIe; small batches for parity tests can be generated on the host with
the same recipe (numpy) and copied over.

C1/C2 recipe: printable ASCII (0x20-0x7E) with ~20 % digits (to exercise
partial date matches); a fraction of the haystacks gets one planted
`YYYY-MM-DD` at a uniform offset.
"""
import numpy as np

DATE_LEN = 10


def _plant_dates_np(buf, n, L, frac, rng):
    k = int(round(n * frac))
    idx = rng.choice(n, size=k, replace=False) if k else np.zeros(0, dtype=np.int64)
    offs = rng.integers(0, max(L - DATE_LEN, 0) + 1, size=k)
    digits = rng.integers(0, 10, size=(k, DATE_LEN)).astype(np.uint8) + ord("0")
    digits[:, 4] = ord("-")
    digits[:, 7] = ord("-")
    for j in range(k):
        o = int(idx[j]) * L + int(offs[j])
        buf[o:o + DATE_LEN] = digits[j]
    return np.sort(idx)


def date_haystacks_host(n, L, seed, frac=0.01, digit_frac=0.2):
    """Host (numpy) batch: n x L bytes, fixed stride L."""
    rng = np.random.default_rng(seed)
    r = rng.integers(0, 1 << 31, size=n * L, dtype=np.int64)
    is_digit = (r % 1000) < int(digit_frac * 1000)
    v = (r >> 10)
    buf = np.where(is_digit, ord("0") + v % 10, 0x20 + v % 95).astype(np.uint8)
    planted = _plant_dates_np(buf, n, L, frac, rng)
    return buf, planted


def date_haystacks_device(n, L, seed, device, frac=0.01, digit_frac=0.2, chunk=1 << 28):
    """Device (torch) batch of the same recipe; returns (uint8 tensor, planted idx)."""
    import torch
    total = n * L
    out = torch.empty(total, dtype=torch.uint8, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    for s in range(0, total, chunk):
        e = min(total, s + chunk)
        r = torch.randint(0, 1 << 31, (e - s,), generator=g, device=device, dtype=torch.int64)
        is_digit = (r % 1000) < int(digit_frac * 1000)
        v = r >> 10
        out[s:e] = torch.where(is_digit, 48 + v % 10, 32 + v % 95).to(torch.uint8)
        del r, is_digit, v
    rng = np.random.default_rng(seed ^ 0x5EED)
    k = int(round(n * frac))
    idx = np.sort(rng.choice(n, size=k, replace=False)) if k else np.zeros(0, dtype=np.int64)
    offs = rng.integers(0, max(L - DATE_LEN, 0) + 1, size=k)
    digits = rng.integers(0, 10, size=(k, DATE_LEN)).astype(np.uint8) + ord("0")
    digits[:, 4] = ord("-")
    digits[:, 7] = ord("-")
    if k:
        pos = torch.from_numpy((idx * L + offs)[:, None] + np.arange(DATE_LEN)[None, :]).to(device)
        out[pos.reshape(-1)] = torch.from_numpy(digits.reshape(-1)).to(device)
    return out, idx


# ------------------------------------------------------------------- C4
# 64 small patterns over synthetic log lines: literals,
# classes, counted repeats, anchors, alternations, a few word boundaries.
C4_PATTERNS = [
    r"ERROR", r"WARN", r"INFO", r"DEBUG", r"FATAL", r"(?i)timeout", r"(?i)exception", r"panic:",
    r"status=[45]\d\d", r"status=2\d\d", r"status=3\d\d", r"user=\w+", r"uid=\d+", r"session=[0-9a-f]{8}",
    r"\d+\.\d+\.\d+\.\d+", r"port=\d{2,5}", r"^GET ", r"^POST ", r"^PUT ", r"^DELETE ", r"ms$", r"s$",
    r"latency=\d+ms", r"size=\d+[KMG]B", r"/api/v\d+/", r"/static/", r"\.php", r"\.js\b", r"HTTP/1\.[01]",
    r"HTTP/2", r"retry=\d", r"attempt \d+ of \d+", r"(?i)failed", r"(?i)denied", r"(?i)success",
    r"conn(ection)? reset", r"disk (full|quota)", r"cpu=\d{2,3}%", r"mem=\d+MB", r"\[[A-Z]+\]",
    r"id=[A-Z]{3}-\d{4}", r"[a-z]+@[a-z]+\.com", r"https?://[a-z.]+", r"\bkernel\b", r"sshd\[\d+\]",
    r"^\d{4}-\d{2}-\d{2}", r"T\d{2}:\d{2}:\d{2}", r"Z$", r"\+\d{2}:\d{2}", r"level=(warn|error)",
    r"trace_id=[0-9a-f]{16}", r"span=\d+", r"queue=[a-z_]+", r"shard-\d+", r"node\d{1,3}", r"region=us-\w+",
    r"(?i)deadlock", r"oom", r"killed", r"exit code [1-9]\d*", r"code=E\d{3}", r"v\d+\.\d+\.\d+", r"=null\b",
    r"\bnil\b",
]

_C4_WORDS = [
    "GET", "POST", "PUT", "DELETE", "ERROR", "WARN", "INFO", "DEBUG", "FATAL", "Timeout", "exception",
    "panic:", "kernel", "sshd[{d}]", "user=alice", "user=bob_{d}", "uid={d}", "session={h8}", "status={s}",
    "port={d}", "latency={d}ms", "size={d}KB", "/api/v{d}/items", "/static/app.js", "/index.php",
    "HTTP/1.1", "HTTP/2", "retry={d}", "attempt {d} of {d}", "failed", "Denied", "SUCCESS",
    "connection reset", "conn reset", "disk full", "disk quota", "cpu={d}%", "mem={d}MB", "[AUTH]",
    "id=ABC-{d4}", "ops@example.com", "https://example.org", "2017-12-30T12:34:56Z", "+05:30",
    "level=warn", "level=error", "trace_id={h8}{h8}", "span={d}", "queue=jobs_main", "shard-{d}",
    "node{d}", "region=us-east", "deadlock", "oom", "killed", "exit code {d}", "code=E{d3}", "v1.2.{d}",
    "x=null", "nil", "10.0.{d}.{d}", "ms", "s", "ok", "the", "request", "served", "in", "from", "to",
]


def _c4_stream(seed, nbytes):
    """A seeded token stream (host bytes) and the offsets of token starts."""
    rng = np.random.default_rng(seed)
    out, starts, size = [], [], 0
    hexd = "0123456789abcdef"
    while size < nbytes:
        w = _C4_WORDS[int(rng.integers(len(_C4_WORDS)))]
        while "{" in w:
            a = w.index("{")
            b = w.index("}", a)
            kind = w[a + 1:b]
            if kind == "d":
                v = str(int(rng.integers(0, 100000)) >> int(rng.integers(0, 16)))
            elif kind == "d3":
                v = "%03d" % int(rng.integers(0, 1000))
            elif kind == "d4":
                v = "%04d" % int(rng.integers(0, 10000))
            elif kind == "s":
                v = str(int(rng.integers(100, 600)))
            else:
                v = "".join(hexd[int(x)] for x in rng.integers(0, 16, 8))
            w = w[:a] + v + w[b + 1:]
        tok = (w + " ").encode()
        starts.append(size)
        out.append(tok)
        size += len(tok)
    return np.frombuffer(b"".join(out), dtype=np.uint8), np.asarray(starts, dtype=np.int64)


def log_lines_host(n, seed=0x5EED0004, lo=40, hi=160):
    """n lines, length uniform in [lo, hi], each a window of the token stream
    starting at a token.  Returns (buf uint8, offsets int64 (n+1))."""
    s, st = _c4_stream(seed, 1 << 22)
    rng = np.random.default_rng(seed ^ 0xC4)
    lens = rng.integers(lo, hi + 1, size=n)
    ok = st[st + hi < len(s)]
    starts = ok[rng.integers(0, len(ok), size=n)]
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    idx = np.repeat(starts - offs[:-1], lens) + np.arange(offs[-1])
    return s[idx], offs


def log_lines_device(n, device, seed=0x5EED0004, lo=40, hi=160, chunk=1 << 20):
    """The same recipe generated on the device (the stream is built on the
    host once, ~4 MiB, then lines are gathered on the GPU)."""
    import torch
    s, st = _c4_stream(seed, 1 << 22)
    rng = np.random.default_rng(seed ^ 0xC4)
    lens = rng.integers(lo, hi + 1, size=n)
    ok = st[st + hi < len(s)]
    starts = ok[rng.integers(0, len(ok), size=n)]
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    sd = torch.from_numpy(s).to(device)
    buf = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device=device)
    buf[-16:] = 0
    lens_d = torch.from_numpy(lens).to(device)
    delta = torch.from_numpy(starts - offs[:-1]).to(device)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        o0, o1 = int(offs[a]), int(offs[b])
        pos = torch.arange(o0, o1, device=device)
        d = torch.repeat_interleave(delta[a:b], lens_d[a:b], output_size=o1 - o0)
        buf[o0:o1] = sd[pos + d]
        del pos, d
    return buf, torch.from_numpy(offs).to(device)
