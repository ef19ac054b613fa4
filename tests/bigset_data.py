"""Pattern sets of more than 64 patterns (RegexSet has no size bound in the
reference: re_set.rs:86-213, compile.rs:162-198, rure.rs:468-566).  The GPU
runs them in groups of 64 consecutive patterns (runtime.hpp, rure_set)."""
from regex_amd.workloads import C4_PATTERNS

EXTRA = [
    r"GET", r"POST /api", r"user=alice", r"user=bob_\d+", r"uid=1\d*", r"session=[0-9a-f]{4}",
    r"status=404", r"status=5\d\d", r"port=80\b", r"latency=\d{3,}ms", r"size=\d+KB", r"/api/v1/",
    r"index\.php", r"app\.js", r"HTTP/1\.1", r"retry=[0-3]", r"attempt 1 of", r"(?i)fail", r"Denied",
    r"connection", r"disk", r"cpu=9\d%", r"mem=\d{3}MB", r"\[AUTH\]", r"id=ABC-0", r"ops@", r"example\.(com|org)",
    r"2017-12-30", r"T12:34", r"\+05:30", r"level=warn", r"trace_id=", r"span=0", r"queue=jobs", r"shard-1",
    r"node[0-4]", r"us-east", r"dead", r"oom\b", r"killed$", r"exit code 1", r"code=E0", r"v1\.2\.3",
    r"x=null", r"^nil", r"10\.0\.", r"\bms\b", r"^s ", r"ok$", r"the request", r"served in", r"from to",
    r"\d{6}", r"[A-Z]{4,}", r"\w+=\w+ \w+=\w+", r"^[a-z]+$", r"(?m)^INFO", r"[^ -~]", r"\s{2}", r"z+",
    r"q\w*u", r"(a|e)(i|o)", r"^\S+$", r"INFO.*ERROR", r"ERROR.*INFO", r"(?i)WARN\w*",
]

# 65 (64 + a one-pattern group), 100 and 130 patterns
SETS = {
    65: C4_PATTERNS + EXTRA[:1],
    100: C4_PATTERNS + EXTRA[:36],
    130: C4_PATTERNS + EXTRA[:66],
}
