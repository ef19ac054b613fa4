#!/bin/bash
# Kernel trace of tools/replace_bench.py (strip + one IUB substitution on the
# 2 GiB regex-dna stream): per-kernel times under gpurun_out/<tag>/.
# usage: tools/prof_replace.sh <tag>   (env passes through: RURE_AMD_DEBUG=replace_generic=1 ...)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-repprof}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$R/tools/replace_bench.py" > "$OUT/bench.txt" 2> "$OUT/trace.err" || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/run_kernel_stats.csv", recursive=True) + glob.glob(sys.argv[1] + "/trace/run_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("%-70s %6s calls  avg %10.1f us  total %8.2f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
