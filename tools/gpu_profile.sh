#!/bin/bash
# Profile the headline bench with rocprofv3 (kernel trace + stats, then a
# separate FETCH_SIZE counter pass).  Writes under gpurun_out/<tag>/.
# usage: tools/gpu_profile.sh <tag> [bench args...]
set -e
TAG=${1:-prof}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$R/bench.py" --no-cpu "$@" > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o pmc -- \
  python3 "$R/bench.py" --no-cpu --steps 3 --warmup 1 "$@" > "$OUT/bench_pmc.json" 2> "$OUT/pmc.err"
echo "profile done"
