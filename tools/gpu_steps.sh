#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that ends
# with a test failure (exit 1) lets the next run, anything else (fault,
# abort, segfault, time limit) stops the call there.
# usage: tools/gpu_steps.sh <outdir> <seconds> <name> <cmd> [<seconds> <name> <cmd> ...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p "$OUT"
cd "$R"
while [ $# -ge 3 ]; do
  secs=$1; name=$2; cmd=$3; shift 3
  echo "== $name ($(date +%T))" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.out" 2> "$OUT/$name.err"
  rc=$?
  echo "== $name rc=$rc ($(date +%T))" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.out"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
exit 0
