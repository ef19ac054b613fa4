#!/bin/bash
# The round's final bench lines: every config with its CPU baseline, one
# process each under its own time limit; lines go to gpurun_out/<tag>/.
# usage: tools/final_lines.sh <tag>
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-final}
mkdir -p "$OUT"
cd "$R"
for c in c2 c1 c3 c4 c5; do
  echo "== $c ($(date +%T))"
  timeout -k 10 300 python bench.py --config $c > "$OUT/$c.json" 2> "$OUT/$c.err"
  rc=$?
  echo "== $c rc=$rc"
  tail -c 400 "$OUT/$c.json"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
