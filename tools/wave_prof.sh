#!/bin/bash
# kernel trace of the wave-served find_iter bench (tools/wave_iter_bench.py)
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/wave_prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/wave_iter_bench.py '\b\w+n\b' > $OUT/bench.jsonl 2> $OUT/err.log
rc=$?; cat $OUT/bench.jsonl; echo "rc=$rc"
f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1); head -25 "$f"
exit $rc
