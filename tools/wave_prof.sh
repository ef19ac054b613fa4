#!/bin/bash
# kernel trace of the wave-served find_iter bench (tools/wave_iter_bench.py)
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/wave_prof
mkdir -p $OUT
export TMPDIR=/tmp
export WAVE_TEXTS=as_is
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/wave_iter_bench.py '\b\w+n\b' > $OUT/bench.jsonl 2> $OUT/err.log
rc=$?; cat $OUT/bench.jsonl; echo "rc=$rc"
f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1); cut -c1-60,400- "$f" | head -14; python3 -c "import csv,sys; r=list(csv.DictReader(open(sys.argv[1]))); [print(x['Name'][:90], x['Calls'], x['TotalDurationNs'], x['MaxNs']) for x in r[:12]]" "$f"
exit $rc
