#!/bin/bash
# temporary: C4 timing under a kernel knob: tools/c4_exp.sh VAR v1 v2 ...
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/c4exp
var=$1; shift
for e in "$@"; do
  env $var=$e timeout -k 10 200 python bench.py --config c4 --no-cpu --steps 10 > gpurun_out/c4exp/e$e.json 2>&1 || exit 1
  echo "$var=$e $(python -c "import json;d=json.loads(open('gpurun_out/c4exp/e$e.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['roofline']['kernel_ms'])")"
done
