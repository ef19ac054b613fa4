#!/bin/bash
# PMC passes over the C4 bench (set_core_kernel), one counter group per run.
# usage: tools/pmc_c4.sh [tag]   (RURE_AMD_DEBUG passes through to the bench)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-c4pmc}
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
           "SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/$TAG/p$i -o pmc -- python3 $R/bench.py --config c4 --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
