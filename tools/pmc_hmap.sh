#!/bin/bash
# PMC passes over the shootout pipeline (tools/pipeline_prof.py): the chain's
# hmap kernels, one counter group per run
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/hmappmc/p$i -o pmc -- python3 $R/tools/pipeline_prof.py --reps 1 > $R/gpurun_out/hmappmc_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
