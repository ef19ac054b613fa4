#!/bin/bash
# Counter passes (one rocprofv3 run per group) over one command, for one
# kernel's counters: tools/pmc_kernel.sh <tag> <cmd...>
# (summaries: python tools/pmc_summary.py gpurun_out/<tag> <kernel substring>)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$@" > "$OUT/trace.log" 2>&1 || exit 1
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
           "FETCH_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- "$@" >> "$OUT/pmc.log" 2>&1 || exit 1
done
echo pmc done
