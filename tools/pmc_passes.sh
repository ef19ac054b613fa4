#!/bin/bash
# Counter passes (one rocprofv3 run per counter group) over tools/kbench_one.py.
TAG=${1:-pmc}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 "$R/tools/kbench_one.py" "$@" > "$OUT/p$i.log" 2>&1 || echo "pass $i failed"
done
echo pmc done
