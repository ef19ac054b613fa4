#!/bin/bash
# Counter passes (one rocprofv3 run per group, groups separated by ';' in $1)
# over one command: tools/pmc_groups.sh <tag> "<grp1>;<grp2>;..." <cmd...>
# (summaries: python tools/pmc_summary.py gpurun_out/<tag> <kernel substring>)
TAG=$1; GROUPS_=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
IFS=';' read -ra GS <<< "$GROUPS_"
for grp in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- "$@" >> "$OUT/pmc.log" 2>&1 || exit 1
done
echo pmc done
