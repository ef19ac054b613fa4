#!/bin/bash
# round 6 final: per-config rocprofv3 kernel trace + FETCH_SIZE pass (written
# BEFORE the bench lines, so the lines cite this round's summaries)
R=$GRAFT_REPO_ROOT
cd $R
for c in c2 c1 c3 c4 c5; do
  echo "== profile $c ($(date +%T))"
  bash tools/gpu_profile.sh r06_$c --config $c --steps 5 || { echo "profile $c failed"; exit 1; }
done
echo "profiles done"
