#!/bin/bash
# The round's measurements in one GPU call: GPU tests first (stop on any
# failure), then the bench lines of every config with their CPU baselines
# (tools/final_lines.sh), then per-config rocprofv3 kernel traces + FETCH_SIZE
# passes (tools/gpu_profile.sh); everything under gpurun_out/<tag>*.
# usage: tools/round_final.sh <tag> [pytest selection...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-final}; shift || true
cd "$R"
mkdir -p "gpurun_out/$TAG"
SEL=${*:-tests}
echo "== tests ($(date +%T))"
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread \
  > "gpurun_out/$TAG/tests.out" 2> "gpurun_out/$TAG/tests.err"
rc=$?
tail -3 "gpurun_out/$TAG/tests.out"
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
bash tools/final_lines.sh "${TAG}_lines" || exit $?
for c in c2 c3 c4 c5 c1; do
  echo "== profile $c ($(date +%T))"
  bash tools/gpu_profile.sh "${TAG}_$c" --config $c || exit $?
done
echo "round_final done"
