#!/bin/bash
# the whole -m gpu suite, smoke(), then the wave-served find_iter bench
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_all.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/wave_iter_bench.py > gpurun_out/wave_iter_bench.jsonl 2> gpurun_out/wave_iter_bench.err
rc=$?; cat gpurun_out/wave_iter_bench.jsonl; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/nfa_time.py > gpurun_out/nfa_time.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/nfa_time.log; exit $rc
