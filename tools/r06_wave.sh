#!/bin/bash
# the wave-served chunked find_iter: its tests, then the 1 GiB bench
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_iter_wave.py tests/test_gpu_iter_looks.py tests/test_gpu_sherlock_counts.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wave_tests.log 2>&1
rc=$?; tail -15 gpurun_out/wave_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/wave_iter_bench.py > gpurun_out/wave_iter_bench.jsonl 2> gpurun_out/wave_iter_bench.err
rc=$?; cat gpurun_out/wave_iter_bench.jsonl; tail -3 gpurun_out/wave_iter_bench.err; echo "bench rc=$rc"; exit $rc
