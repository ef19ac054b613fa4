#!/bin/bash
# wave-served units: tests, then the bench with and without the split stamps
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_iter_wave.py tests/test_gpu_iter_looks.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wave_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wave_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
WAVE_TEXTS=as_is timeout -k 10 300 python3 tools/wave_iter_bench.py > gpurun_out/wave_split.jsonl 2> gpurun_out/wave_split.err || exit 1
WAVE_TEXTS=as_is WAVE_KNOBS=wave_tables=0 timeout -k 10 300 python3 tools/wave_iter_bench.py >> gpurun_out/wave_split.jsonl 2>> gpurun_out/wave_split.err
rc=$?; cat gpurun_out/wave_split.jsonl; exit $rc
