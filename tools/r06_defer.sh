#!/bin/bash
# the deferred ASCII-shadow quit: its tests, then the shadow A/B (1 GiB)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_iter_looks.py tests/test_gpu_unicode_fixtures.py tests/test_c_api.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/defer_tests.log 2>&1
rc=$?; tail -3 gpurun_out/defer_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/shadow_bench.py '\w+\s+\w+' '(?m)^\w+' '\w+@\w+\.\w+' > gpurun_out/shadow_defer.jsonl 2> gpurun_out/shadow_defer.err
rc=$?; cat gpurun_out/shadow_defer.jsonl; echo "bench rc=$rc"; exit $rc
