#!/bin/bash
# round 6: replace tests + the shootout pipeline stages and kernel trace
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_replace_class.py tests/test_gpu_shootout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b2_tests.log 2>&1; tail -2 gpurun_out/b2_tests.log
timeout -k 10 200 python tools/pipeline_prof.py --reps 3 > gpurun_out/pipe.json 2>gpurun_out/pipe.err; cat gpurun_out/pipe.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pipeprof -o run -- python3 $R/tools/pipeline_prof.py --reps 2 > $R/gpurun_out/pipeprof.log 2>&1; echo prof rc=$?)
