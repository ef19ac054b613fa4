#!/bin/bash
# round 6: pipeline profile, prefix A/B, run-engine bench (one GPU call)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_replace_class.py tests/test_gpu_long.py tests/test_gpu_prefix*.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b1_tests.log 2>&1; tail -3 gpurun_out/b1_tests.log
timeout -k 10 200 python tools/pipeline_prof.py --reps 3 > gpurun_out/pipe.json 2>gpurun_out/pipe.err; cat gpurun_out/pipe.json
timeout -k 10 300 python tools/prefix_ab.py > gpurun_out/prefix_ab.jsonl 2>gpurun_out/prefix_ab.err; echo prefix rc=$?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pipeprof -o run -- python3 $R/tools/pipeline_prof.py --reps 2 > $R/gpurun_out/pipeprof.log 2>&1; echo prof rc=$?)
