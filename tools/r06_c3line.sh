#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r06_lines
timeout -k 10 300 python bench.py --config c3 > gpurun_out/r06_lines/c3.json 2> gpurun_out/r06_lines/c3.err; echo "c3 rc=$?"
timeout -k 10 200 python tools/pipeline_prof.py --reps 3 > gpurun_out/pipe.json 2>gpurun_out/pipe.err; cat gpurun_out/pipe.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pipeprof -o run -- python3 $R/tools/pipeline_prof.py --reps 2 > $R/gpurun_out/pipeprof.log 2>&1; echo prof rc=$?)
