set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_iter -o run -- python3 $R/tools/iter_one.py 4000 > $R/gpurun_out/prof_iter.log 2>&1
