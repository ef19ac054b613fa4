set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for idx in ${C3_PASSES:-1 3}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${C3_TAG:-c3p}$idx/trace -o run -- python3 $R/tools/c3_pass.py $idx 3 > $R/gpurun_out/${C3_TAG:-c3p}$idx.log 2>&1
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" "FETCH_SIZE" "SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/${C3_TAG:-c3p}$idx/p$i -o pmc -- python3 $R/tools/c3_pass.py $idx 2 >> $R/gpurun_out/${C3_TAG:-c3p}$idx.log 2>&1
  done
done
echo done
