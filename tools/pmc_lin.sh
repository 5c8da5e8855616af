# SQ counter passes over the linearize-dominated driver (tools/bench_lin.py),
# one rocprofv3 --pmc run per pass (never combined with tracing domains).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$tag -o run -- python3 tools/bench_lin.py 2 > gpurun_out/pmc_$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 gpurun_out/pmc_$tag.log; exit 1; }
done
echo pmc done
