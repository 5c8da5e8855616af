# SQ instruction / cycle passes over the cfg3 aligns (tools/legs.py cfg3: graph aligns only), one
# rocprofv3 --pmc run each (never combined with tracing); prints per-kernel
# averages of the search / moment / LM kernels and removes the raw passes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  tag=$(echo $set | cut -d" " -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$tag -o run -- python3 tools/legs.py cfg3 20 > gpurun_out/pmc_$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 gpurun_out/pmc_$tag.log; exit 1; }
done
python3 tools/pmc_kernels.py gpurun_out/pmc_SQ_WAVES gpurun_out/pmc_SQ_WAVE_CYCLES > gpurun_out/pmc_sq.txt
rm -rf gpurun_out/pmc_SQ_WAVES gpurun_out/pmc_SQ_WAVE_CYCLES
python3 - <<'PY'
import re
out=[]; keep=False
for l in open('gpurun_out/pmc_sq.txt'):
    if not l.startswith(' '):
        keep = any(k in l for k in ('k_cell_lookup', 'k_nn_seed', 'k_nn_scan', 'k_moments', 'k_lm_step', 'k_align_init'))
    if keep: out.append(l.rstrip())
print('\n'.join(out))
PY
