# verified-reuse A/B: GPU tests, then cfg3 / cfg2 legs per knob setting (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
fi
B="--no-cpu --no-sharded --no-batch --no-odom --steps ${STEPS:-100} --warmup 5 --gn-steps 10"
for cfg in "DDLO_REUSE=0" "DDLO_REUSE=1" ${EXTRA_CFGS}; do
  env $cfg timeout -k 10 200 python3 bench.py $B > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "FAIL $cfg"; tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$cfg', 'cfg3', d['ms_per_step'], 'lin', d['roofline']['avg_launch_us'], 'cfg2', d['s2s_gn']['ms_per_align'], d['s2s_gn']['iters_per_s'])"
done
