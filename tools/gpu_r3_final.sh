# Round-3 evidence on HEAD (used via gpurun): PMC traffic passes, the default
# bench (all legs, CPU baseline), the rocprofv3 kernel trace + stats of cfg 3.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
bash tools/gpu_r3_profiles.sh || exit 1
DDLO_TRAFFIC_JSON=gpurun_out/r03/traffic.json timeout -k 10 900 python -u bench.py > gpurun_out/r03/bench.json 2> gpurun_out/r03/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03/bench.err; exit 1; }
cat gpurun_out/r03/bench.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
