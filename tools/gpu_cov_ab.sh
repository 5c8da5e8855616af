# sliced covariance kernel: GPU tests, then batch / odometry legs A/B (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
B="--no-cpu --no-sharded --no-gn --steps 5 --warmup 2"
for cfg in "DDLO_COV_TASKS=0" "DDLO_COV_TASKS=1"; do
  env $cfg timeout -k 10 300 python3 bench.py $B > gpurun_out/cab.json 2> gpurun_out/cab.err || { echo "FAIL $cfg"; tail -20 gpurun_out/cab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cab.json')); print('$cfg', 'batch ms/pair', d['batched_s2s']['ms_per_pair'], 'odom ms/frame', d['odometry']['ms_per_frame'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cov -o run -- python3 bench.py --no-cpu --no-sharded --no-gn --no-odom --steps 3 --warmup 1 > gpurun_out/cov.log 2>&1 || { tail -20 gpurun_out/cov.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/cov/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "knn" in r["Name"] or "k_covariances" in r["Name"]:
        print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
