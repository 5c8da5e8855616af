# cfg4 leg with its oracle timing (used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg4cpu
timeout -k 10 600 python -u bench.py --no-batch --no-odom --no-gn --no-seg --steps 20 > gpurun_out/cfg4cpu/bench.json 2> gpurun_out/cfg4cpu/bench.err || { tail -20 gpurun_out/cfg4cpu/bench.err; exit 1; }
python -c "import json; d = json.load(open('gpurun_out/cfg4cpu/bench.json')); print(d['sharded_s2m']); print(d['cpu_baseline']['ms_by_threads'])"
