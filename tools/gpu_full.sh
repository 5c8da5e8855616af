# full GPU suite + default bench (all legs) -> gpurun_out/full_tests.log, gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/full_tests.log 2>&1; rc=$?
tail -4 gpurun_out/full_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" gpurun_out/full_tests.log | head -20; exit 1; }
timeout -k 10 1200 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print({k: d[k] for k in ('value','ms_per_step')}, d['cpu_baseline']['value'], d['cpu_baseline']['speedup_gpu_vs_cpu']); [print(k, json.dumps(d[k])[:400]) for k in ('target_grid','cfg3_walk','cfg3_varied_guesses','s2s_gn','sharded_s2m','batched_s2s','odometry') if k in d]"
