# Quick GPU check (used via gpurun): parity tests of the align path, then a short bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_quick.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 200 python -u bench.py --no-cpu --no-sharded --batch-frames 41 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_quick.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print('ms/scan', d['ms_per_step'], 'iters/s', d['value'], 'lin us', d['roofline']['avg_launch_us'], 'batch', d.get('batched_s2s'))"
timeout -k 10 200 python -u tools/probe_cfg3.py > gpurun_out/probe.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
