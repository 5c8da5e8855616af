# batched-S2S leg: A/B of the search variants + kernel trace (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--no-cpu --no-sharded --no-gn --no-odom --steps 5 --warmup 2"
timeout -k 10 200 python3 bench.py --no-cpu --no-sharded --no-gn --steps 5 --warmup 2 > gpurun_out/bo.json 2> gpurun_out/bo.err || { tail -20 gpurun_out/bo.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bo.json')); print(d['batched_s2s']['ms_per_pair'], d['odometry'])"
timeout -k 10 200 python3 bench.py $B > gpurun_out/bb_tasks.json 2> gpurun_out/bb_tasks.err || { tail -20 gpurun_out/bb_tasks.err; exit 1; }
DDLO_SEARCH=collect timeout -k 10 200 python3 bench.py $B > gpurun_out/bb_collect.json 2> gpurun_out/bb_collect.err || { tail -20 gpurun_out/bb_collect.err; exit 1; }
timeout -k 10 200 python3 bench.py $B --batch-streams 1 > gpurun_out/bb_s1.json 2> gpurun_out/bb_s1.err || { tail -20 gpurun_out/bb_s1.err; exit 1; }
for f in bb_tasks bb_collect bb_s1; do python3 -c "import json,sys; d=json.load(open('gpurun_out/$f.json')); print('$f', d['ms_per_step'], d['batched_s2s']['ms_per_pair'])"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bkt -o run -- python3 bench.py $B > gpurun_out/bkt.log 2>&1 || { tail -20 gpurun_out/bkt.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/bkt/**/run_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:25]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} total {float(r['TotalDurationNs'])/1e6:9.2f} ms avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
