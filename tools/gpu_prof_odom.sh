# kernel trace of the odometry-driver leg (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/po -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-gn --steps 3 --warmup 1 > gpurun_out/po.log 2>&1 || { tail -20 gpurun_out/po.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
d = json.load(open(glob.glob('gpurun_out/po.log')[0].replace('po.log','po.log'))) if False else None
f = glob.glob('gpurun_out/po/**/run_kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:30]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>6s} total {float(r['TotalDurationNs'])/1e6:8.2f} ms avg {float(r['AverageNs'])/1e3:8.2f} us")
print("kernel total ms", tot / 1e6)
for g in glob.glob('gpurun_out/po/**/run_memory_copy_stats.csv', recursive=True):
    for r in csv.DictReader(open(g)):
        print("copy", r.get('Name'), r.get('Calls'), float(r['TotalDurationNs'])/1e6, "ms")
PY
tail -1 gpurun_out/po.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['odometry'])"
