# rocprof kernel stats of the cfg5 legs (batch + odometry) on 200 frames, plus a plain bench of both (used via gpurun).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 5 --warmup 2 --batch-frames ${FRAMES:-200} > gpurun_out/legs.json 2> gpurun_out/legs.err || { echo BENCH_FAIL; tail -20 gpurun_out/legs.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/legs.json").read().strip().splitlines()[-1])
print("cfg3 ms", d["ms_per_step"], "| batch ms/pair", d["batched_s2s"]["ms_per_pair"], "| odom ms/frame", d["odometry"]["ms_per_frame"], d["odometry"]["rank0"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_legs -o run -- python3 bench.py --no-cpu --no-sharded --no-gn --no-seg --no-batch --steps 2 --warmup 1 --batch-frames ${FRAMES:-200} > gpurun_out/prof_legs.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_legs.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_legs/run_kernel_stats.csv")))
print("| kernel (odometry leg) | calls | total ms | avg us | % |")
for r in rows[:30]:
    n = r["Name"].split("(")[0].replace("void ", "").split("::")[-1][:60]
    print(f"| {n} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | {float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
PY
