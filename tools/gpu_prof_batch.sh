# rocprof kernel stats of the cfg5 frame-parallel S2S leg alone (used via gpurun).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_batch -o run -- python3 bench.py --no-cpu --no-sharded --no-odom --no-gn --no-seg --steps 2 --warmup 1 --batch-frames ${FRAMES:-200} "$@" > gpurun_out/prof_batch.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_batch.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_batch/run_kernel_stats.csv")))
print("| kernel | calls | total ms | avg us | % |")
for r in rows[:40]:
    n = r["Name"].split("(")[0].replace("void ", "").split("::")[-1][:60]
    print(f"| {n} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | {float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
PY
