# rocprofv3 kernel-trace stats of a short driver run (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=${KSTATS_OUT:-gpurun_out/kstats}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 "$@" > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
python3 - "$out" <<'PY'
import csv, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f} min {float(r['MinNs'])/1e3:8.1f} max {float(r['MaxNs'])/1e3:9.1f} pct {float(r['Percentage']):5.1f}")
PY
