# Kernel trace of the odometry chain (cfg 5, 300 frames, candidate cells off): per-kernel totals per frame,
# device busy time against the wall time.  Summary only (the trace is deleted).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/odom_prof
mkdir -p $O
rm -rf $O/tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/odom_probe.py --frames 300 --modes 0 > $O/probe.log 2>&1 || { echo PROF_FAIL; tail $O/probe.log; exit 1; }
grep "ms/frame" $O/probe.log
python3 - <<'PY'
import csv
d='gpurun_out/odom_prof/tr'
st=list(csv.DictReader(open(f'{d}/run_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in st)
print(f"kernel time total {tot/1e6:.1f} ms over 304 frames (4 warm-up + 300): {tot/1e3/304:.1f} us/frame")
for r in st[:25]:
    print(f"{r['Name'].split('(')[0].replace('void ','')[:60]:60s} calls {r['Calls']:>6} avg {float(r['AverageNs'])/1e3:7.1f} us  per frame {float(r['TotalDurationNs'])/1e3/304:7.1f} us  {float(r['Percentage']):5.1f}%")
PY
rm -rf $O/tr
