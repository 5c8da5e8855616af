# kernel trace of the cfg3 / cfg2 legs, per-iteration summary (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pi3 -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --steps 20 --warmup 3 > gpurun_out/pi3.log 2>&1 || { tail -20 gpurun_out/pi3.log; exit 1; }
python3 tools/profile_summary.py gpurun_out/pi3 run > gpurun_out/pi3.md
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pi2 -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --steps 2 --warmup 1 --gn-steps 5 > gpurun_out/pi2.log 2>&1 || { tail -20 gpurun_out/pi2.log; exit 1; }
python3 tools/profile_summary.py gpurun_out/pi2 run > gpurun_out/pi2.md
python3 - <<'PY'
for f in ("gpurun_out/pi3.md", "gpurun_out/pi2.md"):
    t = open(f).read()
    print(t[t.index("## Active outer"):])
PY
