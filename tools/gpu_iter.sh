# GPU tests + cfg3 timing + per-iteration kernel profile (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh "$@" || exit 1
timeout -k 10 120 python3 tools/time_cfg3.py || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pi3 -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 20 --warmup 3 > gpurun_out/pi3.log 2>&1 || { tail -20 gpurun_out/pi3.log; exit 1; }
python3 tools/profile_summary.py gpurun_out/pi3 run > gpurun_out/pi3.md
python3 - <<'PY'
t = open("gpurun_out/pi3.md").read()
print(t[:t.index("| k_align_init")])
print(t[t.index("## Active outer"):])
PY
