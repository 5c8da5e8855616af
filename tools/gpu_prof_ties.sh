# per-kernel A/B of the correspondence tie detection on cfg3 (DDLO_TIE_EXACT=1/0), used via gpurun
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 1 0; do
  DDLO_TIE_EXACT=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pt$m -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 50 --warmup 5 > gpurun_out/pt$m.log 2>&1 || { tail -20 gpurun_out/pt$m.log; exit 1; }
  python3 tools/profile_summary.py gpurun_out/pt$m run > gpurun_out/pt$m.md
done
