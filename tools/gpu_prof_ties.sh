# per-kernel A/B of the correspondence tie test on cfg3, used via gpurun:
# ptN = DDLO_TIE_SCAN=N (1 full second distance, 2 slice bests, 3 merge flags + mirrored key), pt0 = Morton order
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 3 2 0; do
  if [ $m = 0 ]; then export DDLO_TIE_EXACT=0 DDLO_TIE_SCAN=3; else export DDLO_TIE_EXACT=1 DDLO_TIE_SCAN=$m; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pt$m -o run -- python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 100 --warmup 5 > gpurun_out/pt$m.log 2>&1 || { tail -20 gpurun_out/pt$m.log; exit 1; }
  python3 tools/profile_summary.py gpurun_out/pt$m run > gpurun_out/pt$m.md
done
unset DDLO_TIE_EXACT
for m in 3; do
  DDLO_TIE_SCAN=$m timeout -k 10 200 python3 tools/ab_ties.py > gpurun_out/ab_ties$m.log 2>&1 || exit 1
done
