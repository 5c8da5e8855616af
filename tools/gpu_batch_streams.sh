# cfg5 frame-parallel S2S ms/pair vs streams per GPU (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ns in 2 3 4; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-sharded --no-odom --no-gn --no-seg --steps 2 --warmup 1 --batch-frames 300 --batch-streams $ns > gpurun_out/bs.json 2>/dev/null || { echo FAIL $ns; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bs.json').read().strip().splitlines()[-1]); print('streams', sys.argv[1], d['batched_s2s']['ms_per_pair'])" $ns
done
