# cfg3 ms/scan under search knobs (used via gpurun): each argument is one env assignment list "A=1,B=2"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "$@"; do
  envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 120 python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 40 --warmup 5 > gpurun_out/sw.json 2>/dev/null || { echo "FAIL $cfg"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], d['roofline']['avg_launch_us'], d['cfg3_varied_guesses']['ms_per_scan'])" "$cfg"
done
