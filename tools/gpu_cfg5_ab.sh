# cfg5 batch / odometry legs under env knobs (used via gpurun): each argument is one env assignment list "A=1,B=2"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "$@"; do
  envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 5 --warmup 2 > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo "FAIL $cfg"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
b=d.get('batched_s2s',{}); o=d.get('odometry',{})
print(sys.argv[1], 'cfg3', d['ms_per_step'], 'batch', {k:v for k,v in b.items() if 'ms' in k}, 'odom', {k:v for k,v in o.items() if 'ms' in k})" "$cfg"
done
