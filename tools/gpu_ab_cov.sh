# A/B of covariance knobs on the cfg5 legs (used via gpurun): each line "ENV=.." runs the batch + odometry legs.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
while read -r line; do
  [ -z "$line" ] && continue
  env $line timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 5 > gpurun_out/abc.json 2> gpurun_out/abc.err || { echo "AB_FAIL $line"; tail -5 gpurun_out/abc.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/abc.json')); print(sys.argv[1], 'batch ms/pair', d['batched_s2s']['ms_per_pair'], 'odom ms/frame', d['odometry']['ms_per_frame'])" "$line"
done < "$1"
