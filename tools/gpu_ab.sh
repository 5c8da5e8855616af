# A/B of search knobs (used via gpurun): each line "ENV=.. ENV2=.." runs a short bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
while read -r line; do
  [ -z "$line" ] && continue
  env $line timeout -k 10 120 python -u bench.py --no-cpu --no-sharded --no-batch --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "AB_FAIL $line"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], 'ms/scan', d['ms_per_step'], 'lin us', d['roofline']['avg_launch_us'], 'cfg2 ms', d.get('s2s_gn', {}).get('ms_per_align'))" "$line"
done < "${1:-tools/ab_cases.txt}"
