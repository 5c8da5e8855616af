# covariance kernel times per variant (used via gpurun): kernel trace of the cfg5 batch leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "DDLO_COV_2LANE=0" "DDLO_COV_2LANE=1" "DDLO_COV_2LANE=1 DDLO_COV_OCC=4"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$tag -o run -- python3 bench.py --no-cpu --no-sharded --no-gn --no-seg --no-odom --steps 3 > gpurun_out/kt_$tag.log 2>&1 || { echo "KT_FAIL $v"; tail -5 gpurun_out/kt_$tag.log; exit 1; }
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/kt_$tag/run_kernel_stats.csv')):
    if 'covariances' in r['Name']: print(sys.argv[1], r['Name'][:50], 'calls', r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3,1))
" "$v"
  rm -rf gpurun_out/kt_$tag
done
