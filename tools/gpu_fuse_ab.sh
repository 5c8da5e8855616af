# The LM step fused into the moment kernel's last block (dev build, DDLO_FUSE_LM=1) against the product
# library and the dev build without it, on the headline (cfg3) and cfg2 legs; twice, interleaved.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
run() {   # name lib fuse
  DDLO_GICP_LIB=$2 DDLO_FUSE_LM=$3 timeout -k 10 240 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-seg --no-walk --steps 100 > gpurun_out/ab/$1.json 2> gpurun_out/ab/$1.err || { echo "FAIL $1"; tail gpurun_out/ab/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$1.json')); print('$1', d['ms_per_step'], d['s2s_gn']['ms_per_align'])"
}
for rep in 1 2; do
  run base $L/libddlo_gicp.so 0 || exit 1
  run dev $L/dev/libddlo_gicp.so 0 || exit 1
  run fuse $L/dev/libddlo_gicp.so 1 || exit 1
done
