# A/B of alternative in-tree builds of libddlo_gicp.so (DDLO_GICP_LIB) on the headline leg (cfg3) and,
# with AB_CFG2=1, the cfg2 leg; each variant twice, interleaved.  Usage: bash tools/gpu_ab.sh base ab16 ab32
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
for rep in 1 2; do
  for v in "$@"; do
    lib=$L/libddlo_gicp.so; [ $v != base ] && lib=$L/$v/libddlo_gicp.so
    DDLO_GICP_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-seg --no-walk $([ "$AB_CFG2" = 1 ] || echo --no-gn) --steps 100 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { echo "FAIL $v"; tail gpurun_out/ab/$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.json')); g=d.get('s2s_gn') or {}; print('$v', d['ms_per_step'], g.get('ms_per_align'))"
  done
done
