# Candidate-cell list bound (dev build, DDLO_GRID_LMAX) on the headline: ms/scan and the cells' build time
# and size, each setting twice, interleaved.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
L=$PWD/dynamic_direct_lidar_odometry_amd/_lib
for rep in 1 2; do
  for lm in 32 16 24 48; do
    DDLO_GICP_LIB=$L/dev/libddlo_gicp.so DDLO_GRID_LMAX=$lm timeout -k 10 240 python -u bench.py --no-cpu --no-sharded --no-batch --no-odom --no-seg --no-walk --no-gn --steps 100 > gpurun_out/ab/lmax$lm.json 2> gpurun_out/ab/lmax$lm.err || { echo "FAIL $lm"; tail gpurun_out/ab/lmax$lm.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/lmax$lm.json')); g=d['target_grid']; print('lmax $lm', d['ms_per_step'], round(g['build_ms'],1), round(g['bytes']/2**20), g['level_cells'], g['entries'])"
  done
done
