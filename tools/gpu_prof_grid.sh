# kernel trace of the cfg3 probe (cells on and off) -> gpurun_out/prof_grid/run_kernel_{trace,stats}.csv
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -rf gpurun_out/prof_grid
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_grid -o run -- python3 tools/grid_probe.py --aligns 30 > gpurun_out/prof_grid.log 2>&1; echo prof rc $?
