cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/nft -o run -- python3 tools/time_cov.py > gpurun_out/nft.log 2>&1 || { tail -5 gpurun_out/nft.log; exit 1; }
python3 tools/nf_trace.py gpurun_out/nft/run_kernel_trace.csv
