cd $GRAFT_REPO_ROOT
DDLO_COV_DEBUG=1 timeout -k 10 200 python3 bench.py --no-cpu --no-sharded --no-gn --no-odom --steps 2 --warmup 1 --batch-frames 12 > /tmp/pc.json 2> gpurun_out/pc.err; grep "\[cov\]" gpurun_out/pc.err | head -12
