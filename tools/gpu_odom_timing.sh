cd $GRAFT_REPO_ROOT
DDLO_GRAPH_DEBUG=1 DDLO_ODOM_TIMING=1 timeout -k 10 300 python3 bench.py --no-cpu --no-sharded --no-gn --no-batch --steps 2 --warmup 1 > /tmp/ot.json 2> gpurun_out/ot.err; grep -E "odom timing|graphs" gpurun_out/ot.err | tail -12; python3 -c "import json; d=json.load(open('/tmp/ot.json')); print(d['odometry']['ms_per_frame'])"
