# odometry-driver parity A/B against an alternative build (used via gpurun)
cd $GRAFT_REPO_ROOT
T="tests/test_gpu_odom.py::test_driver_vs_oracle"
for cfg in "DDLO_REUSE=0" "DDLO_REUSE=1"; do
  env $cfg timeout -k 10 120 python -m pytest $T -x -q --timeout 100 > /tmp/b.log 2>&1; echo "$cfg -> rc $? $(tail -1 /tmp/b.log)"
done
