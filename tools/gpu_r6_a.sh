mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_process.py > gpurun_out/r6_process.log 2>&1; echo "process rc $?"; (DDLO_TORCH_FIRST=0 timeout -k 10 120 python -c "
import dynamic_direct_lidar_odometry_amd as P
L = P.load()
import torch, torch.distributed
u = P.comm_unique_id()
print(\"reverse-order ok\", len(u))
" > gpurun_out/r6_reverse.log 2>&1; echo "reverse rc $?" >> gpurun_out/r6_reverse.log); timeout -k 10 700 python -u -m pytest -x -v -s --timeout 680 --timeout-method thread tests/test_gpu_odom_long.py -k identical > gpurun_out/r6_identical.log 2>&1; echo "identical rc $?"
