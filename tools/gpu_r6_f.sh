mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "not loop_revisit" > gpurun_out/r6_gputests_f.log 2>&1; echo "gpu tests rc $?"
bash tools/gpu_ab.sh base head
