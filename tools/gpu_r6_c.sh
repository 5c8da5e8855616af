mkdir -p gpurun_out
timeout -k 10 200 python -u tools/chain_inputs.py 4 > gpurun_out/r6_chain_inputs.log 2>&1; echo "chain_inputs rc $?"
bash tools/gpu_r6_churn.sh > gpurun_out/r6_churn.log 2>&1; echo "churn rc $?"
