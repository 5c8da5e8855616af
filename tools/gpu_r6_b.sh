# round 6: chain divergence probe + the GPU suite on the current library
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/chain_diff.py 120 > gpurun_out/r6_chain_diff.log 2>&1; echo "chain_diff rc $?"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not identical_input and not loop_revisit" > gpurun_out/r6_gputests.log 2>&1; echo "gpu tests rc $?"
