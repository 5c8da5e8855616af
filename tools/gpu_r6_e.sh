mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not identical_input and not loop_revisit" > gpurun_out/r6_gputests_e.log 2>&1; echo "gpu tests rc $?"
AB_CFG2=1 bash tools/gpu_ab.sh base head
timeout -k 10 600 python -u tools/slab_cells_table.py 2 4 8 > gpurun_out/r6_slab_cells.log 2>&1; echo "slab cells rc $?"
