# td fix check (used via gpurun): the split-group tie tests on the pre-fix library (expected to fail) and on
# HEAD, the tie classification, then the tie / tree / knn GPU tests.
cd $GRAFT_REPO_ROOT
O=gpurun_out/tdfix
mkdir -p $O
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
DDLO_GICP_LIB=$PWD/dynamic_direct_lidar_odometry_amd/_lib/old/libddlo_gicp.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_nftree.py -k "split_groups or ties_lattice" > $O/old.log 2>&1
echo "old lib exit $?"
timeout -k 10 300 $T tests/test_gpu_nftree.py -k "split_groups or ties_lattice" > $O/new.log 2>&1 || { echo NEW_FAIL; tail -30 $O/new.log; exit 1; }
timeout -k 10 300 python -u tools/tie_classify.py 4 > $O/classify.log 2>&1 || { echo CLASSIFY_FAIL; tail -20 $O/classify.log; exit 1; }
timeout -k 10 900 $T tests/test_gpu_nftree.py tests/test_gpu_ties.py tests/test_gpu_knn.py tests/test_gpu_gicp.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo ALL_OK
