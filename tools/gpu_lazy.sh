# lazy tie search check (used via gpurun): parity tests, covariance timing and the cfg 5 legs, lazy vs whole tree.
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_nftree.py > $O/nftree.log 2>&1 || { echo NFTREE_FAIL; tail -30 $O/nftree.log; exit 1; }
DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=5 timeout -k 10 120 python -u tools/tie_classify.py 3 > $O/classify.log 2>&1 || { echo CLASSIFY_FAIL; tail -20 $O/classify.log; exit 1; }
DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=5 timeout -k 10 120 python -u tools/time_cov.py > $O/time_cov_lazy.log 2>&1 || { echo TIMECOV_FAIL; tail -20 $O/time_cov_lazy.log; exit 1; }
timeout -k 10 120 python -u tools/time_cov.py > $O/time_cov_tree.log 2>&1 || { echo TIMECOV0_FAIL; exit 1; }
cat $O/time_cov_lazy.log $O/time_cov_tree.log
DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=5 timeout -k 10 900 $T tests/test_gpu_ties.py tests/test_gpu_knn.py tests/test_gpu_gicp.py tests/test_gpu_batch.py tests/test_gpu_odom.py tests/test_gpu_odom_long.py > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
DDLO_TIE_LAZY=1 DDLO_TIE_PARTIAL_LEVELS=5 timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 50 > $O/bench_lazy.json 2> $O/bench_lazy.err || { echo BENCH_FAIL; tail -20 $O/bench_lazy.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded --no-gn --no-seg --steps 50 > $O/bench_tree.json 2> $O/bench_tree.err || { echo BENCH0_FAIL; tail -20 $O/bench_tree.err; exit 1; }
python - <<'PY'
import json
for tag in ("lazy", "tree"):
    d = json.load(open(f"gpurun_out/lazy/bench_{tag}.json"))
    b, o = d.get("batched_s2s", {}), d.get("odometry", {})
    print(tag, "cfg3", d["ms_per_step"], "batched", {k: v for k, v in b.items() if "ms" in k}, "odom", {k: v for k, v in o.items() if "ms" in k})
PY
echo ALL_OK
