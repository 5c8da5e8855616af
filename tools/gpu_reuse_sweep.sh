# cfg3 ms/scan under verified-reuse recording knobs (used via gpurun)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 120 python3 bench.py --no-cpu --no-sharded --no-batch --no-odom --no-gn --no-seg --steps 40 --warmup 5 > gpurun_out/sw.json 2>/dev/null || { echo "FAIL $*"; return 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1])
print(sys.argv[1:], d['ms_per_step'], d['roofline']['avg_launch_us'], d['cfg3_varied_guesses']['ms_per_scan'])" "$@"
}
run DDLO_X=0 && run DDLO_REUSE_REC_EPS=0.3 && run DDLO_REUSE_REC_EPS=0.3 DDLO_REUSE_GAP=0.02 && run DDLO_REUSE_REC_EPS=1.0 DDLO_REUSE_GAP=0.02 && run DDLO_REUSE_REC_EPS=1.0 DDLO_REUSE_GAP=0.01 && run DDLO_REUSE_REC0=1 DDLO_REUSE_GAP0=0.02 DDLO_REUSE_REC_EPS=1.0 DDLO_REUSE_GAP=0.02 && run DDLO_X=0
