cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  DDLO_FUSE_LM=$v timeout -k 10 120 python -u tools/grid_probe.py --aligns 300 2>&1 | grep "^grid" | python3 -c "import sys,json; l=sys.stdin.read(); d=json.loads(l[l.index('{'):]); print('FUSE_LM=$v', round(d['ms_per_scan'],4), 'dev', round(d['device_ms_median'],4), 'lin', round(d['linearize_us_per_iter'],2))" || exit 1
done
