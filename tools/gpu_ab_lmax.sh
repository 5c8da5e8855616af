cd $GRAFT_REPO_ROOT
for v in 16 24 32 16 24 32; do
  DDLO_GRID_LMAX=$v timeout -k 10 120 python -u tools/grid_probe.py --aligns 300 2>&1 | grep "^grid" | python3 -c "import sys,json; l=sys.stdin.read(); d=json.loads(l[l.index('{'):]); g=d['grid']; print('LMAX=$v', round(d['ms_per_scan'],4), 'dev', round(d['device_ms_median'],4), 'lin', round(d['linearize_us_per_iter'],2), 'build', round(g['build_ms'],1), 'MB', g['bytes']>>20, 'levels', g['level_cells'])" || exit 1
done
