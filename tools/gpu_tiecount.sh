# tied-query counts per scan of the cfg5 frames (k=10 covariances; used via gpurun)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tiecount
DDLO_TIE_DEBUG=1 timeout -k 10 300 python3 -u tools/batch_prof.py 1 > gpurun_out/tiecount/o.txt 2> gpurun_out/tiecount/ties.txt || { tail -20 gpurun_out/tiecount/ties.txt; exit 1; }
python3 - <<'PY'
import re
v = [int(m.group(1)) for m in re.finditer(r"tied (\d+)", open("gpurun_out/tiecount/ties.txt").read())]
v.sort()
print(len(v), "scans; zero", sum(x == 0 for x in v), "p50", v[len(v)//2], "p75", v[3*len(v)//4], "p90", v[9*len(v)//10], "max", v[-1], "sum", sum(v))
print("over 64:", sum(x > 64 for x in v), "over 128:", sum(x > 128 for x in v))
PY
