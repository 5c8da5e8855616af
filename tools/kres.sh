# kernel resource usage (VGPR/SGPR/spill/scratch/LDS) of a code object or a host object with an embedded fatbin
# usage: bash tools/kres.sh <file.o|file.co> [name-regex]
f=$1; pat=${2:-.}
d=$(mktemp -d)
if /opt/rocm/lib/llvm/bin/llvm-objdump -h "$f" | grep -q hip_fatbin; then
  /opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$d/fb.bin "$f"
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$d/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/k.co
  f=$d/k.co
fi
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$f" > $d/notes.txt
python3 - "$d/notes.txt" "$pat" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
for blk in t.split('- .agpr_count')[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk).group(1)
    if not re.search(sys.argv[2], name): continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\S+)', blk) or [None, None])[1]
    print(f"{name[:60]:60s} vgpr {g('vgpr_count')} sgpr {g('sgpr_count')} spill {g('vgpr_spill_count')} scratch {g('private_segment_fixed_size')} lds {g('group_segment_fixed_size')}")
PY
rm -rf $d
