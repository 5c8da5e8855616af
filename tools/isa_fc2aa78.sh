# Reproduce the ISA evidence for the fc2aa78 fault (profiles/r04_fc2aa78_isa.md):
# compile the PRE-fix nftree.hip (fc2aa78^) for gfx950 and print the
# coordinate-load loop of k_nf_small (small_tree's lim1/lim2 count over Q[i]).
set -e
d=$(mktemp -d)
git archive fc2aa78^ dynamic_direct_lidar_odometry_amd/csrc include | tar -x -C $d
( cd $d/dynamic_direct_lidar_odometry_amd/csrc && /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 \
    -ffp-contract=off --cuda-device-only -S -o $d/pre.s nftree.hip )
a=$(grep -n "^.LBB3_19:" $d/pre.s | cut -d: -f1)
b=$(grep -n "^.LBB3_33:" $d/pre.s | cut -d: -f1)
sed -n "${a},$((b-1))p" $d/pre.s
rm -rf $d
