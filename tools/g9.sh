#!/bin/bash
# A/B: non-temporal BN-backward-apply stores (librod_nt.so) vs default
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
L=road-object-detection-for-bdd100k_amd/lib
timeout -k 10 200 python tools/bn_bench.py --out /tmp/bn_a.pt > $O/g9_bn_a.log 2>&1 || exit 1
ROD_LIB=$PWD/$L/librod_nt.so timeout -k 10 200 python tools/bn_bench.py --check /tmp/bn_a.pt > $O/g9_bn_nt.log 2>&1 || exit 1
grep -v amdgpu $O/g9_bn_a.log $O/g9_bn_nt.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g9_b_a.log 2>&1 || exit 1
ROD_LIB=$PWD/$L/librod_nt.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g9_b_nt.log 2>&1 || exit 1
grep -h '^{' $O/g9_b_a.log $O/g9_b_nt.log | cut -c1-200
