#!/bin/bash
# A/B conv_fwd XCD-aware N-tile order (librod.so) vs previous (librod_prev.so): outputs, timing, tests, bench
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
L=$PWD/road-object-detection-for-bdd100k_amd/lib
ROD_LIB=$L/librod_prev.so timeout -k 10 200 python tools/conv_bench.py --shapes 4,5,6,8 --ops fwd_plain,fwd_stats,bwd_data --out /tmp/g16_prev.pt > $O/g16_prev.log 2>&1 || exit 1
timeout -k 10 200 python tools/conv_bench.py --shapes 4,5,6,8 --ops fwd_plain,fwd_stats,bwd_data --check /tmp/g16_prev.pt > $O/g16_new.log 2>&1 || exit 1
grep -hv amdgpu $O/g16_prev.log $O/g16_new.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g16_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/g16_tests.log; exit 1; }
tail -1 $O/g16_tests.log
for v in librod_prev librod; do
ROD_LIB=$L/$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g16_$v.log 2>&1 || exit 1
echo $v $(grep -h '^{' $O/g16_$v.log | cut -c60-100)
done
