#!/bin/bash
# gpu tests (default lib) + A/B bench: non-temporal output stores in depthwise/GEMM (librod_ntout.so)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
L=$PWD/road-object-detection-for-bdd100k_amd/lib
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g10_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/g10_tests.log; exit 1; }
tail -1 $O/g10_tests.log
for i in 1 2; do
for v in librod librod_ntout; do
ROD_LIB=$L/$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g10_$v.$i.log 2>&1 || exit 1
echo $v $(grep -h '^{' $O/g10_$v.$i.log | cut -c60-140)
done
done
