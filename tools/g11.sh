#!/bin/bash
# gpu tests + wgrad shapes (XCD-aware tile order) + bench
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g11_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/g11_tests.log; exit 1; }
tail -1 $O/g11_tests.log
timeout -k 10 200 python tools/conv_bench.py --ops wgrad > $O/g11_wgrad.log 2>&1 || exit 1
grep -v amdgpu $O/g11_wgrad.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference > $O/g11_bench.log 2>&1 || exit 1
grep -h '^{' $O/g11_bench.log | cut -c1-120
