#!/bin/bash
# gpu tests + conv_bench fwd (statistics epilogue rounding once) + bench
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g14_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/g14_tests.log; exit 1; }
tail -1 $O/g14_tests.log
timeout -k 10 200 python tools/conv_bench.py --ops fwd_plain,fwd_stats > $O/g14_fwd.log 2>&1 || exit 1
grep -v amdgpu $O/g14_fwd.log | grep -E "TOTAL|fwd_stats"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g14_bench.log 2>&1 || exit 1
grep -h '^{' $O/g14_bench.log | cut -c1-120
