#!/bin/bash
# gpu tests + bench + short kernel trace
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g13_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/g13_tests.log; exit 1; }
tail -1 $O/g13_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g13_bench.log 2>&1 || exit 1
grep -h '^{' $O/g13_bench.log | cut -c1-120
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_g13 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g13_prof.log 2>&1 || exit 1
echo done
