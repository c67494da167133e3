#!/bin/bash
# gpu tests, stem A/B, conv wgrad shapes, full bench
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g8_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/g8_tests.log; exit 1; }
tail -2 $O/g8_tests.log
ROD_DEBUG_OLDSTEMFWD=1 ROD_DEBUG_OLDSTEMWG=1 timeout -k 10 120 python tools/conv_bench.py --shapes 9 --ops fwd_plain,fwd_stats,wgrad --out /tmp/g8_old.pt > $O/g8_old.log 2>&1 || exit 1
timeout -k 10 120 python tools/conv_bench.py --shapes 9 --ops fwd_plain,fwd_stats,wgrad --check /tmp/g8_old.pt > $O/g8_new.log 2>&1 || exit 1
grep -v amdgpu $O/g8_old.log $O/g8_new.log
timeout -k 10 200 python tools/conv_bench.py --ops wgrad > $O/g8_wgrad.log 2>&1 || exit 1
grep -v amdgpu $O/g8_wgrad.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/g8_bench.log 2>&1 || exit 1
grep '^{' $O/g8_bench.log | cut -c1-400
