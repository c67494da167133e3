#!/bin/bash
# stem kernels: gpu tests + conv_bench A/B (generic vs dedicated stem wgrad)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g7_tests.log 2>&1 || { echo TESTS FAILED rc=$?; tail -30 $O/g7_tests.log; exit 1; }
tail -2 $O/g7_tests.log
ROD_DEBUG_OLDSTEMFWD=1 ROD_DEBUG_OLDSTEMWG=1 timeout -k 10 120 python tools/conv_bench.py --shapes 9 --ops fwd_plain,fwd_stats,wgrad --out /tmp/g7_old.pt > $O/g7_old.log 2>&1 || exit 1
timeout -k 10 120 python tools/conv_bench.py --shapes 9 --ops fwd_plain,fwd_stats,wgrad --check /tmp/g7_old.pt > $O/g7_new.log 2>&1 || exit 1
cat $O/g7_old.log $O/g7_new.log
