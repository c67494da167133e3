#!/bin/bash
# depthwise A/B on the GPU box: parity tests, then legacy vs LDS-exchange micro-benchmark
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; T=${1:-dw}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k "depthwise or dw_" --timeout=200 -p no:cacheprovider > $O/${T}_tests.log 2>&1; rc=$?
tail -3 $O/${T}_tests.log; [ $rc -gt 1 ] && exit $rc
ROD_DW_LEGACY=1 timeout -k 10 300 python tools/dw_bench.py --out /tmp/ref.pt > $O/${T}_legacy.log 2>&1 || exit $?
cat $O/${T}_legacy.log | grep TOTAL
timeout -k 10 300 python tools/dw_bench.py --check /tmp/ref.pt > $O/${T}_new.log 2>&1 || exit $?
cat $O/${T}_new.log
