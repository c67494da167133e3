#!/bin/bash
# BN-backward micro-benchmark + kernel trace.  usage: tools/gpu_bn.sh <tag> [check-file]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1
CHK=${2:+--check $2}
timeout -k 10 300 python tools/bn_bench.py $CHK > gpurun_out/bn_$T.log 2>&1 || exit $?
cat gpurun_out/bn_$T.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bnprof_$T -o run --output-format csv -- python3 tools/bn_bench.py --iters 5 > /dev/null 2>&1 || exit $?
echo done
