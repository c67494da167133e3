#!/bin/bash
# depthwise A/B on the GPU box: old library (lib/librod_old.so) vs the current build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; T=${1:-dwx}; OPS=${2:-fwd,fwdpro,bwd_data,bwd_filter}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_gred.py -q -x -k "depthwise or dw_" --timeout=200 -p no:cacheprovider > $O/${T}_tests.log 2>&1; rc=$?
tail -2 $O/${T}_tests.log; [ $rc -gt 1 ] && exit $rc
ROD_LIB=$PWD/road-object-detection-for-bdd100k_amd/lib/librod_old.so timeout -k 10 300 python tools/dw_bench.py --ops $OPS --out /tmp/ref.pt > $O/${T}_old.log 2>&1 || exit $?
timeout -k 10 300 python tools/dw_bench.py --ops $OPS --check /tmp/ref.pt > $O/${T}_new.log 2>&1 || exit $?
paste <(grep -v "CHECK\|amdgpu\|TOTAL" $O/${T}_old.log | awk '{print $1, $2}') <(grep -v "CHECK\|amdgpu\|TOTAL" $O/${T}_new.log | awk '{print $2, $4}')
grep TOTAL $O/${T}_old.log $O/${T}_new.log
grep CHECK $O/${T}_new.log | awk '{print $2, $6, $7, $8}'
