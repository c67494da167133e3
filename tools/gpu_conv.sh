#!/bin/bash
# conv A/B on the GPU box: old library (lib/librod_old.so) vs the current build, then tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; T=${1:-cv}
ROD_LIB=$PWD/road-object-detection-for-bdd100k_amd/lib/librod_old.so timeout -k 10 300 python tools/conv_bench.py --out /tmp/ref.pt > $O/${T}_old.log 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --check /tmp/ref.pt > $O/${T}_new.log 2>&1 || exit $?
paste <(grep -v "CHECK\|amdgpu" $O/${T}_old.log | awk '{print $1, $2}') <(grep -v "CHECK\|amdgpu" $O/${T}_new.log | awk '{print $2, $4, $6}')
grep CHECK $O/${T}_new.log | awk '{print $2, $3, $4, $5}'
