#!/bin/bash
# pw_bwd micro-benchmark: baseline library vs the working tree, block-count sweep.
# usage: tools/gpu_pw.sh <tag> [nblk...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; shift
L=road-object-detection-for-bdd100k_amd/lib
if [ -f $L/librod_base.so ]; then
  ROD_LIB=$L/librod_base.so timeout -k 10 300 python tools/pwbwd_bench.py --pw-only > gpurun_out/pw_${T}_base.log 2>&1 || exit $?
  tail -1 gpurun_out/pw_${T}_base.log
fi
for n in "${@:-1024}"; do
  ROD_PW_NBLK=$n timeout -k 10 300 python tools/pwbwd_bench.py --pw-only > gpurun_out/pw_${T}_$n.log 2>&1 || exit $?
  echo "nblk=$n"; tail -1 gpurun_out/pw_${T}_$n.log
done
if [ -n "$PW_FULL" ]; then
  ROD_PW_NBLK=${PW_FULL} timeout -k 10 300 python tools/pwbwd_bench.py > gpurun_out/pw_${T}_full.log 2>&1 || exit $?
  cat gpurun_out/pw_${T}_full.log
fi
