cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-g3}
timeout -k 10 300 python -m pytest tests/test_gpu_gred.py -q -x --timeout=200 -p no:cacheprovider > gpurun_out/${T}_gred.log 2>&1; rc=$?; echo "gred tests rc=$rc"; tail -3 gpurun_out/${T}_gred.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/dw_bench.py --ops bwd_data,bwd_data_gred > gpurun_out/${T}_dwb.log 2>&1 || exit $?
grep TOTAL gpurun_out/${T}_dwb.log
bash tools/gpu_run.sh $T tests prof
