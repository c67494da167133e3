set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_dwfused.py -m gpu -q -x --timeout=250 -p no:cacheprovider > $O/r3g_dwft.log 2>&1; echo dwft rc=$?
timeout -k 10 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_d3.so python -m pytest tests/test_gpu_dwfused.py -m gpu -q -x --timeout=250 -p no:cacheprovider > $O/r3g_dwft3.log 2>&1; echo dwft3 rc=$?
timeout -k 10 200 env ROD_DWF_V1=1 python tools/dwfused_bench.py > $O/r3g_dwf1.log 2>&1 || exit $?
timeout -k 10 200 python tools/dwfused_bench.py > $O/r3g_dwf2.log 2>&1 || exit $?
timeout -k 10 200 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_d3.so python tools/dwfused_bench.py > $O/r3g_dwf3.log 2>&1 || exit $?
tail -n 3 $O/r3g_dwft.log; tail -n 3 $O/r3g_dwft3.log
grep s2 $O/r3g_dwf1.log $O/r3g_dwf2.log $O/r3g_dwf3.log; grep TOTAL $O/r3g_dwf*.log
timeout -k 10 900 python -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_dp_equiv.py -m gpu -q -x --timeout=500 -p no:cacheprovider > $O/r3g_train.log 2>&1; echo train rc=$?; tail -n 3 $O/r3g_train.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg > $O/r3g_bench.log 2>&1; grep '^{' $O/r3g_bench.log | cut -c1-200
