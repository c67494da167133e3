# depthwise kernels with buffer I/O: parity + A/B (librod_base.so = previous commit)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_dwfused.py tests/test_gpu_kernels.py > $O/r4c_tests.log 2>&1
rc=$?; tail -5 $O/r4c_tests.log; [ $rc -ne 0 ] && exit $rc
B=road-object-detection-for-bdd100k_amd/lib/librod_base.so
timeout -k 10 300 env ROD_LIB=$B python tools/dwfused_bench.py > $O/r4c_dwfb_base.log 2>&1 || exit $?
timeout -k 10 300 python tools/dwfused_bench.py > $O/r4c_dwfb.log 2>&1 || exit $?
timeout -k 10 300 env ROD_LIB=$B python tools/dw_bench.py > $O/r4c_dwb_base.log 2>&1 || exit $?
timeout -k 10 300 python tools/dw_bench.py > $O/r4c_dwb.log 2>&1 || exit $?
tail -13 $O/r4c_dwfb_base.log; tail -13 $O/r4c_dwfb.log; tail -12 $O/r4c_dwb_base.log; tail -12 $O/r4c_dwb.log
