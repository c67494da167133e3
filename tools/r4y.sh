#!/bin/bash
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_pwbwd.py tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_dp_equiv.py > $O/r4y_tests.log 2>&1
rc=$?; tail -3 $O/r4y_tests.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0"
timeout -k 10 400 $B > $O/r4y_bench.log 2>&1 || exit $?
ROD_DISABLE=chainpro timeout -k 10 400 $B > $O/r4y_bench_off.log 2>&1 || exit $?
for f in r4y_bench r4y_bench_off; do grep -h "^{" $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
