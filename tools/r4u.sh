#!/bin/bash
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_stem.py tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_fullsize.py > $O/r4u_tests.log 2>&1
rc=$?; tail -3 $O/r4u_tests.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0"
timeout -k 10 400 $B > $O/r4u_bench.log 2>&1 || exit $?
ROD_DISABLE=pro3 timeout -k 10 400 $B > $O/r4u_bench_off.log 2>&1 || exit $?
for f in r4u_bench r4u_bench_off; do grep -h "^{" $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
