#!/bin/bash
# Linear-BatchNorm fast paths in the chained prologue / gred sums: parity, then bench A/B (chain on/off, twice).
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_pwbwd.py tests/test_gpu_train.py tests/test_gpu_fullsize.py > $O/r4z_tests.log 2>&1
rc=$?; tail -3 $O/r4z_tests.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0"
for i in 1 2; do
timeout -k 10 400 $B > $O/r4z_bench_$i.log 2>&1 || exit $?
ROD_DISABLE=chainpro timeout -k 10 400 $B > $O/r4z_bench_off_$i.log 2>&1 || exit $?
done
for f in r4z_bench_1 r4z_bench_off_1 r4z_bench_2 r4z_bench_off_2; do grep -h "^{" $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
