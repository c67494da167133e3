#!/bin/bash
# round 4: project backward with the depthwise BatchNorm's sums (rod_pw_bwd_gred): parity, step tests, bench
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_pwbwd.py 2>&1 | tee $O/r4f_tests.log &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_train.py 2>&1 | tail -5 | tee -a $O/r4f_tests.log &&
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0" &&
timeout -k 10 400 $B > $O/r4f_bench.log 2>&1 &&
timeout -k 10 400 env ROD_DISABLE=pwgred $B > $O/r4f_bench_off.log 2>&1 &&
for f in r4f_bench r4f_bench_off; do echo "$f $(grep -h '^{' $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; done
