#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_pwbwd.py 2>&1 | tail -3 | tee $O/r4h_tests.log &&
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0" &&
timeout -k 10 400 $B > $O/r4h_bench.log 2>&1 &&
echo "bench $(grep -h '^{' $O/r4h_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" &&
bash tools/r4prof.sh r4h 2>&1 | grep -E "kernel time|gred|pw_bwd|apply|reduce" | cut -c1-120
