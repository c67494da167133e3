#!/bin/bash
# One-launch BatchNorm statistic merge: parity, bench, graphed-step kernel trace.
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_pwbwd.py -k "finalize or epilogue_bn or pw_stream or pw_bwd or gred" > $O/r4aa_k.log 2>&1
rc=$?; tail -3 $O/r4aa_k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_train.py > $O/r4aa_tests.log 2>&1
rc=$?; tail -3 $O/r4aa_tests.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0"
for i in 1 2; do timeout -k 10 400 $B > $O/r4aa_bench_$i.log 2>&1 || exit $?; done
for f in r4aa_bench_1 r4aa_bench_2; do grep -h "^{" $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
bash tools/r4prof.sh r4aa > /dev/null || exit $?
grep -i "merge\|total\|bn_" $O/prof_r4aa/summary.txt | head -20 | cut -c1-140
