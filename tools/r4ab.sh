#!/bin/bash
# after the watchdog fix: the DP graph tests, the default bench (all legs), the graphed-step trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -x tests/test_gpu_graph_dp.py > $O/r4ab_tests.log 2>&1
rc=$?; tail -2 $O/r4ab_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py > $O/r4final_bench.log 2>&1 || exit $?
grep -h '^{' $O/r4final_bench.log > $O/r4final_bench.json
python -c "import json; d=json.load(open('$O/r4final_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['tfrecord']['value'], d['inference']['value'], d['inference_1080p']['value'], d['training_fp32']['value'], d['dp_overhead'])"
bash tools/r4prof.sh r4final > /dev/null 2>&1; head -3 $O/prof_r4final/summary.txt
