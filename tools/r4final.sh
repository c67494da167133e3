#!/bin/bash
# round-4 final: full -m gpu suite, smoke, default bench (all legs), graphed-step trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -x tests > $O/r4final_tests.log 2>&1
rc=$?; tail -3 $O/r4final_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4final_smoke.log 2>&1 || exit $?
tail -1 $O/r4final_smoke.log
timeout -k 10 900 python bench.py > $O/r4final_bench.log 2>&1 || exit $?
grep -h '^{' $O/r4final_bench.log > $O/r4final_bench.json
python -c "import json; d=json.load(open('$O/r4final_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['tfrecord']['value'], d['inference']['value'], d['inference_1080p']['value'], d['training_fp32']['value'])"
bash tools/r4prof.sh r4final > /dev/null 2>&1; head -3 $O/prof_r4final/summary.txt
