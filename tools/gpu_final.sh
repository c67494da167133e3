#!/bin/bash
# end-of-session check: full -m gpu suite, smoke, default bench (all legs), graphed-step trace
# usage (on the GPU box): bash tools/gpu_final.sh TAG   -> gpurun_out/TAG_*
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-final}
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -x tests > $O/${T}_tests.log 2>&1
rc=$?; tail -3 $O/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${T}_smoke.log 2>&1 || exit $?
tail -1 $O/${T}_smoke.log
timeout -k 10 900 python bench.py > $O/${T}_bench.log 2>&1 || exit $?
grep -h '^{' $O/${T}_bench.log > $O/${T}_bench.json
python -c "import json; d=json.load(open('$O/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['tfrecord']['value'], d['inference']['value'], d['inference_1080p']['value'], d['training_fp32']['value'])"
bash tools/gpu_prof.sh ${T} > /dev/null 2>&1; head -3 $O/prof_${T}/summary.txt
