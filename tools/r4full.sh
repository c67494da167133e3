#!/bin/bash
# full -m gpu suite, then bench (all legs) and the graphed-step trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4full}
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -x tests > $O/${T}_tests.log 2>&1
rc=$?; tail -4 $O/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py > $O/${T}_bench.log 2>&1 || exit $?
grep -h '^{' $O/${T}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'], d.get('tfrecord',{}).get('value'), d.get('cpu_baseline'))" | cut -c1-600
