#!/bin/bash
# end-of-round A/B of the step's opt-out / opt-in switches against the default (same box)
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0"
for v in "default:" "pro3:ROD_DISABLE=pro3" "stembn:ROD_DISABLE=stembn" "pwgred:ROD_DISABLE=pwgred" "side:ROD_ENABLE=side" "default2:"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 300 $B > $O/r4ad_$n.log 2>&1 || exit $?
  grep -h "^{" $O/r4ad_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'])"
done
