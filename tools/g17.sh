#!/bin/bash
# A/B: 192-wide N tiles for Cout % 192 == 0 (> 256) vs 128-wide (ROD_DEBUG_N128=1)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out
ROD_DEBUG_N128=1 timeout -k 10 200 python tools/conv_bench.py --shapes 5,6,10,11,12 --ops fwd_plain,fwd_stats,bwd_data --out /tmp/g17_old.pt > $O/g17_old.log 2>&1 || exit 1
timeout -k 10 200 python tools/conv_bench.py --shapes 5,6,10,11,12 --ops fwd_plain,fwd_stats,bwd_data --check /tmp/g17_old.pt > $O/g17_new.log 2>&1 || exit 1
grep -hv amdgpu $O/g17_old.log $O/g17_new.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g17_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/g17_tests.log; exit 1; }
tail -1 $O/g17_tests.log
for v in 1 0; do
if [ $v = 1 ]; then export ROD_DEBUG_N128=1; else unset ROD_DEBUG_N128; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > $O/g17_b$v.log 2>&1 || exit 1
echo n128=$v $(grep -h '^{' $O/g17_b$v.log | cut -c60-100)
done
