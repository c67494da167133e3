set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_gred.py -m gpu -q -x --timeout=250 -p no:cacheprovider > $O/r3k_k.log 2>&1; echo k rc=$?; tail -n 2 $O/r3k_k.log
timeout -k 10 300 env ROD_DISABLE=gredpw python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --kernel-steps 0 > $O/r3k_bench0.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --kernel-steps 0 > $O/r3k_bench1.log 2>&1 || exit $?
grep -h '^{' $O/r3k_bench0.log $O/r3k_bench1.log | cut -c1-150
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --probe-table $O/r3k_pt1.json > $O/r3k_pt1.log 2>&1 || exit $?
