# round 4: train.py graphed feed + split DP graph + slab range flush
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_graph_dp.py tests/test_gpu_bench_dp.py tests/test_gpu_fullsize.py -k "graph or tfrecord or two_ranks or cli" > $O/r4b_tests.log 2>&1
rc=$?; tail -15 $O/r4b_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --kernel-steps 0 > $O/r4b_bench.log 2>&1
rc=$?; tail -c 3000 $O/r4b_bench.log; exit $rc
