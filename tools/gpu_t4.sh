#!/bin/bash
# graph-replayed step: equivalence test + bench with and without --graph
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider "tests/test_gpu_train.py::test_step_graphed_bit_identical" > gpurun_out/t4.log 2>&1; rc=$?; tail -3 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 > gpurun_out/t4_eager.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 --graph > gpurun_out/t4_graph.log 2>&1 || exit $?
tail -1 gpurun_out/t4_eager.log | cut -c1-260; tail -1 gpurun_out/t4_graph.log | cut -c1-260
