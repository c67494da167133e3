#!/bin/bash
# Targeted GPU check: BN-backward micro-bench (f64-checked), ABI, DP step equivalence,
# ALL-mode deconv/merge variants, then the bench.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bn_bench.py > gpurun_out/bn_t1.log 2>&1; rc=$?; cat gpurun_out/bn_t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_abi.py tests/test_gpu_dp_equiv.py "tests/test_gpu_train.py::test_all_mode_step_matches_oracle" -s > gpurun_out/g1.log 2>&1
rc=$?; grep -E "PASS|FAIL|sync |Error|decisions" gpurun_out/g1.log | cut -c1-300; tail -3 gpurun_out/g1.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference > gpurun_out/bench_t1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_t1.log | cut -c1-900
exit $rc
