#!/bin/bash
# DP step equivalence + training bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_dp_equiv.py -s > gpurun_out/g1.log 2>&1
rc=$?; grep -E "PASS|FAIL|sync |Error|decisions" gpurun_out/g1.log | cut -c1-300; tail -3 gpurun_out/g1.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference > gpurun_out/bench_t2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_t2.log | cut -c1-400
exit $rc
