#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_msf.py > gpurun_out/t3.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/t3.log | cut -c1-400 | head -40; tail -3 gpurun_out/t3.log
exit $rc
