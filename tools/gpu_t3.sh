#!/bin/bash
# VGG-16 kernels + REFINE step parity.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_vgg.py > gpurun_out/t3_vgg.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/t3_vgg.log | cut -c1-300 | head -40; tail -3 gpurun_out/t3_vgg.log
exit $rc
