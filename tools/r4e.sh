#!/bin/bash
# round 4: buffer-store fence check (depthwise sweep) + streaming pw_bwd parity and timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=road-object-detection-for-bdd100k_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_dwsweep.py tests/test_gpu_pwbwd.py 2>&1 | tee gpurun_out/r4e_tests.log &&
timeout -k 10 200 python -u tools/pwbwd_bench.py --pw-only 2>&1 | tee gpurun_out/r4e_pwb_stream.log &&
ROD_PWB_STREAM=0 timeout -k 10 200 python -u tools/pwbwd_bench.py --pw-only 2>&1 | tee gpurun_out/r4e_pwb_block.log
