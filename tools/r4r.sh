#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
ROD_DWF_S2P_V=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_gpu_dwfused.py tests/test_gpu_dwfused_oracle.py 2>&1 | tail -2 &&
echo "== V4" && timeout -k 10 200 python -u tools/dwfused_bench.py 2>&1 | grep -E " s2 |TOTAL" &&
echo "== V2" && ROD_DWF_S2P_V=2 timeout -k 10 200 python -u tools/dwfused_bench.py 2>&1 | grep -E " s2 |TOTAL"
