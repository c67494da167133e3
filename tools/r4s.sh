#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
ROD_DWF_S2P_D=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_gpu_dwfused.py 2>&1 | tail -2 &&
echo "== V2 D2" && timeout -k 10 200 python -u tools/dwfused_bench.py 2>&1 | grep -E " s2 |TOTAL" &&
echo "== V2 D3" && ROD_DWF_S2P_D=3 timeout -k 10 200 python -u tools/dwfused_bench.py 2>&1 | grep -E " s2 |TOTAL"
