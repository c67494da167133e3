#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u tools/dwfused_bench.py 2>&1 | grep -v amdgpu.ids | grep -E "fused|TOTAL" | awk '{print $1, $2, $6, $7}' || exit 1; }
run X=0
run ROD_DWF_RING=6
run ROD_DW_WANT=512
run ROD_DW_WANT=2048
run ROD_DW_RBMIN=16
run ROD_DWF_C2=0
