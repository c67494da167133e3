#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 4 8; do echo "== V=$v"; ROD_DW_FWD_V=$v timeout -k 10 200 python -u tools/dw_bench.py --ops fwdpro 2>&1 | grep -v amdgpu.ids || exit 1; done
for w in 512 2048 4096; do echo "== WANT=$w"; ROD_DW_WANT=$w timeout -k 10 200 python -u tools/dw_bench.py --ops fwdpro 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "== RBMIN=4"; ROD_DW_RBMIN=4 timeout -k 10 200 python -u tools/dw_bench.py --ops fwdpro 2>&1 | grep -v amdgpu.ids
