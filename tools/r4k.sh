#!/bin/bash
# depthwise forward (BN prologue + statistics): per-shape timing + PMC instruction mix
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/dw_bench.py --ops fwdpro 2>&1 | grep -v amdgpu.ids | tee $O/r4k_dwfwd.log &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $O/pmc_r4k -o p --output-format csv -- python3 tools/dw_bench.py --ops fwdpro --iters 2 > $O/r4k_pmc.log 2>&1 &&
python tools/pmc_kernel_summary.py $O/pmc_r4k/p_counter_collection.csv dw3x3_fwd 2>&1 | head -60
