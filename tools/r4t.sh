#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY -d $O/pmc_r4t -o p --output-format csv -- python3 tools/dwfused_bench.py > $O/r4t_pmc.log 2>&1 &&
python tools/pmc_kernel_summary.py $O/pmc_r4t/p_counter_collection.csv fused2 s2p 2>&1 | head -40
