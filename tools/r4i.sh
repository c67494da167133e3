#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/pwgred_bench.py 2>&1 | grep -v amdgpu.ids | tee $O/r4i_pwgred.log &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM -d $O/pmc_r4i -o p --output-format csv -- python3 tools/pwgred_bench.py --only --iters 3 > $O/r4i_pmc.log 2>&1 &&
python tools/pmc_kernel_summary.py $O/pmc_r4i/p_counter_collection.csv pw_bwd_gred 2>&1 | head -40
