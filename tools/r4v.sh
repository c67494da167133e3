#!/bin/bash
# round 4 evidence: fresh C5 (1080p predict) PMC roofline report and the training step's PMC traffic
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r4 c5 pmcfetch pmcwrite || exit $?
f=$(ls gpurun_out/pmcf_r4/*counter_collection.csv) && w=$(ls gpurun_out/pmcw_r4/*counter_collection.csv) &&
python tools/pmc_traffic.py $f $w gpurun_out/r4_pmc_traffic.json REFINE 8 720 1280 bf16 && gzip -f $f $w && cat gpurun_out/r4_c5_report.json | head -60
