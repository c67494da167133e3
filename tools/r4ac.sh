#!/bin/bash
# end-of-round PMC traffic of the training step (FETCH_SIZE / WRITE_SIZE passes) -> pmc_traffic.json
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r4e pmcfetch pmcwrite || exit $?
f=$(ls gpurun_out/pmcf_r4e/*counter_collection.csv) && w=$(ls gpurun_out/pmcw_r4e/*counter_collection.csv) &&
python tools/pmc_traffic.py $f $w gpurun_out/r4e_pmc_traffic.json REFINE 8 720 1280 bf16 && gzip -f $f $w && python -c "
import json; d=json.load(open('gpurun_out/r4e_pmc_traffic.json')); print(json.dumps(d)[:1500])"
