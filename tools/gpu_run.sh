#!/bin/bash
# GPU-box runner: each GPU step under its own timeout; stop at the first fault/abort/timeout
# (exit 124/134/137/139 or signal), continue past ordinary test failures (exit 1).
# usage: tools/gpu_run.sh <tag> <step>...   steps: tests smoke bench prof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=$1; shift
fatal() { case $1 in 124|134|137|139|130|143) return 0;; *) [ $1 -gt 128 ] && return 0; return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/${TAG}_steps.log
  timeout -k 10 $to "$@" > $OUT/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/${TAG}_steps.log
  tail -5 $OUT/${TAG}_${name}.log
  if fatal $rc; then echo "FATAL rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    tests) run tests 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider ;;
    testsall) run testsall 900 python -m pytest tests -m gpu -q --timeout=600 -p no:cacheprovider ;;
    clitest) run clitest 400 python -m pytest tests/test_gpu_fullsize.py -m gpu -q -k cli --timeout=300 -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 10 --warmup 3 ;;
    benchfast) run benchfast 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    benchall) run benchall 600 python bench.py --steps 5 --warmup 2 --train_range ALL --no-cpu-baseline --no-inference ;;
    benchallfr) run benchallfr 600 python bench.py --steps 5 --warmup 2 --train_range ALL --no-fix-refine --no-cpu-baseline --no-inference ;;
    benchaug) run benchaug 600 python bench.py --steps 10 --warmup 3 --augment --no-cpu-baseline --no-inference --probe-table $OUT/${TAG}_probe_aug.json ;;
    benchaug2) run benchaug2 600 python bench.py --steps 10 --warmup 3 --augment --no-cpu-baseline --no-inference ;;
    cli) run cli_train 300 python road-object-detection-for-bdd100k_amd/train.py --train_range=ALL --batch_size=2 --max_number_of_steps=4 --log_every_n_steps=2 --save_every_n_steps=4 --checkpoint_refine=None --train_dir=gpurun_out/ckpt --summary_dir=gpurun_out/summ &&
         run cli_eval 300 python road-object-detection-for-bdd100k_amd/evaluate.py --checkpoint_path=gpurun_out/ckpt --batch_size=2 --num_images=6 --eval_dir=gpurun_out/eval &&
         run cli_predict 300 python road-object-detection-for-bdd100k_amd/predict.py --checkpoint_all=gpurun_out/ckpt/mobilenet_v2.model --batch_size=2 --num_batches=2 --output=gpurun_out/pred.json ;;
    probetable) run probetable 400 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-inference --probe-table $OUT/${TAG}_probe_table.json ;;
    probetableall) run probetableall 400 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-inference --train_range ALL --probe-table $OUT/${TAG}_probe_table_all.json ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference ;;
    profall) run profall 600 rocprofv3 --kernel-trace --stats -d $OUT/profall_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference --train_range ALL ;;
    profpred) run profpred 400 rocprofv3 --kernel-trace --stats -d $OUT/profpred_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 720 --batch 32 --iters 10 ;;
    profpred1080) run profpred1080 400 rocprofv3 --kernel-trace --stats -d $OUT/profpred1080_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 8 --iters 10 ;;
    pmcfetch) run pmcfetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-inference ;;
    pmcwrite) run pmcwrite 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-inference ;;
    *) echo "unknown step $step" ;;
  esac
done
echo ALLDONE
