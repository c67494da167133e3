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
# kernel-trace CSVs can be tens of MB (gpurun copies back <= 64 MiB): summarise on the box, keep
# the per-kernel stats CSV, drop the raw trace
summ() {  # dir marker iterations title
  python tools/trace_summary.py $1/run_kernel_trace.csv "$2" $3 "$4" > $1/summary.txt 2>&1
  rm -f $1/run_kernel_trace.csv $1/run_agent_info.csv
  head -25 $1/summary.txt | cut -c1-200
}
for step in "$@"; do
  case $step in
    rcinf) run rcinftest 300 python -u -m pytest tests/test_gpu_recompute.py -k predict -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider &&
         for i in 1 2; do run pinf0_$i 200 env ROD_DISABLE=rcinf python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run pinf1_$i 200 python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run pinf720_0_$i 200 env ROD_DISABLE=rcinf python tools/predict_bench.py --res 720 --batch 32 --iters 20 && run pinf720_1_$i 200 python tools/predict_bench.py --res 720 --batch 32 --iters 20; done; grep -H ms_per_batch $OUT/${TAG}_pinf*.log ;;
    rcinfab) for i in 1 2; do for cfg in "" "ROD_DISABLE=irblock" "ROD_DISABLE=irblock ROD_ENABLE=rcinf1"; do n=$(echo "$cfg" | tr -c 'a-z0-9\n' '_'); run pq${n}_$i 200 env $cfg python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run pq720${n}_$i 200 env $cfg python tools/predict_bench.py --res 720 --batch 32 --iters 20; done; done; grep -H ms_per_batch $OUT/${TAG}_pq*.log ;;
    rcfwdab) run rcfwdtest 400 python -u -m pytest tests/test_gpu_recompute.py tests/test_gpu_irblock.py -k "dw3x3_fwd_rc or predict or step or backbone" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
         run rcb_prev 200 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python tools/rc_bench.py b1 b2 b3 b6 && run rcb_new 200 python tools/rc_bench.py b1 b2 b3 b6 && run rcb_narrow 200 env ROD_STATS_NARROW=1 python tools/rc_bench.py b1 b3 &&
         for i in 1 2; do run pr0_$i 200 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run pr1_$i 200 python tools/predict_bench.py --res 1080 --batch 8 --iters 30; done &&
         for i in 1 2; do run tr0_$i 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run tr1_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done;
         grep -H "dwfwd\|expand" $OUT/${TAG}_rcb_*.log; grep -H ms_per_batch $OUT/${TAG}_pr*.log; grep -H -o '"value": [0-9.]*' $OUT/${TAG}_tr*.log ;;
    rcv) run rcvtest 300 env ROD_DW_RC_V=4 python -u -m pytest tests/test_gpu_recompute.py -k predict -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider &&
         for i in 1 2; do run pv8_$i 200 python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run pv4_$i 200 env ROD_DW_RC_V=4 python tools/predict_bench.py --res 1080 --batch 8 --iters 30; done &&
         for i in 1 2; do run qv8_$i 200 python tools/predict_bench.py --res 720 --batch 32 --iters 20 && run qv4_$i 200 env ROD_DW_RC_V=4 python tools/predict_bench.py --res 720 --batch 32 --iters 20; done;
         grep -H ms_per_batch $OUT/${TAG}_pv*.log $OUT/${TAG}_qv*.log ;;
    statsab) run statstest 400 python -u -m pytest tests/test_gpu_recompute.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
         run stb0 200 env ROD_STATS_TILE=0 python tools/rc_bench.py b1 b3 && run stb1 200 python tools/rc_bench.py b1 b3 &&
         for i in 1 2; do run st0_$i 300 env ROD_STATS_TILE=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run st1_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done;
         grep -H "expand" $OUT/${TAG}_stb*.log; grep -H -o '"value": [0-9.]*' $OUT/${TAG}_st?_*.log ;;
    c5heads) run cbh0 200 python tools/conv_bench.py --shapes 19,20,21,22,23 --ops fwd_plain && run cbh1 200 env ROD_DISABLE=splitk python tools/conv_bench.py --shapes 19,20,21,22,23 --ops fwd_plain ;;
    cinpad) run cptest 400 python -u -m pytest tests/test_gpu_bnepi.py tests/test_gpu_fullsize.py -k "bnepi or cinpad or 1080p" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
         for i in 1 2; do run cp0_$i 200 env ROD_DISABLE=cinpad python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run cp1_$i 200 python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run cq0_$i 200 env ROD_DISABLE=cinpad python tools/predict_bench.py --res 720 --batch 32 --iters 20 && run cq1_$i 200 python tools/predict_bench.py --res 720 --batch 32 --iters 20; done;
         grep -H ms_per_batch $OUT/${TAG}_cp?_*.log $OUT/${TAG}_cq?_*.log ;;
    dwtable) run dwtable 300 python tools/dw_bench.py --ops fwd,fwdpro && grep -E "^fwd|TOTAL" $OUT/${TAG}_dwtable.log > $OUT/${TAG}_dw_fwd_table.txt ;;
    slabab) run slabtest 400 env ROD_SLAB_POLICY=1 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_train.py -k "defer or refine" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
         for i in 1 2 3; do run sl0_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run sl1_$i 300 env ROD_SLAB_POLICY=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done;
         grep -H -o '"value": [0-9.]*' $OUT/${TAG}_sl?_*.log ;;
    predprev) for i in 1 2; do run pp0_$i 200 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run pp1_$i 200 python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run pq0_$i 200 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python tools/predict_bench.py --res 720 --batch 32 --iters 20 && run pq1_$i 200 python tools/predict_bench.py --res 720 --batch 32 --iters 20; done;
         grep -H ms_per_batch $OUT/${TAG}_pp?_*.log $OUT/${TAG}_pq?_*.log ;;
    trprev) run trtest 400 python -u -m pytest tests/test_gpu_recompute.py tests/test_gpu_pwbwd.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
         for i in 1 2 3; do run tp0_$i 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run tp1_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done;
         grep -H -o '"value": [0-9.]*' $OUT/${TAG}_tp?_*.log ;;
    profab) run profa 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so rocprofv3 --kernel-trace --stats -d $OUT/profa_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 &&
         run profb 300 rocprofv3 --kernel-trace --stats -d $OUT/profb_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 &&
         rm -f $OUT/profa_$TAG/run_kernel_trace.csv $OUT/profb_$TAG/run_kernel_trace.csv ;;
    trprev2) run trtest2 400 python -u -m pytest tests/test_gpu_recompute.py tests/test_gpu_pwbwd.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
         for i in 1 2; do run tq0_$i 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run tq1_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done;
         grep -H -o '"value": [0-9.]*' $OUT/${TAG}_tq?_*.log ;;
    sepi) run sepitest 400 python -u -m pytest tests/test_gpu_bnepi.py tests/test_gpu_recompute.py -k "predict" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
         for i in 1 2; do run se0_$i 200 env ROD_DISABLE=streamepi python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run se1_$i 200 python tools/predict_bench.py --res 1080 --batch 8 --iters 30 && run sf0_$i 200 env ROD_DISABLE=streamepi python tools/predict_bench.py --res 720 --batch 32 --iters 20 && run sf1_$i 200 python tools/predict_bench.py --res 720 --batch 32 --iters 20; done;
         grep -H ms_per_batch $OUT/${TAG}_se?_*.log $OUT/${TAG}_sf?_*.log ;;
    bnsmall) for v in 4 2 1; do run bnsmall_$v 200 env ROD_BN_SMALL_CVB=$v python tools/bn_bench.py --iters 20; done; grep -H -E "M= *(1920|480|120) |TOTAL" $OUT/${TAG}_bnsmall_*.log ;;
    tests) run tests 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider ;;
    testsall) run testsall 900 python -m pytest tests -m gpu -q --timeout=600 -p no:cacheprovider ;;
    clitest) run clitest 400 python -m pytest tests/test_gpu_fullsize.py -m gpu -q -k cli --timeout=300 -p no:cacheprovider ;;
    merge) run merge 400 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_kernels.py tests/test_gpu_defer.py -k "merge or finalize or defer" -m gpu -v --timeout=300 --timeout-method thread -p no:cacheprovider &&
        run mergedbg 300 env ROD_DEBUG_MERGE=1 python bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 ;;
    abmerge) for i in 1 2; do run abm2_$i 300 env ROD_MERGE_TWO_LAUNCH=1 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abm1_$i 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done; grep -h '"value"' $OUT/${TAG}_abm*.log | cut -c1-60 ;;
    abproj) for i in 1 2; do run abp0_$i 300 env ROD_PW_PROJ=0 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abp1_$i 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done; grep -h '"value"' $OUT/${TAG}_abp*.log | cut -c1-60 ;;
    cbproj) run cbproj0 300 env ROD_PW_PROJ=0 python tools/conv_bench.py --ops fwd_stats --shapes 1,3,16,17,18 &&
        run cbproj1 300 python tools/conv_bench.py --ops fwd_stats --shapes 1,3,16,17,18 ;;
    cbdeep) run cbd0 300 env ROD_PW_PROJ=0 python tools/conv_bench.py --ops fwd_stats --shapes 16 &&
        run cbd2 300 python tools/conv_bench.py --ops fwd_stats --shapes 16 &&
        run cbexp 300 python tools/conv_bench.py --ops fwd_plain,fwd_stats --shapes 0,2,4 ;;
    abprev) for i in 1 2; do run abq0_$i 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abq1_$i 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; done; grep -h '"value"' $OUT/${TAG}_abq*.log | cut -c1-60 ;;
    abprev3) run abr0_1 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abr1_1 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abr1_2 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abr0_2 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abr0_3 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_prev.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abr1_3 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; grep -h '"value"' $OUT/${TAG}_abr*.log | cut -c1-60 ;;
    abproj3) run abs0_1 300 env ROD_PW_PROJ=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abs1_1 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abs1_2 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abs0_2 300 env ROD_PW_PROJ=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abs0_3 300 env ROD_PW_PROJ=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abs1_3 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; grep -h '"value"' $OUT/${TAG}_abs*.log | cut -c1-60 ;;
    absplit3) run abt0_1 300 env ROD_SPLIT_FUSE=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abt1_1 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abt1_2 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abt0_2 300 env ROD_SPLIT_FUSE=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abt0_3 300 env ROD_SPLIT_FUSE=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 && run abt1_3 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0; grep -h '"value"' $OUT/${TAG}_abt*.log | cut -c1-60 ;;
    splittest) run splittest 400 python -u -m pytest tests/test_gpu_splitk.py tests/test_gpu_bwd_data_bn.py tests/test_gpu_kernels.py -k "split or bwd_data or prologue" -m gpu -v --timeout=200 --timeout-method thread -p no:cacheprovider ;;
    streamtest) run streamtest 300 python -u -m pytest tests/test_gpu_pwproj.py tests/test_gpu_kernels.py -k "pw_stream or pw_proj or prologue" -m gpu -v --timeout=200 --timeout-method thread -p no:cacheprovider ;;
    projtest) run projtest 300 python -u -m pytest tests/test_gpu_pwproj.py -m gpu -v --timeout=200 --timeout-method thread -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 10 --warmup 3 ;;
    benchfast) run benchfast 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    benchfp32) run benchfp32 600 python bench.py --dtype fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-inference ;;
    benchgred) run benchgred 400 env ROD_ENABLE=gred python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 &&
               run benchbase 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 &&
               run benchgreddw 400 env ROD_ENABLE=gred,dwbn python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --kernel-steps 0 ;;
    hosttime) run hosttime 300 python tools/host_time.py --steps 10 ;;
    hostprof) run hostprof 300 python -m cProfile -s tottime tools/host_time.py --steps 5 ;;
    bnu) run bnu4 300 python tools/bn_bench.py --out /tmp/${TAG}_bn4.pt && run bnu8 300 env ROD_BN_RED_U=8 python tools/bn_bench.py --check /tmp/${TAG}_bn4.pt ;;
    bna) run bna4 300 python tools/bn_bench.py --out /tmp/${TAG}_bn4.pt && run bna8 300 env ROD_BN_APPLY_U=8 python tools/bn_bench.py --check /tmp/${TAG}_bn4.pt ;;
    dwplan) run dwp0 300 python tools/dw_bench.py --out /tmp/${TAG}_dw.pt &&
            run dwp1 300 env ROD_DW_WANT=2048 python tools/dw_bench.py --check /tmp/${TAG}_dw.pt &&
            run dwp2 300 env ROD_DW_WANT=512 python tools/dw_bench.py --check /tmp/${TAG}_dw.pt &&
            run dwp3 300 env ROD_DW_RBMIN=4 python tools/dw_bench.py --check /tmp/${TAG}_dw.pt &&
            run dwp4 300 env ROD_DW_RBMIN=16 python tools/dw_bench.py --check /tmp/${TAG}_dw.pt ;;
    dwplan2) run dwq0 300 python tools/dw_bench.py --out /tmp/${TAG}_dw.pt &&
             run dwq1 300 env ROD_DW_RBMIN=16 python tools/dw_bench.py --check /tmp/${TAG}_dw.pt &&
             run dwq2 300 env ROD_DW_RBMIN=24 python tools/dw_bench.py --check /tmp/${TAG}_dw.pt &&
             run dwq3 300 env ROD_DW_RBMIN=32 python tools/dw_bench.py --check /tmp/${TAG}_dw.pt ;;
    wgplan) run wg0 300 python tools/conv_bench.py --ops wgrad --out /tmp/${TAG}_wg.pt &&
            run wg1 300 env ROD_WG_TARGET=4096 python tools/conv_bench.py --ops wgrad --check /tmp/${TAG}_wg.pt &&
            run wg2 300 env ROD_WG_TARGET=1024 python tools/conv_bench.py --ops wgrad --check /tmp/${TAG}_wg.pt &&
            run wg3 300 env ROD_WG_MINROWS=256 python tools/conv_bench.py --ops wgrad --check /tmp/${TAG}_wg.pt &&
            run wg4 300 env ROD_WG_MINROWS=1024 python tools/conv_bench.py --ops wgrad --check /tmp/${TAG}_wg.pt ;;
    bnwant) run bw0 300 python tools/bn_bench.py --out /tmp/${TAG}_bn.pt &&
            run bw1 300 env ROD_BN_RED_WANT=2048 python tools/bn_bench.py --check /tmp/${TAG}_bn.pt &&
            run bw2 300 env ROD_BN_RED_WANT=512 python tools/bn_bench.py --check /tmp/${TAG}_bn.pt &&
            run bw3 300 env ROD_BN_RED_WANT=256 python tools/bn_bench.py --check /tmp/${TAG}_bn.pt ;;
    benchall) run benchall 600 python bench.py --steps 5 --warmup 2 --train_range ALL --no-cpu-baseline --no-inference ;;
    benchallfr) run benchallfr 600 python bench.py --steps 5 --warmup 2 --train_range ALL --no-fix-refine --no-cpu-baseline --no-inference ;;
    benchaug) run benchaug 600 python bench.py --steps 10 --warmup 3 --augment --no-cpu-baseline --no-inference --probe-table $OUT/${TAG}_probe_aug.json ;;
    benchaug2) run benchaug2 600 python bench.py --steps 10 --warmup 3 --augment --no-cpu-baseline --no-inference ;;
    cli) run cli_train 300 python road-object-detection-for-bdd100k_amd/train.py --train_range=ALL --batch_size=2 --max_number_of_steps=4 --log_every_n_steps=2 --save_every_n_steps=4 --checkpoint_refine=None --train_dir=gpurun_out/ckpt --summary_dir=gpurun_out/summ &&
         run cli_eval 300 python road-object-detection-for-bdd100k_amd/evaluate.py --checkpoint_path=gpurun_out/ckpt --batch_size=2 --num_images=6 --eval_dir=gpurun_out/eval &&
         run cli_predict 300 python road-object-detection-for-bdd100k_amd/predict.py --checkpoint_all=gpurun_out/ckpt/mobilenet_v2.model --batch_size=2 --num_batches=2 --output=gpurun_out/pred.json ;;
    probetable) run probetable 400 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --probe-table $OUT/${TAG}_probe_table.json ;;
    probetableall) run probetableall 400 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-inference --train_range ALL --probe-table $OUT/${TAG}_probe_table_all.json ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --kernel-steps 0 &&
         summ $OUT/prof_$TAG normalize_image 5+2 "REFINE train step bf16 b8 720p, graph replays" ;;
    profall) run profall 600 rocprofv3 --kernel-trace --stats -d $OUT/profall_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference --train_range ALL ;;
    profpred) run profpred 400 rocprofv3 --kernel-trace --stats -d $OUT/profpred_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 720 --batch 32 --iters 10 &&
         summ $OUT/profpred_$TAG normalize_image 10 "predict path bf16 b32 720p, graph replays" ;;
    profpred1080) run profpred1080 400 rocprofv3 --kernel-trace --stats -d $OUT/profpred1080_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 8 --iters 10 &&
         summ $OUT/profpred1080_$TAG normalize_image 10 "predict path bf16 b8 1080p, graph replays" ;;
    pmcfetch) run pmcfetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --kernel-steps 0 ;;
    pmcwrite) run pmcwrite 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --kernel-steps 0 ;;
    cbhead) run cbhead 300 python tools/conv_bench.py --shapes 7,13,14,15 ;;
    cball) run cball 300 python tools/conv_bench.py ;;
    convtests) run convtests 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_stem.py -m gpu -q -x --timeout=300 -p no:cacheprovider ;;
    c5probe) run c5probe 300 python tools/c5_report.py probe --res 1080 --batch 8 --out $OUT/${TAG}_c5_probe.json ;;
    c5) run c5probe 300 python tools/c5_report.py probe --res 1080 --batch 8 --out $OUT/${TAG}_c5_probe.json &&
        run c5f 130 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/c5f_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 8 --iters 3 --no-graph &&
        run c5w 130 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/c5w_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 8 --iters 3 --no-graph &&
        run c5m 130 timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/c5m_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 8 --iters 3 --no-graph &&
        f=$(ls $OUT/c5f_$TAG/*counter_collection.csv) && w=$(ls $OUT/c5w_$TAG/*counter_collection.csv) && m=$(ls $OUT/c5m_$TAG/*counter_collection.csv) &&
        python tools/c5_report.py pmc $OUT/${TAG}_c5_probe.json $f $w $m --out $OUT/${TAG}_c5_report.json &&
        gzip -f $f $w $m ;;
    c5b32) run c5b32probe 300 python tools/c5_report.py probe --res 1080 --batch 32 --out $OUT/${TAG}_c5b32_probe.json &&
        run c5b32f 200 timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE -d $OUT/c5b32f_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 32 --iters 2 --no-graph &&
        run c5b32w 200 timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE -d $OUT/c5b32w_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 32 --iters 2 --no-graph &&
        run c5b32m 200 timeout -s KILL 190 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/c5b32m_$TAG -o run --output-format csv -- python3 tools/predict_bench.py --res 1080 --batch 32 --iters 2 --no-graph &&
        f=$(ls $OUT/c5b32f_$TAG/*counter_collection.csv) && w=$(ls $OUT/c5b32w_$TAG/*counter_collection.csv) && m=$(ls $OUT/c5b32m_$TAG/*counter_collection.csv) &&
        python tools/c5_report.py pmc $OUT/${TAG}_c5b32_probe.json $f $w $m --out $OUT/${TAG}_c5b32_report.json &&
        gzip -f $f $w $m ;;
    irpmc) run irpmc 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -d $OUT/irpmc_$TAG -o run --output-format csv -- python3 tools/irblock_bench.py --iters 3 --res 1080 &&
           python tools/pmc_kernel_summary.py $OUT/irpmc_$TAG/run_counter_collection.csv ir_block_fwd > $OUT/${TAG}_irpmc.txt &&
           gzip -f $OUT/irpmc_$TAG/run_counter_collection.csv && cat $OUT/${TAG}_irpmc.txt ;;
    irbench) run irbench 300 python tools/irblock_bench.py --iters 10 --res 720 1080 ;;
    dwpmc) run dwpmc 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES -d $OUT/dwpmc_$TAG -o run --output-format csv -- python3 tools/dw_bench.py --iters 3 &&
           python tools/pmc_kernel_summary.py $OUT/dwpmc_$TAG/run_counter_collection.csv dw3x3 > $OUT/${TAG}_dwpmc.txt &&
           gzip -f $OUT/dwpmc_$TAG/run_counter_collection.csv && cat $OUT/${TAG}_dwpmc.txt ;;
    dwfpmc) run dwfpmc 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/dwfpmc_$TAG -o run --output-format csv -- python3 tools/dwfused_bench.py --iters 3 &&
           python tools/pmc_kernel_summary.py $OUT/dwfpmc_$TAG/run_counter_collection.csv dw3x3_bwd_fused > $OUT/${TAG}_dwfpmc.txt &&
           gzip -f $OUT/dwfpmc_$TAG/run_counter_collection.csv && cat $OUT/${TAG}_dwfpmc.txt ;;
    dwfb) run dwfb 300 python tools/dwfused_bench.py ;;
    pws) run pws0 300 env ROD_PW_STREAM=0 python tools/conv_bench.py --ops fwd_plain,fwd_stats --out /tmp/${TAG}_pws.pt &&
         run pws1 300 python tools/conv_bench.py --ops fwd_plain,fwd_stats --check /tmp/${TAG}_pws.pt ;;
    bnpmc) run bnpmc 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $OUT/bnpmc_$TAG -o run --output-format csv -- python3 tools/bn_bench.py --iters 3 &&
           python tools/pmc_kernel_summary.py $OUT/bnpmc_$TAG/run_counter_collection.csv bn_ > $OUT/${TAG}_bnpmc.txt &&
           gzip -f $OUT/bnpmc_$TAG/run_counter_collection.csv && cat $OUT/${TAG}_bnpmc.txt ;;
    dwbench) run dwbench 300 python tools/dw_bench.py ;;
    bnbench) run bnbench 300 python tools/bn_bench.py ;;
    cbench) run cbench 300 python tools/conv_bench.py ;;
    dwab) run dwa 300 env ROD_LIB=road-object-detection-for-bdd100k_amd/lib/librod_w0.so python tools/dw_bench.py --out /tmp/${TAG}_dw0.pt &&
          run dwb 300 python tools/dw_bench.py --check /tmp/${TAG}_dw0.pt ;;
    dwbn) run dwbn 600 python -m pytest tests/test_gpu_dwbn.py tests/test_gpu_train.py tests/test_gpu_kernels.py -m gpu -q -x --timeout=500 -p no:cacheprovider ;;
    traintests) run traintests 800 python -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_vgg.py tests/test_gpu_msf.py tests/test_gpu_dp_equiv.py -m gpu -q -x --timeout=500 -p no:cacheprovider ;;
    irtests) run irtests 300 python -m pytest tests/test_gpu_irblock.py -m gpu -q -x --timeout=250 -p no:cacheprovider ;;
    *) echo "unknown step $step" ;;
  esac
done
echo ALLDONE
