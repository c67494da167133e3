#!/bin/bash
# graphed-step kernel trace (rocprofv3 --kernel-trace --stats) -> gpurun_out/prof_$1/summary.txt
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-cur}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$T -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 > $O/prof_$T.log 2>&1 || exit $?
python tools/trace_summary.py $O/prof_$T/run_kernel_trace.csv normalize_image 5+2 "REFINE train step bf16 b8 720p, graph replays" > $O/prof_$T/summary.txt 2>&1
rm -f $O/prof_$T/run_kernel_trace.csv $O/prof_$T/run_agent_info.csv
head -60 $O/prof_$T/summary.txt | cut -c1-150
