# full GPU suite + fused dw bench + bench (default / gredpw) + graphed-step kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -x tests > $O/r4d_tests.log 2>&1
rc=$?; tail -8 $O/r4d_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/dwfused_bench.py > $O/r4d_dwfb.log 2>&1 || exit $?
tail -13 $O/r4d_dwfb.log
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0"
timeout -k 10 400 $B > $O/r4d_bench.log 2>&1 || exit $?
timeout -k 10 400 env ROD_ENABLE=gredpw $B > $O/r4d_bench_gredpw.log 2>&1 || exit $?
for f in r4d_bench r4d_bench_gredpw; do echo "$f $(grep -h '^{' $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])")"; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_r4d -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0 > $O/r4d_prof.log 2>&1 || exit $?
python tools/trace_summary.py $O/prof_r4d/run_kernel_trace.csv normalize_image 5+2 "REFINE train step bf16 b8 720p, graph replays" > $O/prof_r4d/summary.txt 2>&1
rm -f $O/prof_r4d/run_kernel_trace.csv $O/prof_r4d/run_agent_info.csv
head -40 $O/prof_r4d/summary.txt | cut -c1-160
