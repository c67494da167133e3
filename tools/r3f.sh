set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 200 env ROD_PW_STREAM=0 python tools/conv_bench.py --ops fwd_plain,fwd_stats,bwd_data --out /tmp/ref.pt > $O/r3l_pw0.log 2>&1 || exit $?
timeout -k 10 200 python tools/conv_bench.py --ops fwd_plain,fwd_stats,bwd_data --check /tmp/ref.pt > $O/r3l_pw1.log 2>&1 || exit $?
for want in 1024 2048 512; do for rb in 8 16; do
timeout -k 10 200 env ROD_DW_WANT=$want ROD_DW_RBMIN=$rb python tools/dwfused_bench.py > $O/r3l_dwf_${want}_${rb}.log 2>&1 || exit $?
done; done
grep -h TOTAL $O/r3l_dwf_*.log
for wt in 2048 1024 512; do
timeout -k 10 300 env ROD_WG_TARGET=$wt python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --kernel-steps 0 > $O/r3l_wg$wt.log 2>&1 || exit $?
done
grep -h '^{' $O/r3l_wg*.log | cut -c1-120
