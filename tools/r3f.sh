set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for cfg in "ROD_DWF_C2=1 ROD_DWF_RING=6" "ROD_DWF_RING=6"; do
env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_dwfused.py -m gpu -q -x --timeout=120 --timeout-method thread -p no:cacheprovider > $O/r3c2_t.log 2>&1 || { tail -n 30 $O/r3c2_t.log; exit 1; }
tail -n 1 $O/r3c2_t.log
done
timeout -k 10 200 python tools/dwfused_bench.py > $O/r3c2_a.log 2>&1 || exit $?
ROD_DWF_C2=1 timeout -k 10 200 python tools/dwfused_bench.py > $O/r3c2_b.log 2>&1 || exit $?
ROD_DWF_C2=1 ROD_DWF_RING=6 timeout -k 10 200 python tools/dwfused_bench.py > $O/r3c2_c.log 2>&1 || exit $?
ROD_DWF_RING=6 timeout -k 10 200 python tools/dwfused_bench.py > $O/r3c2_d.log 2>&1 || exit $?
for f in a b c d; do grep -v '^/opt' $O/r3c2_$f.log | awk '{print $1, $2, $6}' > $O/r3c2_$f.s; done
paste $O/r3c2_a.s $O/r3c2_b.s $O/r3c2_c.s $O/r3c2_d.s
