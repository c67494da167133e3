set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -q -x --timeout=300 --timeout-method thread -p no:cacheprovider > $O/r3c2_t.log 2>&1 || { tail -n 30 $O/r3c2_t.log; exit 1; }
tail -n 1 $O/r3c2_t.log
for cfg in "ROD_SLAB_VEC=0" "ROD_X=1" "ROD_SLAB_VEC=0" "ROD_X=1"; do
env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --no-tfrecord-leg --no-inference --no-inference-1080 --kernel-steps 0 > $O/r3e_1.log 2>&1 || { tail -n 20 $O/r3e_1.log; exit 1; }
echo "$cfg $(grep -h '^{' $O/r3e_1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
