set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for cfg in "ROD_X=1" "ROD_WG_MINROWS=64" "ROD_WG_MINROWS=256" "ROD_X=1" "ROD_WG_MINROWS=64" "ROD_WG_MINROWS=256"; do
env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --no-tfrecord-leg --no-inference --no-inference-1080 --kernel-steps 0 > $O/r3e_1.log 2>&1 || { tail -n 20 $O/r3e_1.log; exit 1; }
echo "$cfg $(grep -h '^{' $O/r3e_1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
