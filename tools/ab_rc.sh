# A/B of the recompute forms on one box: ROD_DISABLE=$1 against the defaults, alternating, 2 + 2
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${2:-r6ab}
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-inference --no-fp32-leg --no-tfrecord-leg --no-dp-leg --kernel-steps 0"
for i in 1 2; do
  timeout -k 10 300 env ROD_DISABLE=$1 $B > gpurun_out/${T}_off_$i.log 2>&1 || exit 1
  timeout -k 10 300 $B > gpurun_out/${T}_on_$i.log 2>&1 || exit 1
done
for f in gpurun_out/${T}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
