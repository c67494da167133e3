set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_fullsize.py tests/test_gpu_eval.py tests/test_gpu_irblock.py tests/test_gpu_detect.py -m gpu -q -x --timeout=500 -p no:cacheprovider > $O/r3q_t.log 2>&1; echo t rc=$?; tail -n 2 $O/r3q_t.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --no-tfrecord-leg --kernel-steps 0 > $O/r3q_b.log 2>&1 || exit $?
grep -h '^{' $O/r3q_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['inference']['value'], d['inference_1080p']['value'])"
