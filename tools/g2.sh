cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_gred.py -q --timeout=200 -p no:cacheprovider > gpurun_out/g2_tests.log 2>&1; echo "tests rc=$?"
tail -25 gpurun_out/g2_tests.log
bash tools/gpu_run.sh g2 prof
