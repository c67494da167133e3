cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_abi.py tests/test_gpu_dp_equiv.py "tests/test_gpu_train.py::test_all_mode_step_matches_oracle" -s > gpurun_out/g1.log 2>&1
rc=$?; tail -30 gpurun_out/g1.log; exit $rc
