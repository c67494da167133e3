cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for L in librod_old.so librod.so; do
ROD_LIB=$PWD/road-object-detection-for-bdd100k_amd/lib/$L timeout -k 10 300 python -m pytest tests/test_gpu_train.py -q -x -k "all_mode_step" --timeout=200 -p no:cacheprovider 2>&1 | grep -E "passed|failed|AssertionError: \[" | cut -c1-300
done
