set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "passed|failed|Error" gpurun_out/t_all.log | head -5
[ $rc -le 1 ] || exit $rc
bash tools/_xa_ab2.sh "$@"
