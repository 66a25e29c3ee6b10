# full GPU test suite on the default build, then the A/B bench of the named variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "passed|failed|Error" gpurun_out/t_all.log | head -5
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || { grep -B5 -A25 "^____" gpurun_out/t_all.log | head -60; }
bash tools/_xa_ab2.sh "$@"
