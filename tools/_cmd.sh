set -u
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -v --timeout 300 --timeout-method thread > $O/pc_tests.log 2>&1; rc=$?
tail -30 $O/pc_tests.log
exit $rc
