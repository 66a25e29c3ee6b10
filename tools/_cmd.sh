# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_pc.log 2>&1; rc=$?
tail -3 $O/pytest_pc.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_REPS=3 bash tools/ab.sh r05m_ab k3new=default k3old=$V/libzfft_k3old.so
