# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05a
timeout -k 10 300 env ZFFT_LIB_PATH=pypanadapter_amd/lib/variants/libzfft_stamps.so python tools/pc_stamps.py 4096 > gpurun_out/r05a/stamps.log 2>&1 || exit $?
cat gpurun_out/r05a/stamps.log
bash tools/gpu_session.sh r05a quick || exit $?
TESTK="tests/test_gpu_pc.py tests/test_gpu_parity.py" bash tools/gpu_session.sh r05a tests_k
