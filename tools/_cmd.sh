# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
TESTK="tests/test_render.py tests/test_gpu_parity.py" bash tools/gpu_session.sh r06g tests_k || exit $?
mkdir -p gpurun_out/r06g
timeout -k 10 300 python -c "
import json, torch, bench
print(json.dumps(bench.display_timing(torch.device('cuda:0')), indent=1))" > gpurun_out/r06g/display.log 2>&1; cat gpurun_out/r06g/display.log
