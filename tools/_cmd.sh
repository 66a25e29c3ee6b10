# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r05j tests smoke driver
