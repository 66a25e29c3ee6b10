# Scratch GPU command of the last session (run as: gpurun -- 'bash tools/_cmd.sh'):
# K3 rewritten with one wave per frame and side (not kept): GPU parity suite and a
# quick bench for its time.
set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r04x tests quick
