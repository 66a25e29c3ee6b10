# Scratch GPU command of the last session (run as: gpurun -- 'bash tools/_cmd.sh'):
# the final confirmation at the round's last commit: GPU parity suite, smoke, the driver's
# own bench line.
set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r04w tests smoke driver
