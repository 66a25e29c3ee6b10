# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# cfg5 PMC traffic (complex64, complex32) at the final sources, and the schedule sweep.
set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r05fin6b pmc5
