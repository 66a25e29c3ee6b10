# Scratch GPU command of the last session (run as: gpurun -- 'bash tools/_cmd.sh'):
# every BASELINE config at the final sources, and the driver's bench line on the same box.
set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r04fin driver cfgs
