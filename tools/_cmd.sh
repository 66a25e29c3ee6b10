# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# the final-sources session: GPU tests, smoke, the driver's bench line, rocprofv3 kernel
# trace, PMC traffic and SQ counters (stamped into profiles/), every BASELINE config.
set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r05fin6 tests smoke driver prof pmc sq stamp cfgs
