set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r04o tests smoke pmc sq stamp driver prof cfgs pmc5 sweep
