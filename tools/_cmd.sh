set -u
export TMPDIR=/tmp
bash tools/gpu_session.sh r04t tests smoke
