set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/wc.log 2>&1 || { echo "fail $*"; tail -3 gpurun_out/wc.log; exit 1; }; grep '^{' gpurun_out/wc.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], d['kernels'])"; }
run --config cfg3 --welch 1
run --config cfg3 --welch 2
run --config cfg1
run --config cfg1 --path 4
