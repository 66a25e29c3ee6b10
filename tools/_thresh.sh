set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/th.log 2>&1 || { echo "fail $*"; tail -3 gpurun_out/th.log; exit 1; }; grep '^{' gpurun_out/th.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], round(d['value']/1e3,1), 'GS/s')"; }
for F in 256 512 1024; do for p in 2 4; do run --frames $F --path $p; done; done
run --config cfg5 --frames 512 --path 2
run --config cfg5 --frames 512 --path 4
run --config cfg5 --frames 2048 --path 4
