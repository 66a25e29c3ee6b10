#!/bin/bash
# rocprofv3 kernel stats of the cfg3 and cfg5 benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in cfg3 cfg5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_$c" -o run -- python3 "$PWD/bench.py" --config $c --steps 5 --warmup 1 --no-cpu > gpurun_out/prof_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/prof_$c.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'], d['kernels'])"
done
