#!/bin/bash
# Every BASELINE config and input format at HEAD, one bench line each (no CPU leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/cfgs
for spec in "cfg1 complex64" "cfg3 complex64" "cfg5 complex64" "cfg5 complex32" "cfg2 complex32" "cfg2 cu8"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --in-dtype $2 --steps 5 --warmup 1 --no-cpu > gpurun_out/cfgs/$1_$2.log 2>&1 || { echo "$spec failed"; tail -5 gpurun_out/cfgs/$1_$2.log; exit 1; }
  grep '^{' gpurun_out/cfgs/$1_$2.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$1 $2', d['config']['frames_per_rank'], d['ms_per_step'], round(d['value']/1e3,1), 'GS/s frac', d['roofline']['frac'], d['kernels'])"
done
