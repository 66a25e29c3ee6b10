#!/bin/bash
# waterfall batch-push parity + cfg2/cfg5 bench at HEAD, then scheduler-strategy variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k waterfall -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/wf_tests.log 2>&1; rc=$?
tail -3 gpurun_out/wf_tests.log; [ $rc -eq 0 ] || exit $rc
for c in cfg2 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu > gpurun_out/wf_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/wf_$c.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'], d['roofline']['frac'], d['kernels'])"
done
bash tools/_xa_ab2.sh "$@"
