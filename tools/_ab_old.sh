#!/bin/bash
# GPU tests at HEAD, then bench A/B against the previous build (variants/libzfft_old.so) for
# each quoted argument set, e.g. tools/_ab_old.sh "--config cfg3" "--config cfg5"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
k=0
for a in "$@"; do
  k=$((k + 1))
  for v in new old new old; do
    if [ $v = new ]; then lp=$PWD/pypanadapter_amd/lib/libzfft.so; else lp=$PWD/pypanadapter_amd/lib/variants/libzfft_old.so; fi
    ZFFT_LIB_PATH=$lp timeout -k 10 200 python bench.py $a --steps 5 --warmup 1 --no-cpu > gpurun_out/abo_${k}_$v.log 2>&1 || exit $?
    grep '^{' gpurun_out/abo_${k}_$v.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$a $v', d['ms_per_step'], d['kernels'])"
  done
done
