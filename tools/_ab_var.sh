#!/bin/bash
# bench A/B of build variants (variants/libzfft_<name>.so) for one bench argument set:
# tools/_ab_var.sh "<bench args>" name1 name2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
a=$1; shift
for v in default "$@" default "$@"; do
  if [ $v = default ]; then lp=$PWD/pypanadapter_amd/lib/libzfft.so; else lp=$PWD/pypanadapter_amd/lib/variants/libzfft_$v.so; fi
  ZFFT_LIB_PATH=$lp timeout -k 10 200 python bench.py $a --steps 5 --warmup 1 --no-cpu > gpurun_out/abv_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/abv_$v.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['kernels'])"
done
