#!/bin/bash
# A/B of library variants on the GPU box: alternating runs of the quick cfg2 bench.
# usage: tools/ab.sh <tag> <name=libpath|default> ...   (env AB_ARGS: extra bench args, AB_REPS)
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 ${AB_REPS:-2}); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = default ]; then unset ZFFT_LIB_PATH; else export ZFFT_LIB_PATH=$lib; fi
    timeout -k 10 300 python bench.py --steps 100 --warmup 3 --no-cpu --no-e2e --no-check ${AB_ARGS:-} > $OUT/${name}_$rep.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$OUT/${name}_$rep.log') if l.startswith('{')][0]); print('$name', d['ms_per_step'], d['kernels'])"
  done
done
