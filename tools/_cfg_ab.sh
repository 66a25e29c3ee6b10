# A/B of library variants on one config: bash tools/_cfg_ab.sh <config> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cfg=$1; shift
for v in default "$@"; do
  if [ $v = default ]; then lp=$PWD/pypanadapter_amd/lib/libzfft.so; else lp=$PWD/pypanadapter_amd/lib/variants/libzfft_$v.so; fi
  ZFFT_LIB_PATH=$lp timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --config $cfg > gpurun_out/cab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/cab_$v.log; exit 1; }
  grep '^{' gpurun_out/cab_$v.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$cfg $v', d['ms_per_step'], d['kernels'])"
done
