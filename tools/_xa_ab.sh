set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "every_schedule or fused_interior" > gpurun_out/xa_tests.log 2>&1; rc=$?
tail -3 gpurun_out/xa_tests.log
[ $rc -le 1 ] || exit $rc
for v in default "$@"; do
  if [ $v = default ]; then lp=$PWD/pypanadapter_amd/lib/libzfft.so; else lp=$PWD/pypanadapter_amd/lib/variants/libzfft_$v.so; fi
  ZFFT_LIB_PATH=$lp timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --path 4 > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  grep '^{' gpurun_out/ab_$v.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['kernels'])"
done
ZFFT_LIB_PATH=$PWD/pypanadapter_amd/lib/variants/libzfft_stamps.so timeout -k 10 300 python tools/xa_stamps.py 2048
