set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in default "$@"; do
  if [ $v = default ]; then lp=$PWD/pypanadapter_amd/lib/libzfft.so; else lp=$PWD/pypanadapter_amd/lib/variants/libzfft_$v.so; fi
  ZFFT_LIB_PATH=$lp timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "every_schedule or fused_interior" > gpurun_out/t_$v.log 2>&1; rc=$?
  echo "== $v rc=$rc"; grep -E "passed|failed|AssertionError" gpurun_out/t_$v.log | head -6
  [ $rc -le 1 ] || exit $rc
done
