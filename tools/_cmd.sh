set -u
export TMPDIR=/tmp
O=gpurun_out/r03dpp; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
for v in new pp0 orig; do
  if [ $v = new ]; then unset ZFFT_LIB_PATH; else export ZFFT_LIB_PATH=pypanadapter_amd/lib/variants/libzfft_$v.so; fi
  for cfg in cfg2 cfg1 cfg3; do
    timeout -k 10 120 python bench.py --config $cfg --steps 100 --warmup 3 --no-cpu --no-e2e --no-check > $O/${v}_${cfg}_$i.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/${v}_${cfg}_$i.log') if l.startswith('{')][0]); k=d['kernels']; print('$v $cfg', d['ms_per_step'], [round(x,4) for n,x in k.items() if 'welch' in n])"
  done
done
done
