set -u
export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
FAST="--min-seconds 0 --no-cpu --no-e2e --no-check"
for v in old new; do
  if [ $v = old ]; then export ZFFT_LIB_PATH=pypanadapter_amd/lib/variants/libzfft_old.so; else unset ZFFT_LIB_PATH; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --steps 2 --warmup 1 $FAST > $O/pmc_$v.log 2>&1 || exit $?
done
for i in 1 2 3; do
for v in old new; do
  if [ $v = old ]; then export ZFFT_LIB_PATH=pypanadapter_amd/lib/variants/libzfft_old.so; else unset ZFFT_LIB_PATH; fi
  timeout -k 10 120 python bench.py --steps 200 --warmup 5 --no-cpu --no-e2e > $O/b_${v}_$i.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/b_${v}_$i.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['kernels'], d['parity_checked_frames']['pass'])"
done
done
