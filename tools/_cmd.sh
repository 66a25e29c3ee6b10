set -u
export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
for v in main np; do
  if [ $v = main ]; then unset ZFFT_LIB_PATH; else export ZFFT_LIB_PATH=pypanadapter_amd/lib/variants/libzfft_$v.so; fi
  for cfg in cfg5 cfg3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_${cfg}_$i -o run -- python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu --no-e2e > $O/${v}_${cfg}_$i.log 2>&1 || exit $?
  python3 -c "
import csv,json
d=json.loads([l for l in open('$O/${v}_${cfg}_$i.log') if l.startswith('{')][-1])
r=[(x['Name'][:28], round(float(x['AverageNs'])/1e6,4)) for x in csv.DictReader(open('$O/${v}_${cfg}_$i/run_kernel_stats.csv')) if 'welch' in x['Name']]
print('$v $cfg', d['ms_per_step'], r, d['parity_checked_frames']['pass'])
"
  done
done
done
