cd $GRAFT_REPO_ROOT
for v in "$@"; do
  ZFFT_LIB_PATH=$PWD/pypanadapter_amd/lib/variants/libzfft_$v.so timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu --path 3 > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  grep '^{' gpurun_out/ab_$v.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['kernels'])"
done
