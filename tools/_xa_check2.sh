set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "every_schedule or fused_interior" > gpurun_out/xa_tests.log 2>&1; rc=$?
tail -3 gpurun_out/xa_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --path 4 > gpurun_out/xa_bench.log 2>&1 || { tail -20 gpurun_out/xa_bench.log; exit 1; }
grep '^{' gpurun_out/xa_bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d['roofline']['frac'])"
ZFFT_LIB_PATH=$PWD/pypanadapter_amd/lib/variants/libzfft_stamps.so timeout -k 10 300 python tools/xa_stamps.py 2048
