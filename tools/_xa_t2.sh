set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/_xa_t.sh "$@" || exit $?
ZFFT_LIB_PATH=$PWD/pypanadapter_amd/lib/variants/libzfft_stamps.so timeout -k 10 300 python tools/xa_stamps.py 2048
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --path 4 > gpurun_out/xa_bench.log 2>&1 || { tail -20 gpurun_out/xa_bench.log; exit 1; }
grep '^{' gpurun_out/xa_bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d['roofline']['frac'])"
