set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ZFFT_LIB_PATH=$PWD/pypanadapter_amd/lib/variants/libzfft_stamps.so timeout -k 10 120 python -u tools/xa_stamps.py 2048 2>&1 | tee gpurun_out/stamps.log
