set -u
export TMPDIR=/tmp
O=gpurun_out/r03fend; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
AB_REPS=3 bash tools/ab.sh r03fend base=default fend0=pypanadapter_amd/lib/variants/libzfft_fend0.so u8=pypanadapter_amd/lib/variants/libzfft_u8.so u16=pypanadapter_amd/lib/variants/libzfft_u16.so
