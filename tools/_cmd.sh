set -u
bash tools/gpu_session.sh r03j tests || exit $?
V=pypanadapter_amd/lib/variants
AB_REPS=3 bash tools/ab.sh r03j_ab defer=default nodefer=$V/libzfft_nodefer.so
