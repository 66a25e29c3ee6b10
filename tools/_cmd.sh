set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
bash tools/gpu_session.sh r04v pmc sq stamp driver prof sweep || exit $?
AB_REPS=2 bash tools/ab.sh r04u base=default ilp=$V/libzfft_ilp.so mclause=$V/libzfft_mclause.so
