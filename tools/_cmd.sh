# Scratch GPU command of the last session (run as: gpurun -- 'bash tools/_cmd.sh'):
# the final-hash stamp session, then the scheduler-strategy A/B (variants from
# tools/build_variants.py).
set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
bash tools/gpu_session.sh r04v pmc sq stamp driver prof sweep || exit $?
AB_REPS=2 bash tools/ab.sh r04u base=default ilp=$V/libzfft_ilp.so mclause=$V/libzfft_mclause.so
