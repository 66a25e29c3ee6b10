# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
AB_REPS=2 bash tools/ab.sh r05d_ab base=default dpp4=$V/libzfft_dpp4.so ko64=$V/libzfft_ko64.so ko128=$V/libzfft_ko128.so ko192=$V/libzfft_ko192.so
