# Scratch GPU command of the last session (run as: gpurun -- 'bash tools/_cmd.sh'):
# timing-only knockouts of K3 (tools/patches/pc_edge_knockouts_r04.patch, ZFFT_DIAG builds from
# tools/build_variants.py: results wrong by design): no input loads (64), no V loads (256), no
# output read-modify-write (128), all three (448).
set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
AB_REPS=2 bash tools/ab.sh r04y base=default ek0=$V/libzfft_ek0.so ekx=$V/libzfft_ekx.so ekv=$V/libzfft_ekv.so eko=$V/libzfft_eko.so ekall=$V/libzfft_ekall.so
