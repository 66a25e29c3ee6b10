# Scratch GPU command of the last session (run as: gpurun -- 'bash tools/_cmd.sh'):
# K3 folded into the walk (tools/patches/pc_walk_fold_edge_maps_r04.patch; not kept):
# GPU parity suite, then against the previous sources (old = K3 as its own launch, built as a
# variant from them), alternating.
set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
bash tools/gpu_session.sh r04z2 tests || exit $?
AB_REPS=3 bash tools/ab.sh r04z2 new=default old=$V/libzfft_old.so
