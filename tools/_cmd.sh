# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# A/B: odd walk workgroups at s_setprio 1 / 3 against none.
set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
AB_REPS=3 bash tools/ab.sh r05x base=$V/libzfft_base.so wgp1=$V/libzfft_wgp1.so wgp3=$V/libzfft_wgp3.so
