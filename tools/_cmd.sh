set -u
TESTK="-x -k fused" bash tools/gpu_session.sh r03h tests_k || exit $?
V=pypanadapter_amd/lib/variants
AB_REPS=2 bash tools/ab.sh r03h_ab base=default fd1=$V/libzfft_fd1.so
