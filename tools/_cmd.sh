# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
V=pypanadapter_amd/lib/variants
O=gpurun_out/r05g; mkdir -p $O
run() {  # name lib path
  if [ "$2" = default ]; then unset ZFFT_LIB_PATH; else export ZFFT_LIB_PATH=$2; fi
  timeout -k 10 300 python bench.py --steps 100 --warmup 3 --no-cpu --no-e2e --no-check --path $3 > $O/$1.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/$1.log') if l.startswith('{')][0]); print('$1', d['ms_per_step'], d['kernels'])"
}
for rep in 1 2; do
  run p5_$rep default 5
  run p6_$rep default 6
  run p6cp1_$rep $V/libzfft_sp_cp1.so 6
  run p6cp2_$rep $V/libzfft_sp_cp2.so 6
  run p6dppcp2_$rep $V/libzfft_sp_dpp4cp2.so 6
done
run p6ko16 $V/libzfft_ko16.so 6
run p6ko7 $V/libzfft_ko7.so 6
run p5ko16 $V/libzfft_ko16.so 5
run p5ko7 $V/libzfft_ko7.so 5
