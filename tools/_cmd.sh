# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# the PC head + XA tail (zoom >= 16): its GPU tests, then zoom 16 / 32 on cfg2's frames, auto
# (head) against XA alone (path 3).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05p; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pc.py tests/test_gpu_parity.py -k "head or auto_schedule or refuses" > $OUT/pytest_head.log 2>&1 || { tail -30 $OUT/pytest_head.log; exit 1; }
tail -3 $OUT/pytest_head.log
for z in 16 32; do
  for spec in "auto:0" "xa:3"; do
    IFS=: read name path <<< "$spec"
    timeout -k 10 300 python bench.py --zoom $z --path $path --steps 20 --warmup 2 --no-cpu --no-e2e > $OUT/z${z}_$name.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$OUT/z${z}_$name.log') if l.startswith('{')][0]); print('z$z $name', d['ms_per_step'], d['kernels'], (d.get('parity_checked_frames') or {}).get('pass'))"
  done
done
