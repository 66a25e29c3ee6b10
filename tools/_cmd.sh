# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# zoom-4 tiles automatic below 1024 frames: all GPU tests, tiles vs XA at 512 / 768 frames,
# cfg1 (XA at 4096) and the cfg2 headline.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05v; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for F in 512 768; do
  for spec in "tiles:4" "xa:3"; do
    IFS=: read name path <<< "$spec"
    timeout -k 10 300 python bench.py --config cfg1 --frames $F --path $path --steps 20 --warmup 2 --no-cpu --no-e2e > $OUT/F${F}_$name.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$OUT/F${F}_$name.log') if l.startswith('{')][0]); print('F$F $name', d['ms_per_step'], {k: round(v, 3) for k, v in d['kernels'].items()})"
  done
done
for c in cfg1 cfg2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-e2e > $OUT/$c.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$c.log') if l.startswith('{')][0]); print('$c', d['ms_per_step'], d['kernels'])"
done
