# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# zoom 2 as PC tiles in XA's factorisation: the band-edge row errors of tiles / XA / blocked,
# all GPU tests, then tiles vs XA vs the blocked passes at 1 ... 2048 frames of cfg2's length,
# one frame end to end.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05y; mkdir -p $OUT
timeout -k 10 300 python tools/dbg/pc2_formats_diag.py > $OUT/pc2_formats_diag.log 2>&1 || { tail -20 $OUT/pc2_formats_diag.log; exit 1; }
grep -E "^complex" $OUT/pc2_formats_diag.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for F in 1 64 384 1024 2048; do
  for spec in "tiles:4" "xa:3" "blocked:1"; do
    IFS=: read name path <<< "$spec"
    if [ $name = blocked ] && [ $F -gt 384 ]; then continue; fi
    timeout -k 10 300 python bench.py --zoom 2 --frames $F --path $path --steps 20 --warmup 2 --no-cpu --no-e2e > $OUT/F${F}_$name.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$OUT/F${F}_$name.log') if l.startswith('{')][0]); print('F$F $name', d['ms_per_step'], {k: round(v, 3) for k, v in d['kernels'].items()}, (d.get('parity_checked_frames') or {}).get('pass'))"
  done
done
timeout -k 10 300 python bench.py --zoom 2 --frames 64 --steps 5 --warmup 1 --no-cpu --e2e-frames 64 > $OUT/z2_e2e.log 2>&1 || exit $?
python3 -c "import json; d=json.loads([l for l in open('$OUT/z2_e2e.log') if l.startswith('{')][0]); print('z2 one frame', d['end_to_end']['single_frame_latency_ms'])"
