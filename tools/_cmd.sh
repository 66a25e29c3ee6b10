# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# the PC head's few-frame tail on zoom 2's tiles: all GPU tests, then one frame end to end at
# zoom 16 and 32, and 64 frames per call at zoom 16.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05z; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for z in 16 32; do
  timeout -k 10 300 python bench.py --zoom $z --frames 64 --steps 5 --warmup 1 --no-cpu --e2e-frames 64 > $OUT/z${z}.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$OUT/z${z}.log') if l.startswith('{')][0]); e=d['end_to_end']; print('z$z one frame', e['single_frame_latency_ms']['p50'], e['single_frame_latency_ms']['p99'], '64 frames', d['ms_per_step'], {k: round(v, 3) for k, v in d['kernels'].items()})"
done
