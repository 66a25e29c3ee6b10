# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh'):
# the split DIF Welch for few frames per call: all GPU tests, then single-frame latency at
# zoom 2, 4, 8, 16 on cfg2's frames and the cfg2 headline.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05t; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for z in 2 4 8 16; do
  timeout -k 10 300 python bench.py --zoom $z --frames 64 --steps 5 --warmup 1 --no-cpu --e2e-frames 64 > $OUT/z${z}.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$OUT/z${z}.log') if l.startswith('{')][0]); e=d['end_to_end']; print('z$z', e['single_frame_latency_ms']['p50'], e['single_frame_latency_ms']['p99'], d['ms_per_step'], d['kernels'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $OUT/cfg2.log 2>&1 || exit $?
python3 -c "import json; d=json.loads([l for l in open('$OUT/cfg2.log') if l.startswith('{')][0]); print('cfg2', d['ms_per_step'], d['kernels'])"
