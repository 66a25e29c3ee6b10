set -u
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -q --timeout 300 --timeout-method thread > $O/pc_tests.log 2>&1 || { tail -30 $O/pc_tests.log; exit 1; }
tail -3 $O/pc_tests.log
for p in 4; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 3 --no-cpu --no-e2e --path $p > $O/bench_p$p.log 2>&1 || { tail -20 $O/bench_p$p.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_p$p.log') if l.startswith('{')][0]); print('path $p', d['ms_per_step'], d['kernels'], d.get('parity_checked_frames'))"
done
