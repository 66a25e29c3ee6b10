set -u
export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for dt in complex64 complex32; do
  timeout -k 10 200 python bench.py --config cfg5 --in-dtype $dt --steps 20 --warmup 2 --no-cpu --no-e2e > $O/cfg5_$dt.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/cfg5_$dt.log').read().strip().splitlines()[-1]); print('$dt', d['ms_per_step'], d['kernels'], d['parity_checked_frames'])"
done
