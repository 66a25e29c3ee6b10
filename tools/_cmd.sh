# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "pc4" > $O/pytest_pc4.log 2>&1; rc=$?
tail -15 $O/pytest_pc4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ $rc -eq 0 ] || exit 0
for rep in 1 2; do
  for p in 3 5; do
    timeout -k 10 300 python bench.py --config cfg1 --steps 50 --warmup 2 --no-cpu --no-e2e --path $p > $O/cfg1_p${p}_$rep.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/cfg1_p${p}_$rep.log') if l.startswith('{')][0]); print('cfg1 path $p', d['ms_per_step'], d['kernels'], d.get('parity_checked_frames'))"
  done
done
