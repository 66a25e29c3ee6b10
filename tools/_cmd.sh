set -u
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 900 python tools/sweep_schedule.py $O/sweep_schedule.json > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
tail -3 $O/sweep.log
