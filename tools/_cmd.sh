set -u
export TMPDIR=/tmp
O=gpurun_out/r03r; mkdir -p $O
for fz in 2 3; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$fz -o run -- python3 bench.py --fuse $fz --steps 2 --warmup 1 --min-seconds 0 --no-cpu --no-e2e --no-check > $O/f$fz.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$fz -o run -- python3 bench.py --fuse $fz --steps 2 --warmup 1 --min-seconds 0 --no-cpu --no-e2e --no-check > $O/w$fz.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $O/f$fz $O/w$fz 4096 cfg2 $O/traffic_cfg2_fuse$fz.json complex64 > $O/traffic_fuse$fz.log || exit $?
done
