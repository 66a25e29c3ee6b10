set -u
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/r04m
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04m/pc.log 2>&1 || { tail -20 gpurun_out/r04m/pc.log; exit 1; }
tail -2 gpurun_out/r04m/pc.log
bash tools/gpu_session.sh r04m pmc sq stamp driver prof || exit $?
O=gpurun_out/r04m
FAST="--no-cpu --no-e2e --no-check"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc4_fetch -o run -- python3 $R/bench.py --path 4 --steps 2 --warmup 1 $FAST > $O/pmc4_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc4_write -o run -- python3 $R/bench.py --path 4 --steps 2 --warmup 1 $FAST > $O/pmc4_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $O/pmc4_fetch $O/pmc4_write 4096 cfg2 $O/traffic_cfg2_path4.json complex64 > $O/traffic4.log 2>&1 || exit $?
tail -20 $O/traffic4.log
