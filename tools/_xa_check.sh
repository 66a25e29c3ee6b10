set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "every_schedule or fused_interior" > gpurun_out/xa_tests.log 2>&1; rc=$?
tail -5 gpurun_out/xa_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --path 4 > gpurun_out/xa_bench.log 2>&1 || { tail -20 gpurun_out/xa_bench.log; exit 1; }
grep '^{' gpurun_out/xa_bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d['roofline']['frac'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/sq_xa -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --path 4 > gpurun_out/sq.log 2>&1 || { tail -5 gpurun_out/sq.log; exit 1; }
python3 tools/sq_counters.py gpurun_out/sq_xa
