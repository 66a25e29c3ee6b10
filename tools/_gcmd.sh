set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider -rf -x -k "every_schedule or fused_interior or batched" > gpurun_out/tx.log 2>&1 || { tail -30 gpurun_out/tx.log; exit 1; }
tail -2 gpurun_out/tx.log
bash tools/gpu_session.sh r01x3 ab || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/sq_xt -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --path 3 > gpurun_out/sq.log 2>&1 || exit 1
python3 tools/sq_counters.py gpurun_out/sq_xt
