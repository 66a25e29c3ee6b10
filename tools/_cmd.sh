# Scratch GPU command of the current session (run as: gpurun -- 'bash tools/_cmd.sh').
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05l; mkdir -p $O
FAST="--no-cpu --no-e2e --no-check"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_a -o run -- python3 $R/bench.py --steps 2 --warmup 1 $FAST > $O/pmc_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_b -o run -- python3 $R/bench.py --steps 2 --warmup 1 $FAST > $O/pmc_b.log 2>&1 || exit $?
ls $O/pmc_a $O/pmc_b
