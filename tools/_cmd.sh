set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/clk
timeout -k 10 120 tools/ubench/valu_rate > gpurun_out/clk/valu_rate.log 2>&1 || exit $?
timeout -k 10 60 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/clk/vr -o run -- tools/ubench/valu_rate > /dev/null 2>&1 || exit $?
timeout -k 10 60 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/clk/sp -o run -- tools/ubench/stream_pattern 3 > gpurun_out/clk/sp.log 2>&1 || exit $?
cat gpurun_out/clk/valu_rate.log
