set -u
export TMPDIR=/tmp
O=gpurun_out/r03blk; mkdir -p $O
timeout -k 10 300 python3 tools/dbg/single_frame_blocks.py > $O/blk.log 2>&1 || { tail -5 $O/blk.log; exit 1; }
cat $O/blk.log
