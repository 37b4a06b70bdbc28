set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6k}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/blk -o blk --output-format csv -- python3 tools/block_ab.py 1 1 5 > $O/block.log 2>&1 || exit 1
python tools/block_trace.py /tmp/blk > $O/block_breakdown.txt 2>&1
cat $O/block_breakdown.txt
