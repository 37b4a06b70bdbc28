set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe4
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/blk4 -o blk --output-format csv -- python3 tools/block_ab.py 1 1 5 > gpurun_out/probe4/block.log 2>&1 || exit 1
python tools/block_trace.py /tmp/blk4 > gpurun_out/probe4/block_breakdown.txt 2>&1
