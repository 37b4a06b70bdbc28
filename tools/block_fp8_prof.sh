#!/bin/bash
# Kernel breakdown of one Gemma2 layer fwd+bwd (tools/block_ab.py profile mode) in bf16 and with the fp8 projections,
# on the same box: tools/block_fp8_prof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-blkf8}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/blk16 -o blk --output-format csv -- python3 $R/tools/block_ab.py 1 1 5 > $O/bf16.log 2>&1 && \
python3 $R/tools/block_trace.py /tmp/blk16 > $O/bf16_breakdown.txt && \
SVLA_BLOCK_FP8=1 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/blk8 -o blk --output-format csv -- python3 $R/tools/block_ab.py 1 1 5 > $O/fp8.log 2>&1 && \
python3 $R/tools/block_trace.py /tmp/blk8 > $O/fp8_breakdown.txt
rc=$?
tail -1 $O/bf16_breakdown.txt $O/fp8_breakdown.txt; grep "fwd+bwd" $O/bf16.log $O/fp8.log
exit $rc
