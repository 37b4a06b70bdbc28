#!/bin/bash
# Kernel traces of the training step or the isolated Gemma2 block (what r6k_block_trace.sh / r6o_step_gaps.sh did):
#   TAG=r8a tools/trace.sh step|block
# step:  rocprofv3 --kernel-trace --stats over bench.py (3 steps) -> gpurun_out/$TAG/${TAG}_step_breakdown.txt (+ gaps)
# block: rocprofv3 --kernel-trace over tools/block_ab.py -> gpurun_out/$TAG/block_breakdown.txt
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-trace}
O=gpurun_out/$TAG
mkdir -p "$O"
case $1 in
  step)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_s -o trace --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-fp8-leg > "$O/bench_prof.json" \
      2> "$O/bench_prof.err" || exit 1
    python tools/summarize_profile.py trace /tmp/prof_s "$O/$TAG" > "$O/trace_summary.log" 2>&1
    head -20 "$O/${TAG}_step_breakdown.txt" ;;
  block)
    timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/blk -o blk --output-format csv -- \
      python3 tools/block_ab.py 1 1 5 > "$O/block.log" 2>&1 || exit 1
    python tools/block_trace.py /tmp/blk > "$O/block_breakdown.txt" 2>&1
    cat "$O/block_breakdown.txt" ;;
  *) echo "usage: tools/trace.sh step|block"; exit 2 ;;
esac
