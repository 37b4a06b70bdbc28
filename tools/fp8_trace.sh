#!/bin/bash
# Kernel trace of the fp8 training step (bench.py --fp8): tools/fp8_trace.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-f8tr}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o trace --output-format csv -- python3 bench.py --fp8 --steps 3 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err && \
python tools/summarize_profile.py trace /tmp/prof_$TAG $O/$TAG > $O/trace_summary.log 2>&1
