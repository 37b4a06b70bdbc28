#!/bin/bash
# Final-measurement call A: the whole GPU test suite and the bench line (tools/measure_b.sh: traces and PMC).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r5}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || exit $?
head -c 3500 $O/bench.json; echo
