#!/bin/bash
# One GPU-box call: GPU tests, GEMM shape microbench vs torch (hipBLASLt yardstick), short bench.
# Usage: tools/gpu_check.sh <tag> [pytest selection]
set -o pipefail
TAG=${1:-r2}
SEL=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.txt
ok $rc || exit $rc
if [ -z "$SKIP_GEMM" ]; then
  timeout -k 10 300 python -u tools/gemm_bench.py > $OUT/gemm_bench.txt 2>&1; rc=$?; echo "gemm_bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err
fi
exit $rc
