#!/bin/bash
# Round-4 iteration call: the GPU tests touched by the last change, the GEMM A/Bs and the isolated block trace.
# Each GPU step has its own time limit; a crash or timeout stops the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4q}
mkdir -p $O
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -gt 1 ]; then echo "[$name] stopping: crash or timeout"; exit $rc; fi
  return 0
}
if [ -n "$TESTS" ]; then
  step pytest 600 python -u -m pytest tests -m gpu -k "$TESTS" -x -v --timeout 500 --timeout-method thread > $O/t.txt 2>&1
  tail -4 $O/t.txt
  cp gpurun_out/parity/*.json $O/ 2>/dev/null
fi
if [ -n "$AB_LIB" ]; then
  step gemm_ab 300 python -u tools/gemm_ab.py spatialvla_amd/libsvla.so $AB_LIB $AB_SHAPES > $O/gemm_ab.txt 2>&1
  cat $O/gemm_ab.txt
fi
if [ -n "$VARIANTS" ]; then
  SVLA_VARIANTS=$VARIANTS step gemm_bench 300 python -u tools/gemm_bench.py $AB_SHAPES > $O/gemm_bench.txt 2>&1
  cat $O/gemm_bench.txt
fi
if [ -n "$BLOCK" ]; then
  step block 300 rocprofv3 --kernel-trace -d /tmp/blk_q -o blk --output-format csv -- python3 tools/block_ab.py 1 1 5 > $O/block.log 2>&1
  python tools/block_trace.py /tmp/blk_q > $O/block_breakdown.txt 2>&1
  cat $O/block_breakdown.txt
fi
