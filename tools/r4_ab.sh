#!/bin/bash
# Round-4 A/B of the in-tree build against ab/lib_prev.so (the previous commit's library): norm passes, attention
# (plus optional variant libs), greedy decode (prev / new / prev), then the affected GPU tests (AB_TESTS).
# usage: bash tools/r4_ab.sh [variant.so ...]
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
timeout -k 10 300 python -u tools/norm_ab.py ab/lib_prev.so spatialvla_amd/libsvla.so > $O/norm_ab.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/attn_bench.py ab/lib_prev.so spatialvla_amd/libsvla.so "$@" > $O/attn.txt 2>&1 || exit $?
for arm in prev new prev2; do
  lib=ab/lib_prev.so; [ $arm = new ] && lib=spatialvla_amd/libsvla.so
  SVLA_LIB=$lib timeout -k 10 300 python -u tools/decode_bench.py --reps 3 --no-uncached > $O/decode_$arm.json 2> $O/decode_$arm.err || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${AB_TESTS:-tests/test_decode_gpu.py} \
  -s > $O/tests.txt 2>&1
