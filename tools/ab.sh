#!/bin/bash
# Same-box A/B driver (one script for what the round-4..7 one-off r*_ab.sh scripts did):
#   TAG=r8a AB_TESTS="tests/test_decode_gpu.py" tools/ab.sh MODE ROUNDS "CFG" ["CFG" ...]
# MODE    decode  tools/decode_bench.py            -> ms per decode token
#         step    bench.py --steps 8 --warmup 2    -> ms per step, Gemma2 block ms
#         block   tools/block_ab.py 1 1 5 (isolated Gemma2 block) -> its summary line
# CFG     space-separated VAR=value assignments applied to the run ("SVLA_LIB=diag/libsvla_x.so SVLA_DECODE_MLP_COOP=0"),
#         "-" for the defaults.  Configurations alternate within each round, so box drift hits every arm alike.
# AB_TESTS (optional) runs first, once per CFG, under the same settings; a failing test stops the script.
# Every GPU step has its own time limit, and the script stops at the first failure (no retries).
set -o pipefail
export TMPDIR=/tmp
MODE=$1; ROUNDS=${2:-2}; shift 2
O=gpurun_out/${TAG:-ab}
mkdir -p "$O"
run_cfg() {  # run_cfg "CFG" cmd... : the command with CFG's variables in its environment
  local cfg=$1; shift
  if [ "$cfg" = "-" ]; then "$@"; else env $cfg "$@"; fi
}
if [ -n "$AB_TESTS" ]; then
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    run_cfg "$cfg" timeout -k 10 600 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
      > "$O/pytest_$i.txt" 2>&1
    rc=$?; echo "[tests] $cfg: $(tail -1 "$O/pytest_$i.txt")"; [ $rc -ne 0 ] && exit $rc
  done
fi
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    f="$O/${MODE}_${i}_$r"
    case $MODE in
      decode)
        run_cfg "$cfg" timeout -k 10 300 python -u tools/decode_bench.py --no-uncached > "$f.json" 2> "$f.err" || exit 1
        python -c "import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);print('[$cfg]', d['ms_per_decode_token'])" ;;
      step)
        run_cfg "$cfg" timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-decode \
          --no-fp8-leg > "$f.json" 2> "$f.err" || exit 1
        python -c "import json;d=json.load(open('$f.json'));print('[$cfg]', d['ms_per_step'], d['gemma2_block']['ms_fwd_bwd'])" ;;
      block)
        run_cfg "$cfg" timeout -k 10 300 python -u tools/block_ab.py 1 1 5 > "$f.txt" 2>&1 || exit 1
        echo "[$cfg] $(tail -1 "$f.txt")" ;;
      *) echo "unknown mode $MODE"; exit 2 ;;
    esac
  done
done
