#!/bin/bash
# Whole-step A/B of one environment switch, alternating runs of bench.py: tools/ab_env.sh VAR [rounds] [off] [on]
# (e.g. SVLA_ZOE_STREAM, SVLA_WGRAD_STREAM; values default to 0 / 1); prints ms_per_step and the block time.
set -o pipefail
VAR=$1; N=${2:-2}; V0=${3:-0}; V1=${4:-1}
mkdir -p gpurun_out/ab_env
for r in $(seq 1 $N); do for v in $V0 $V1; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ab_env/${VAR}_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_env/${VAR}_${v}_$r.json'));print('$VAR=$v', d['ms_per_step'], d['gemma2_block']['ms_fwd_bwd'], flush=True)"
done; done
