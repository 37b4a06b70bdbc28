set -o pipefail
for r in 1 2; do for v in 4 0; do
  SVLA_GEMM_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ab_v${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_v${v}_$r.json'));print('v$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['gemma2_block']['ms_fwd_bwd'])"
done; done
