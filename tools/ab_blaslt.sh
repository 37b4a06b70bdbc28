# In-situ A/B: GEMM dispatch with (variant 0) and without (variant 5) the hipBLASLt route for plain TN stores.
set -o pipefail
for r in 1 2; do for v in 5 0; do
  SVLA_GEMM_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/abl_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abl_${v}_$r.json'));print('variant=$v', d['ms_per_step'], d['final_loss'], d['gemma2_block']['ms_fwd_bwd'])"
done; done
