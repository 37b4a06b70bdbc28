# In-situ A/B of the GEMM dispatch: kernel traces of bench.py under two SVLA_GEMM_VARIANT values, paired per call.
set -o pipefail
export TMPDIR=/tmp
VA=${VA:-4}; VB=${VB:-0}
for v in $VA $VB; do
  SVLA_GEMM_LOG=/tmp/gemm_log.json SVLA_GEMM_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/abp_$v -o t --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abp_$v.out 2> gpurun_out/abp_$v.err || exit 1
done
python tools/ab_trace.py $(find /tmp/abp_$VA -name "*kernel_trace.csv" | head -1) $(find /tmp/abp_$VB -name "*kernel_trace.csv" | head -1) /tmp/gemm_log.json
