# In-situ A/B of two libsvla builds: kernel traces of bench.py, paired per GEMM call (tools/ab_trace.py).
set -o pipefail
export TMPDIR=/tmp
LA=${LA:-diag/libsvla_old.so}; LB=${LB:-spatialvla_amd/libsvla.so}
i=0
for lib in $LA $LB; do
  i=$((i+1))
  SVLA_LIB=$lib SVLA_GEMM_LOG=/tmp/gemm_log.json timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/abl_$i -o t --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-fp8-leg > gpurun_out/abl_$i.out 2> gpurun_out/abl_$i.err || exit 1
done
python tools/ab_trace.py $(find /tmp/abl_1 -name "*kernel_trace.csv" | head -1) $(find /tmp/abl_2 -name "*kernel_trace.csv" | head -1) /tmp/gemm_log.json > gpurun_out/ab_lib.txt 2>&1
