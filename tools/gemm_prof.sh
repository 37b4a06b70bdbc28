# Kernel trace of bench.py with the GEMM call log -> per-shape GEMM table (tools/gemm_table.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SVLA_GEMM_LOG=/tmp/gemm_log.json timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gp -o t --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/gp.out 2> gpurun_out/gp.err || exit 1
python tools/gemm_table.py $(find /tmp/gp -name "*kernel_trace.csv" | head -1) /tmp/gemm_log.json
