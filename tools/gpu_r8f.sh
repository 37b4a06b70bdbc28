set -o pipefail
export TMPDIR=/tmp
bash tools/fp8_trace.sh r8f_f8 && head -60 gpurun_out/r8f_f8/r8f_f8_step_breakdown.txt
