set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe3
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/probe3/kt.txt 2>&1; rc=$?
tail -3 gpurun_out/probe3/kt.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/epi_ab.py > gpurun_out/probe3/epi_ab.txt 2>&1 || exit 1
timeout -k 10 200 python tools/gemm_bench.py lm_head > gpurun_out/probe3/lm.txt 2>&1 || exit 1
