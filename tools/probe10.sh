set -o pipefail
mkdir -p gpurun_out/probe10
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "tiny or softcap or gelu_rows" > gpurun_out/probe10/t.txt 2>&1; rc=$?
tail -3 gpurun_out/probe10/t.txt
[ $rc -gt 1 ] && exit $rc
SVLA_VARIANTS=0,1,9 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/probe10/pfg.txt 2>&1
