set -o pipefail
mkdir -p gpurun_out/probe13
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/probe13/t.txt 2>&1; rc=$?
tail -3 gpurun_out/probe13/t.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/gemm_epi_bench.py > gpurun_out/probe13/epi.txt 2>&1
SVLA_VARIANTS=0,3 timeout -k 10 200 python tools/gemm_probe.py 416x2304x265408:nn 265344x2304x416:tn > gpurun_out/probe13/lmbwd.txt 2>&1
