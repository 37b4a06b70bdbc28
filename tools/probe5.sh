set -o pipefail
mkdir -p gpurun_out/probe5
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_full4b_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/probe5/kt.txt 2>&1; rc=$?
tail -3 gpurun_out/probe5/kt.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode --no-fp8-leg > gpurun_out/probe5/bench.json 2> gpurun_out/probe5/bench.err
