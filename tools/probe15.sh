set -o pipefail
mkdir -p gpurun_out/probe15
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/probe15/pytest_gpu.txt 2>&1; rc=$?; tail -2 gpurun_out/probe15/pytest_gpu.txt; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/probe15/bench.json 2> gpurun_out/probe15/bench.err || exit $?
timeout -k 10 200 python tools/beit_attn_probe.py > gpurun_out/probe15/beit.txt 2>&1
