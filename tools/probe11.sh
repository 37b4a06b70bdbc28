set -o pipefail
mkdir -p gpurun_out/probe11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/probe11/t.txt 2>&1; rc=$?
tail -3 gpurun_out/probe11/t.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/probe11/dec.json 2> gpurun_out/probe11/dec.err || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode --no-fp8-leg > gpurun_out/probe11/bench.json 2> gpurun_out/probe11/bench.err
