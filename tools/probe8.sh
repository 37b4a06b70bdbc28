set -o pipefail
mkdir -p gpurun_out/probe8
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/probe8/t.txt 2>&1; rc=$?
tail -3 gpurun_out/probe8/t.txt
[ $rc -gt 1 ] && exit $rc
for f in 0 1 0 1; do SVLA_DECODE_NORM_FUSED=$f timeout -k 10 300 python -u tools/decode_bench.py >> gpurun_out/probe8/dec_$f.json 2> gpurun_out/probe8/dec_$f.err || exit 1; done
