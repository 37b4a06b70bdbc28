set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_fp8_gpu.py tests/test_bench_dist_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
TAG=r8a tools/ab.sh decode 2 "-" "SVLA_DECODE_MLP_COOP=0" "SVLA_DECODE_MLP_PERSIST=0"
