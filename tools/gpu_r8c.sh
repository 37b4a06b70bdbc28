set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for u in 1 2 4 8; do SVLA_QUANT_MX_ITEMS=$u timeout -k 10 120 python -u tools/quant_bench.py || exit 1; done
