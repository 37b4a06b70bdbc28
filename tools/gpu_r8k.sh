set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_full4b_gpu.py -m gpu -k "fp8" -x -v -s --timeout 800 --timeout-method thread > $O/pytest4b.txt 2>&1
rc=$?; grep -E "4B fp8 vs|passed|failed|Error" $O/pytest4b.txt | tail -5 | cut -c1-700; exit $rc
