set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_bench_dist_gpu.py -m gpu -x -v --timeout 420 --timeout-method thread 2>&1 | tail -5
