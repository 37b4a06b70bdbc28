set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; grep -E "drift guard" $O/pytest.txt; exit $rc
