set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; tail -3 $O/smoke.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 3000 $O/bench.json; exit $rc
