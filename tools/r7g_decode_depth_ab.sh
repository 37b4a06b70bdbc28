set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r7g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_decode.txt 2>&1
rc=$?; tail -1 $O/pytest_decode.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for L in spatialvla_amd/libsvla.so diag/libsvla_dd2.so; do
    SVLA_LIB=$L timeout -k 10 300 python -u tools/decode_bench.py --no-uncached > $O/d.json 2> $O/d.err || exit 1
    python -c "import json;d=json.loads(open('$O/d.json').read().strip().splitlines()[-1]);print('$L', d['ms_per_decode_token'])"
  done
done
