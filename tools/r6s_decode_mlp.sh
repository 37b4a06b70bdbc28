set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6s}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_decode.txt 2>&1
rc=$?; tail -3 $O/pytest_decode.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in 0 1; do
  SVLA_DECODE_MLP_PERSIST=$v timeout -k 10 300 python -u tools/decode_bench.py --no-uncached > $O/decode_${v}_$r.json 2> $O/decode_${v}_$r.err || exit 1
  python -c "import json;d=json.loads(open('$O/decode_${v}_$r.json').read().strip().splitlines()[-1]);print('persist=$v', {k: v for k, v in d.items() if 'ms' in k})"
done; done
