set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8y
mkdir -p $O
SVLA_ZOE_STREAM_CAPTURE=1 timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_full4b_gpu.py -m gpu -k "decode or predict or greedy" -x -q -W error::UserWarning --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in 0 1; do
  SVLA_ZOE_STREAM_CAPTURE=$v timeout -k 10 300 python -u tools/decode_bench.py --no-uncached > $O/d_$v.json 2> $O/d_$v.err || exit 1
  python -c "import json;d=json.loads(open('$O/d_$v.json').read().strip().splitlines()[-1]);print('capture_zoe=$v', d['ms_prefill_plus_first'], d['ms_total'], d['ms_per_decode_token'])"
done; done
