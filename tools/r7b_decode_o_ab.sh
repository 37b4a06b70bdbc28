set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r7b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_decode.txt 2>&1
rc=$?; tail -2 $O/pytest_decode.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for cfg in "0 0" "1 0" "1 1"; do
    set -- $cfg
    SVLA_DECODE_MLP_PERSIST=$1 SVLA_DECODE_O_FUSED=$2 timeout -k 10 300 python -u tools/decode_bench.py --no-uncached > $O/d.json 2> $O/d.err || exit 1
    python -c "import json;d=json.loads(open('$O/d.json').read().strip().splitlines()[-1]);print('persist=$1 o_fused=$2', d['ms_per_decode_token'])"
  done
done
