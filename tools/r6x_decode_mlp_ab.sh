set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -k "decode_mlp" -x -q --timeout 200 --timeout-method thread > $O/pytest_decode.txt 2>&1
rc=$?; tail -2 $O/pytest_decode.txt; [ $rc -ne 0 ] && exit $rc
SVLA_LIB=diag/libsvla_dm3.so timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -k "decode_mlp_persistent_bitwise" -x -q --timeout 200 --timeout-method thread > $O/pytest_decode3.txt 2>&1
rc=$?; tail -2 $O/pytest_decode3.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for cfg in "0 spatialvla_amd/libsvla.so" "1 spatialvla_amd/libsvla.so" "1 diag/libsvla_dm3.so"; do
    set -- $cfg
    SVLA_LIB=$2 SVLA_DECODE_MLP_PERSIST=$1 timeout -k 10 300 python -u tools/decode_bench.py --no-uncached > $O/d.json 2> $O/d.err || exit 1
    python -c "import json;d=json.loads(open('$O/d.json').read().strip().splitlines()[-1]);print('persist=$1 $2', d['ms_per_decode_token'])"
  done
done
