set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6z}
mkdir -p $O
for L in diag/libsvla_dmg32.so diag/libsvla_dmg64.so diag/libsvla_dmb1g16.so; do
  SVLA_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -k "decode_mlp_persistent_bitwise" -x -q --timeout 200 --timeout-method thread > $O/pytest_$(basename $L).txt 2>&1
  rc=$?; tail -1 $O/pytest_$(basename $L).txt; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for cfg in "0 spatialvla_amd/libsvla.so" "1 spatialvla_amd/libsvla.so" "1 diag/libsvla_dmg32.so" "1 diag/libsvla_dmg64.so" "1 diag/libsvla_dmb1g16.so"; do
    set -- $cfg
    SVLA_LIB=$2 SVLA_DECODE_MLP_PERSIST=$1 timeout -k 10 300 python -u tools/decode_bench.py --no-uncached > $O/d.json 2> $O/d.err || exit 1
    python -c "import json;d=json.loads(open('$O/d.json').read().strip().splitlines()[-1]);print('persist=$1 $2', d['ms_per_decode_token'])"
  done
done
