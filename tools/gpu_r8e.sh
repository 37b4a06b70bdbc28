set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_full4b_gpu.py tests/test_model_gpu.py -m gpu -k "fp8" -x -v -s --timeout 800 --timeout-method thread > $O/pytest4b.txt 2>&1
rc=$?; grep -E "fp8 ablation qkv\+o\+gate_up\+down|passed|failed|Error" $O/pytest4b.txt | tail -5 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for sites in "qkv,o,gate_up,down" "qkv,o,down"; do
  SVLA_FP8_SITES=$sites timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-decode > $O/bench_$sites.json 2> $O/bench_$sites.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_$sites.json'));print('$sites', 'bf16', d['ms_per_step'], 'fp8', d['fp8']['ms_per_step'], round(d['fp8']['value']/d['value'],4))"
done
