set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_full4b_gpu.py -m gpu -k "fp8" -x -v -s --timeout 800 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "fp8 ablation|passed|failed|Error" $O/pytest.txt | tail -20; [ $rc -ne 0 ] && exit $rc
bash tools/fp8_trace.sh r8b_f8 && head -45 gpurun_out/r8b_f8/r8b_f8_step_breakdown.txt
