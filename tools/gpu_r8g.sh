set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -m gpu -k "checkpointing or attention or attn" -x -q --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_bench.py spatialvla_amd/libsvla.so diag/libsvla_dq64.so > $O/attn_ab.txt 2>&1; rc=$?; cat $O/attn_ab.txt | tail -12; [ $rc -ne 0 ] && exit $rc
TAG=r8g_dec bash tools/decode_prof.sh && cat gpurun_out/r8g_dec/r8g_dec_step_breakdown.txt && tail -2 gpurun_out/r8g_dec/decode_prof.json
