set -o pipefail
mkdir -p gpurun_out/probe14
timeout -k 10 300 python tools/beit_attn_probe.py spatialvla_amd/libsvla.so diag/libsvla_bpf2.so diag/libsvla_rs64.so diag/libsvla_rs64wpe2.so diag/libsvla_rs64bpf2.so > gpurun_out/probe14/beit.txt 2>&1 || exit $?
SVLA_LIB=diag/libsvla_rs64.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "attn or attention or beit or zoe or depth" --timeout 200 --timeout-method thread > gpurun_out/probe14/t.txt 2>&1; rc=$?; tail -2 gpurun_out/probe14/t.txt; [ $rc -gt 1 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for lib in spatialvla_amd/libsvla.so diag/libsvla_rs64.so; do
  n=$(basename $lib .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $GRAFT_REPO_ROOT/gpurun_out/probe14/p1_$n -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/beit_attn_probe.py $GRAFT_REPO_ROOT/$lib > /dev/null || exit $?
done
