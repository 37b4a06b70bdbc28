set -o pipefail
mkdir -p gpurun_out/probe14
timeout -k 10 300 python tools/beit_attn_probe.py spatialvla_amd/libsvla.so diag/libsvla_bpf2.so diag/libsvla_rs64.so diag/libsvla_rs64wpe2.so diag/libsvla_rs64bpf2.so > gpurun_out/probe14/beit.txt 2>&1 || exit $?
SVLA_LIB=diag/libsvla_rs64.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "attn or attention or beit or zoe or depth" --timeout 200 --timeout-method thread > gpurun_out/probe14/t.txt 2>&1; rc=$?; tail -2 gpurun_out/probe14/t.txt; [ $rc -gt 1 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
P="python3 $GRAFT_REPO_ROOT/tools/beit_attn_probe.py $GRAFT_REPO_ROOT/spatialvla_amd/libsvla.so $GRAFT_REPO_ROOT/diag/libsvla_rs64.so"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $GRAFT_REPO_ROOT/gpurun_out/probe14/p1 -o p1 --output-format csv -- $P > /dev/null || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM -d $GRAFT_REPO_ROOT/gpurun_out/probe14/p2 -o p2 --output-format csv -- $P > /dev/null || exit $?
