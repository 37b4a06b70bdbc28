set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_g
for v in 0 3; do
for ctr in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT" "SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr"; do
  tag=$(echo $ctr | cut -c1-12 | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d $R/gpurun_out/pmc_g/v$v/$tag -o run --output-format csv -- python3 $R/tools/gemm_one.py $v "square 8k" 5 > $R/gpurun_out/pmc_g/log_${v}_$tag.txt 2>&1 || exit 1
done
done
