#!/bin/bash
# Gemma2 attention forward PMC passes for the 16x16x32 (SVLA_ATTN32=0) and 32x32x16 (=1) kernels:
# tools/attn_pmc32.sh <tag>  -> gpurun_out/<tag>/a{0,1}_{p1,p2}
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-attpmc32}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  export SVLA_ATTN32=$m
  P="python3 $R/tools/attn_one.py gemma2 fwd 10"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/a${m}_trace -o t --output-format csv -- $P > /dev/null || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $O/a${m}_p1 -o p1 --output-format csv -- $P > /dev/null || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $O/a${m}_p2 -o p2 --output-format csv -- $P > /dev/null || exit $?
done
echo pmc done
