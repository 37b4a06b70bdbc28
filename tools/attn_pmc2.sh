#!/bin/bash
# Gemma2 attention fwd/bwd PMC passes only (busy / wait / LDS counters): tools/attn_pmc2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-attpmc2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for what in fwd bwd; do
  P="python3 $R/tools/attn_one.py gemma2 $what 10"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $O/${what}_p1 -o p1 --output-format csv -- $P > /dev/null || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $O/${what}_p2 -o p2 --output-format csv -- $P > /dev/null || exit $?
done
echo pmc done
