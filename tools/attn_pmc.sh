#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the attention kernels at the training shapes:
# tools/attn_pmc.sh <outdir-tag>   -> gpurun_out/<tag>/{trace,p1..p4}
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-attpmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shp in gemma2 siglip; do
  for what in fwd bwd; do
    P="python3 $R/tools/attn_one.py $shp $what 10"
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/${shp}_${what}_trace -o t --output-format csv -- $P > /dev/null || exit $?
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $O/${shp}_${what}_p1 -o p1 --output-format csv -- $P > /dev/null || exit $?
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $O/${shp}_${what}_p2 -o p2 --output-format csv -- $P > /dev/null || exit $?
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/${shp}_${what}_p3 -o p3 --output-format csv -- $P > /dev/null || exit $?
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $O/${shp}_${what}_p4 -o p4 --output-format csv -- $P > /dev/null || exit $?
  done
done
echo pmc done
