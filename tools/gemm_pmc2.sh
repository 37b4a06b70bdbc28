#!/bin/bash
# Our GEMM vs hipBLASLt (torch.matmul) on one shape: kernel trace (hipBLASLt's kernel name carries its tile config)
# and PMC passes (clock from GRBM_GUI_ACTIVE, MFMA busy, fabric bytes, LDS / VALU instruction mix).
# usage: tools/gemm_pmc2.sh TAG M N K [layout]    -> gpurun_out/<TAG>/<M>x<N>x<K>_<arm>_{trace,p1,p2,p3}
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; M=$2; N=$3; K=$4; LAY=${5:-nt}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for arm in svla torch; do
  P="python3 $R/tools/gemm_pmc_one.py $arm $M $N $K 20"
  D=$O/${M}x${N}x${K}${LAY}_${arm}
  SVLA_LAYOUT=$LAY timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $D/trace -o t --output-format csv -- $P > /dev/null || exit $?
  SVLA_LAYOUT=$LAY timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $D/p1 -o p1 --output-format csv -- $P > /dev/null || exit $?
  SVLA_LAYOUT=$LAY timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $D/p2 -o p2 --output-format csv -- $P > /dev/null || exit $?
  SVLA_LAYOUT=$LAY timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $D/p3 -o p3 --output-format csv -- $P > /dev/null || exit $?
  python3 $R/tools/pmc_table.py $D/p1/* $D/p2/* $D/p3/* $D/trace/* $D/p1 $D/p2 $D/p3 $D/trace > $D.txt 2>&1
done
echo pmc2 done
