#!/bin/bash
# PMC passes on one GEMM shape, our kernel vs hipBLASLt: tools/gemm_pmc.sh M N K
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
M=${1:-8192}; N=${2:-8192}; K=${3:-8192}
timeout -s KILL 60 rocprofv3 -L > $O/list.txt 2>&1 || true
for arm in svla torch; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/${arm}_p1 -o p1 --output-format csv -- python3 $R/tools/gemm_pmc_one.py $arm $M $N $K || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d $O/${arm}_p2 -o p2 --output-format csv -- python3 $R/tools/gemm_pmc_one.py $arm $M $N $K || exit $?
done
echo pmc done
