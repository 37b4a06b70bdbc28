#!/bin/bash
# Our GEMM vs hipBLASLt (torch.matmul) on one x @ W^T shape: kernel names + durations (kernel trace), effective clock
# and MFMA busy (SQ/GRBM pass), L2->fabric fetch (FETCH_SIZE pass).  tools/blaslt_cmp.sh M N K [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
M=$1; N=$2; K=$3; T=${4:-cmp}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for arm in svla torch; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d /tmp/${T}_${arm}_kt -o kt --output-format csv -- python3 $R/tools/gemm_pmc_one.py $arm $M $N $K || exit $?
  cp /tmp/${T}_${arm}_kt/*/kt_kernel_stats.csv $O/${arm}_kernel_stats.csv 2>/dev/null || find /tmp/${T}_${arm}_kt -name "*kernel_stats.csv" -exec cp {} $O/${arm}_kernel_stats.csv \;
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/${T}_${arm}_p1 -o p1 --output-format csv -- python3 $R/tools/gemm_pmc_one.py $arm $M $N $K || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d /tmp/${T}_${arm}_p2 -o p2 --output-format csv -- python3 $R/tools/gemm_pmc_one.py $arm $M $N $K || exit $?
  python3 $R/tools/pmc_table.py /tmp/${T}_${arm}_p1 /tmp/${T}_${arm}_p2 $O > $O/${arm}_pmc.txt 2>&1
done
python3 - "$O" <<'PY'
import csv, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*_kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        print(f.split("/")[-1], r["Name"][:400], r["Calls"], r["AverageNs"])
PY
cat $O/svla_pmc.txt $O/torch_pmc.txt
