set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8o
mkdir -p $O
timeout -k 10 300 python -u tools/zoe_step.py 5 2>&1 | grep predict_depth
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/zt -o zt --output-format csv -- python3 tools/zoe_step.py 5 > $O/zt.log 2>&1 || exit 1
python tools/kernel_table.py /tmp/zt 7 > $O/zoe_kernels.txt; cat $O/zoe_kernels.txt
