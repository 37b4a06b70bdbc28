set -o pipefail
mkdir -p gpurun_out/probe1
SVLA_VARIANTS=0,2,3 timeout -k 10 200 python tools/gemm_probe.py 9984x4096x2304:nt 8192x4096x2304:nt 9984x2304x2048:nt 7168x2304x2048:nt 9216x2304x2048:nt 9984x2304x9216:nt 8192x2304x9216:nt 9984x9216x2304:nn 9984x2048x2304:nn 4096x2304x9984:tn 2304x2048x9984:tn 9984x18432x2304:nt > gpurun_out/probe1/gemm.txt 2>&1
