set -o pipefail
mkdir -p gpurun_out/probe2
for lib in g4s st1 st2; do for s in "1792 2304 2048" "9984 18432 2304"; do
  echo "== $lib $s"; timeout -k 10 60 python tools/gemm_stamps.py diag/libsvla_$lib.so $s | grep blocks || exit 1
done; done > gpurun_out/probe2/stamps3.txt 2>&1
