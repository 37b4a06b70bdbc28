# GEMM A/B: kernel tests, microbenchmark of the product build and variants, barrier stamps.
set -o pipefail
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kt.log 2>&1
for lib in spatialvla_amd/libsvla.so "$@"; do
  echo "== $lib"; SVLA_LIB=$lib timeout -k 10 100 python tools/gemm_bench.py || exit 1
done > gpurun_out/gb.log 2>&1
for d in 12 13 29; do echo "== $d"; SVLA_STAMPS=1 SVLA_LIB=build/diag/libsvla_diag$d.so timeout -k 10 60 python tools/gemm_bench.py || exit 1; done > gpurun_out/stamps.log 2>&1
