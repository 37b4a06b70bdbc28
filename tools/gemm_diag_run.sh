# Run the GEMM microbenchmark against each diagnostic build (see tools/gemm_diag.sh).
set -o pipefail
for d in 0 4 5 6 1 2; do
  if [ $d = 0 ]; then lib=spatialvla_amd/libsvla.so; else lib=build/diag/libsvla_diag$d.so; fi
  echo "== diag $d"
  SVLA_LIB=$lib timeout -k 10 120 python tools/gemm_bench.py "$@" || exit 1
done
