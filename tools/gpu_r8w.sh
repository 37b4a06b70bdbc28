set -o pipefail
export TMPDIR=/tmp
for shp in "18464 3072 1024" "18464 1024 4096" "18464 4096 1024" "9984 18432 2304"; do
  echo "== $shp"
  timeout -k 10 120 python -u tools/gemm_stamps.py diag/libsvla_stamps.so $shp 2>&1 | grep -v amdgpu.ids || exit 1
done
