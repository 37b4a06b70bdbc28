# Build GEMM schedule variants (SVLA_PP_PRIO) into build/var/ for A/B timing with tools/gemm_bench.py.
set -e
cd "$(dirname "$0")/../spatialvla_amd/csrc"
mkdir -p ../../build/var
for v in "$@"; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast $v -c gemm.hip -o ../../build/var/gemm.o
  name=$(echo "$v" | tr -c 'A-Za-z0-9' '_')
  hipcc -shared -fPIC --offload-arch=gfx950 ../../build/obj/runtime.o ../../build/var/gemm.o ../../build/obj/attention.o \
    ../../build/obj/norms.o ../../build/obj/misc.o -o ../../build/var/lib$name.so
  echo "built build/var/lib$name.so"
done
