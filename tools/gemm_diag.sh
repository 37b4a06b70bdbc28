# Build diagnostic variants of libsvla.so (SVLA_GEMM_DIAG bits, see gemm.hip) into build/diag/.
set -e
cd "$(dirname "$0")/../spatialvla_amd/csrc"
mkdir -p ../../build/diag
for d in 1 2 4 5 6 12 13 14 29 31; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -DSVLA_GEMM_DIAG=$d -c gemm.hip -o ../../build/diag/gemm_$d.o
  hipcc -shared -fPIC --offload-arch=gfx950 ../../build/obj/runtime.o ../../build/diag/gemm_$d.o ../../build/obj/attention.o \
    ../../build/obj/norms.o ../../build/obj/misc.o -o ../../build/diag/libsvla_diag$d.so
done
