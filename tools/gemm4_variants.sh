# Build gemm4 schedule variants: tools/gemm4_variants.sh "name:-DFLAG=.. -DFLAG2=.." ...  -> build/var/libsvla_<name>.so
set -e
cd "$(dirname "$0")/../spatialvla_amd/csrc"
mkdir -p ../../build/var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=fast $flags -c gemm.hip -o ../../build/var/gemm_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  others=$(ls ../../build/obj/*.o | grep -v '/gemm\.o$')
  /opt/rocm/bin/hipcc -shared -fPIC -Wl,-Bsymbolic --offload-arch=gfx950 ../../build/var/gemm_$name.o $others -o ../../build/var/libsvla_$name.so
  echo "built build/var/libsvla_$name.so"
done
