#!/bin/bash
# Build a measurement variant of the library: libpgmg_<name>.so = the sources with
# -DPGMG_TUNING and extra -D flags (compile-time A/B of pgmg_fused.hip variants).
#   scripts/build_variant.sh NAME "-DPGMG_PP_BUF=0 ..."
set -e
NAME=$1; shift
FLAGS="$*"
PKG=$(cd "$(dirname "$0")/../parallel-geometric-multigrid-for-poisson-problem_amd" && pwd)
B=$PKG/build_v_$NAME
mkdir -p $B
HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -Wno-unused-result -I$PKG/../include -DPGMG_TUNING $FLAGS"
pids=()
for s in pgmg_fused pgmg_coarse pgmg_kernels pgmg_tail pgmg_gops pgmg_ctx pgmg_ops pgmg_comm; do
  /opt/rocm/bin/hipcc $HIPFLAGS -c $PKG/csrc/$s.hip -o $B/$s.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
printf 'extern "C" const char *pgmg_source_hash(void) { return "variant-%s"; }\n' $NAME > $B/srchash.cpp
g++ -O2 -fPIC -c $B/srchash.cpp -o $B/srchash.o
/opt/rocm/bin/hipcc $HIPFLAGS $B/*.o -shared -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib -o $PKG/libpgmg_$NAME.so
rm -rf $B
echo "built $PKG/libpgmg_$NAME.so"
