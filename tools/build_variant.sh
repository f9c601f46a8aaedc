#!/bin/bash
# Builds an alternative in-tree library monte-carlo-raytracer_amd/libmcrt_<V>.so with extra
# compile definitions for mcrt_kernels.hip (A/B experiments; run with tools/variant_sweep.sh).
# usage: tools/build_variant.sh V "-DFOO=1 -DBAR=2"
set -e
V=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/monte-carlo-raytracer_amd/csrc
make -C "$C" >/dev/null
mkdir -p "$C/build_$V"
FLAGS="-O3 -std=c++17 -fPIC -I$ROOT/include -I/opt/rocm/include --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=on -fno-hip-fp32-correctly-rounded-divide-sqrt"
/opt/rocm/bin/hipcc $FLAGS $DEFS -c "$C/mcrt_kernels.hip" -o "$C/build_$V/mcrt_kernels.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/monte-carlo-raytracer_amd/libmcrt_$V.so" \
  "$C/build_$V/mcrt_kernels.o" $(ls "$C"/build/*.o | grep -v mcrt_kernels.o) -lpthread
echo "built libmcrt_$V.so ($DEFS)"
