#!/bin/bash
# Builds an alternative in-tree library monte-carlo-raytracer_amd/libmcrt_<V>.so with extra
# compile definitions for one kernel source (default mcrt_kernels; A/B experiments, selected with
# MCRT_LIB_PATH; tools/variant_sweep.sh).
# usage: tools/build_variant.sh V "-DFOO=1 -DBAR=2" [mcrt_kernels|mcrt_bdpt]
set -e
V=$1; DEFS=$2; SRC=${3:-mcrt_kernels}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/monte-carlo-raytracer_amd/csrc
make -C "$C" >/dev/null
mkdir -p "$C/build_$V"
FLAGS="-O3 -std=c++17 -fPIC -I$ROOT/include -I/opt/rocm/include --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=on -fno-hip-fp32-correctly-rounded-divide-sqrt"
/opt/rocm/bin/hipcc $FLAGS $DEFS -c "$C/$SRC.hip" -o "$C/build_$V/$SRC.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/monte-carlo-raytracer_amd/libmcrt_$V.so" \
  "$C/build_$V/$SRC.o" $(ls "$C"/build/mcrt_*.o | grep -v "/$SRC.o") -lpthread -lz
echo "built libmcrt_$V.so ($DEFS)"
