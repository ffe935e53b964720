#!/bin/bash
# Builds an experimental variant of libweightedld.so with extra compile flags on
# pair_mfma.hip (other objects shared with the main build):
#   tools/build_variant.sh NAME "-DFLAG ..."   -> build/exp/NAME/libweightedld.so
# SLP=1 builds the source without -fno-slp-vectorize (packed-f32 probe);
# SRC=pair_valu varies pair_valu.hip instead of pair_mfma.hip; SRC="pair_valu
# pair_mfma" both.  SRCFILE=path compiles that file in place of the (single)
# SRC source (e.g. a git revision's copy: git show REV:weightedld_amd/csrc/pair_mfma.hip).
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
src=${SRC:-pair_mfma}
make -s build/obj/encode.o build/obj/prepass.o build/obj/pair_valu.o build/obj/pair_mfma.o build/obj/order.o \
  build/obj/capi.o build/obj/host.o
out=build/exp/$name; mkdir -p $out
slp=-fno-slp-vectorize
[ "${SLP:-0}" = 1 ] && slp=
for one in $src; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $slp -Wall -Iinclude \
    -Iweightedld_amd/csrc $flags -x hip -c ${SRCFILE:-weightedld_amd/csrc/$one.hip} -o $out/$one.o
done
objs=""
for o in encode prepass pair_valu pair_mfma order capi host; do
  if [[ " $src " == *" $o "* ]]; then objs="$objs $out/$o.o"; else objs="$objs build/obj/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libweightedld.so $objs -lpthread
echo "$out/libweightedld.so"
