#!/bin/bash
# Diagnostic builds: the exact split kernel's bit-phase load batch (QKD_EXACT_CHUNK rounds).
set -eu
cd "$(dirname "$0")/../qkd_ldpc_amd/csrc"
make -s -j4
OUT=../../exp_libs
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -x hip"
rm -f $OUT/lib_*.so
for n in ${CHUNKS:-2 3 4}; do
  ( /opt/rocm/bin/hipcc $F -DQKD_EXACT_CHUNK=$n -c decode_split.hip -o $OUT/split_e$n.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_e$n.so ../lib/obj/host.cpp.o ../lib/obj/decode.hip.o $OUT/split_e$n.o ) &
done
wait
rm -f $OUT/*.o
