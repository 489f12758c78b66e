#!/bin/bash
# Diagnostic builds: the speculative bit phase's load batch (QKD_IV_CHUNK rounds).
set -eu
cd "$(dirname "$0")/../qkd_ldpc_amd/csrc"
make -s -j4
OUT=../../exp_libs
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -x hip"
rm -f $OUT/lib_*.so
for n in ${CHUNKS:-3 7 10}; do
  ( /opt/rocm/bin/hipcc $F -DQKD_IV_CHUNK=$n -c decode_split.hip -o $OUT/split_c$n.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_c$n.so ../lib/obj/host.cpp.o ../lib/obj/decode.hip.o $OUT/split_c$n.o ) &
done
wait
rm -f $OUT/*.o
