#!/bin/bash
# Diagnostic builds of the speculative decoder (never the shipped library):
# exp_libs/lib_<name>.so with decode_split.hip compiled under QKD_EXP_* macros.
set -eu
cd "$(dirname "$0")/../qkd_ldpc_amd/csrc"
make -s -j4
OUT=../../exp_libs
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -x hip"
build() {  # name flags...
  local n=$1; shift
  /opt/rocm/bin/hipcc $F "$@" -c decode_split.hip -o $OUT/split_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$n.so ../lib/obj/host.cpp.o ../lib/obj/decode.hip.o $OUT/split_$n.o
}
rm -f $OUT/lib_*.so
build noreplay -DQKD_EXP_NO_REPLAY
rm -f $OUT/*.o
