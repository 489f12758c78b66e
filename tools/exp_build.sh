#!/bin/bash
# Diagnostic builds of the split-store decoder (never the shipped library):
# exp_libs/lib_<name>.so = the in-tree objects of host.cpp and decode.hip plus
# decode_split.hip compiled with QKD_EXP_* macros (decode_split.hip header).
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
build base -DQKD_EXP_NO_STOP &
build nomath -DQKD_EXP_NO_STOP -DQKD_EXP_NO_MATH &
build nosyn -DQKD_EXP_NO_STOP -DQKD_EXP_NO_SYN &
build nomath_nosyn -DQKD_EXP_NO_STOP -DQKD_EXP_NO_MATH -DQKD_EXP_NO_SYN &
wait
rm -f $OUT/*.o
ls -la $OUT
