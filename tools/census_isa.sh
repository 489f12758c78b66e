#!/bin/bash
# The split decoder's ISA for the opcode census (CPU only): decode_split.hip
# compiled as the Makefile does (plus line tables for source attribution, and
# EXTRA definitions), the device assembly into OUT.s, the headline kernel's
# register and spill summary printed, then tools/valu_census.py over it:
#   tools/census_isa.sh OUT.s [PHASE_PMC.json CENSUS_OUT.json]
set -eu
cd "$(dirname "$0")/.."
OUT=$(realpath -m "$1")
TMP=$(mktemp -d)
( cd "$TMP" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -gline-tables-only \
    -mllvm -amdgpu-sched-strategy=gcn-max-ilp ${EXTRA:-} -x hip -c "$OLDPWD/qkd_ldpc_amd/csrc/decode_split.hip" \
    -o k.o --save-temps -Rpass-analysis=kernel-resource-usage 2>&1 ) \
  | grep -A9 "decode_split_kernelILi1ELi0ELi6ELb1ELi1ELb0E" | grep -E "SGPRs Spill|VGPRs:|VGPRs Spill" \
  | sed 's/.*remark: *//' | tr '\n' ' '; echo
cp "$TMP"/decode_split-hip-amdgcn-amd-amdhsa-gfx950.s "$OUT"
rm -rf "$TMP"
if [ $# -ge 3 ]; then python3 tools/valu_census.py census "$OUT" "$2" "$3"; fi
