# Diagnostic builds for per-phase PMC (tools/phase_stop_patch.py): the library of
# a git ref (or WORK = the working tree) with decode_split_kernel stopping every
# frame at phase boundary K, into exp_libs/<name>_s<K>/ (scratch, git-ignored):
#   tools/phase_stop_build.sh <name> <ref|WORK> "<K> <K> ..."
set -eu
cd "$(dirname "$0")/.."
NAME=$1; REF=$2; KS=$3
for K in $KS; do
  TMP=$(mktemp -d)
  if [ "$REF" = WORK ]; then
    mkdir -p "$TMP/qkd_ldpc_amd"; cp -r qkd_ldpc_amd/csrc "$TMP/qkd_ldpc_amd/"; cp -r include "$TMP/"
  else
    git archive "$REF" qkd_ldpc_amd/csrc include | tar -x -C "$TMP"
  fi
  python3 tools/phase_stop_patch.py "$TMP/qkd_ldpc_amd/csrc/decode_split.hip" > /dev/null
  make -s -C "$TMP/qkd_ldpc_amd/csrc" -j8 EXTRA="-DQKD_PMC_STOP=$K"
  mkdir -p exp_libs/${NAME}_s$K
  cp "$TMP/qkd_ldpc_amd/lib/libqkd_ldpc_amd.so" exp_libs/${NAME}_s$K/
  rm -rf "$TMP"
  echo "exp_libs/${NAME}_s$K/libqkd_ldpc_amd.so"
done
