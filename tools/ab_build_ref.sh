# Build the HIP library of a git ref (default HEAD) into exp_libs/<name>/ for
# A/B runs against the working tree (tools/gpu_ab.sh):
#   tools/ab_build_ref.sh <name> [ref] ["-DQKD_X=0 ..."]
set -eu
cd "$(dirname "$0")/.."
NAME=$1; REF=${2:-HEAD}; DEFS=${3:-}
TMP=$(mktemp -d)
git archive "$REF" qkd_ldpc_amd/csrc include | tar -x -C "$TMP"
make -s -C "$TMP/qkd_ldpc_amd/csrc" -j8 EXTRA="$DEFS"
mkdir -p exp_libs/$NAME
cp "$TMP/qkd_ldpc_amd/lib/libqkd_ldpc_amd.so" exp_libs/$NAME/
rm -rf "$TMP"
echo "exp_libs/$NAME/libqkd_ldpc_amd.so"
