# Build the working tree's HIP library with extra compile definitions into
# exp_libs/<name>/ (scratch, git-ignored) for A/B runs (tools/gpu_ab.sh):
#   tools/ab_build.sh <name> "-DQKD_X=0 ..."
set -eu
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2
TMP=$(mktemp -d)
mkdir -p "$TMP/qkd_ldpc_amd"
cp -r qkd_ldpc_amd/csrc "$TMP/qkd_ldpc_amd/"
cp -r include "$TMP/"
make -s -C "$TMP/qkd_ldpc_amd/csrc" -j8 EXTRA="$DEFS"
mkdir -p exp_libs/$NAME
cp "$TMP/qkd_ldpc_amd/lib/libqkd_ldpc_amd.so" exp_libs/$NAME/
rm -rf "$TMP"
echo "exp_libs/$NAME/libqkd_ldpc_amd.so"
