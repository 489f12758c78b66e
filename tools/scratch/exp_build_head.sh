# Build the library of a git revision (default HEAD) into exp_libs/<name>/ for
# tools/gpu_ab_libs.sh (scratch, git-ignored): exp_build_head.sh [rev] [name]
set -eu
cd "$(dirname "$0")/../.."
REV=${1:-HEAD}
NAME=${2:-head}
TMP=$(mktemp -d)
git archive "$REV" qkd_ldpc_amd/csrc include | tar -x -C "$TMP"
make -s -C "$TMP/qkd_ldpc_amd/csrc" -j4 ${EXTRA_MAKE:-}
mkdir -p exp_libs/$NAME
cp "$TMP/qkd_ldpc_amd/lib/libqkd_ldpc_amd.so" exp_libs/$NAME/
rm -rf "$TMP"
echo "exp_libs/$NAME/libqkd_ldpc_amd.so"
