# Build the working tree's library with a patch script applied to a scratch
# copy of the sources, into exp_libs/<name>/ (scratch, git-ignored):
#   exp_build_variant.sh <name> <patch-script.py> [make vars...]
# The patch script gets the scratch csrc directory as its argument.
set -eu
cd "$(dirname "$0")/../.."
NAME=$1; PATCH=$2; shift 2
TMP=$(mktemp -d)
mkdir -p "$TMP/qkd_ldpc_amd"
cp -r qkd_ldpc_amd/csrc "$TMP/qkd_ldpc_amd/"
cp -r include "$TMP/"
python "$PATCH" "$TMP/qkd_ldpc_amd/csrc"
make -s -C "$TMP/qkd_ldpc_amd/csrc" -j4 "$@"
mkdir -p exp_libs/$NAME
cp "$TMP/qkd_ldpc_amd/lib/libqkd_ldpc_amd.so" exp_libs/$NAME/
rm -rf "$TMP"
echo "exp_libs/$NAME/libqkd_ldpc_amd.so"
