set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 120 ./tools/mb/issue_mb > gpurun_out/issue_mb.txt 2>&1 || exit 1
VARIANTS="sp_f64 sp_f32 minsum minsum_sc" OUT=gpurun_out/r03prof bash tools/gpu_profile.sh || exit $?
