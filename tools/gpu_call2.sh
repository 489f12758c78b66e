set -u
cd "$(dirname "$0")/.."
bash tools/gpu_round.sh ${1:-r03b} || exit $?
OUT=gpurun_out/${1:-r03b}/prof bash tools/gpu_profile.sh || exit $?
