# r04j: the final build's bench lines (with CPU baselines) and rocprof kernel traces per config,
# then the GPU suite and smoke
set -o pipefail
bash tools/round_profile.sh bench r04j "$@"
