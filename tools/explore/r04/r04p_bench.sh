# r04p: the final build's bench lines (with CPU baselines) and rocprof kernel traces per config
set -o pipefail
bash tools/round_profile.sh bench r04p "$@"
