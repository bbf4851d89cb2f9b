# r04j: the final build's counters (PMC traffic + SQ) per config: tools/round_profile.sh counters
set -o pipefail
bash tools/round_profile.sh counters r04j "$@"
