set -uo pipefail
bash tools/jobs/r06zj2b.sh && bash tools/jobs/r06zj2c.sh
