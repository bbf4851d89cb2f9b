#!/usr/bin/env bash
# round 5s: AO instruction budget at (d) by section-repeat ablations
set -uo pipefail
timeout -k 10 900 bash tools/sq_budget.sh r05s > gpurun_out/r05s_budget.txt 2>&1
rc=$?
tail -8 gpurun_out/r05s_budget.txt
exit $rc
