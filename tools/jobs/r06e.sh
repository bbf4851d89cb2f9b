#!/usr/bin/env bash
# round 6 GPU job e: the AO kernel's instruction budget at (d) with the round-6 sections (A/B library)
set -uo pipefail
timeout -k 10 900 bash tools/sq_budget.sh r06e_budget > gpurun_out/r06e_budget.txt 2>&1
echo "rc=$?" >> gpurun_out/r06e_budget.txt
tail -14 gpurun_out/r06e_budget.txt
