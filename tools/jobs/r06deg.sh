#!/usr/bin/env bash
set -uo pipefail
bash tools/jobs/r06g.sh
bash tools/jobs/r06e.sh
bash tools/jobs/r06d.sh
