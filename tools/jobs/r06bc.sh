#!/usr/bin/env bash
set -uo pipefail
bash tools/jobs/r06b.sh
bash tools/jobs/r06c.sh
