#!/usr/bin/env bash
# round 5z5: the whole GPU suite on the deferred first-bounce build, with test durations
set -uo pipefail
O=gpurun_out/r05z5
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > $O/gpu_tests.txt 2>&1
rc=$?
tail -22 $O/gpu_tests.txt
exit $rc
