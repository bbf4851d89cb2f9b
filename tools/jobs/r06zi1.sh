#!/usr/bin/env bash
# round 6 final evidence (build with the pool-start priority), part 1: PMC HBM bytes and SQ instruction counters per config on this build
set -uo pipefail
timeout -k 10 1500 bash tools/round_profile.sh counters r06zi d c b a e p ref > gpurun_out/r06zi1.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r06zi1.log
cat real_time_ray_tracer_amd/BUILD_INFO >> gpurun_out/r06zi1.log
exit $rc
