#!/usr/bin/env bash
# round 6 final evidence (build with the pool-start priority), part 2c: config (e) bench line + rocprof, and its N = 8 strip estimate
set -uo pipefail
O=gpurun_out/r06zj; mkdir -p $O
timeout -k 10 900 bash tools/round_profile.sh bench r06zj e > $O/bench_e.log 2>&1 || { tail -20 $O/bench_e.log; exit 1; }
tail -4 $O/bench_e.log
timeout -k 10 400 python -u tools/strip_scaling.py --config e --n 8 --frames 6 --calibrate --warm-ms 300 \
  --save-profile $O/strip_scaling_e_n8.json > $O/strip_scaling_e_n8_calibrated.txt 2>&1 || exit $?
grep -v amdgpu $O/strip_scaling_e_n8_calibrated.txt | tail -4
