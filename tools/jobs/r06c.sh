#!/usr/bin/env bash
# round 6 GPU job c: where hybrid_kernel's time goes at (b) (A/B library): per-wave timeline and
# the timing ablations (1 no shadow rays, 2 no scene tests, 3 primary cull only, 5 no bounces)
set -uo pipefail
O=gpurun_out
RTRT_LIB=build/librtrt_ab.so timeout -k 10 120 python -u tools/explore/wave_timeline.py b > $O/r06c_wave_timeline_b.txt 2>&1 || exit $?
RTRT_LIB=build/librtrt_ab.so timeout -k 10 200 python -u tools/ab.py --config b --env RTRT_HY_ABL --variants 0,1,2,3,5 \
  --rounds 3 --frames 40 --allow-diff > $O/r06c_hybrid_ablations_b.txt 2>&1 || exit $?
tail -3 $O/r06c_hybrid_ablations_b.txt
