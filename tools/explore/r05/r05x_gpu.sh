#!/usr/bin/env bash
# round 5x: shadow occluder test decided in float away from len (production) vs the binary64
# sequence for every t (build/v_shx, RT_SHADOW_FAST=0): decision test, modes 3/4 parity, bursts
set -uo pipefail
O=gpurun_out/r05x
mkdir -p $O
L=build/v_shx/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "shadow or mode_parity or math_primitives or moving_camera" > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs $L --rounds 5 > $O/hybrid_b.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --config a --libs $L --rounds 5 > $O/phong_a.txt 2>&1
rc=$?
tail -3 $O/tests.txt; tail -1 $O/hybrid_b.txt; tail -1 $O/phong_a.txt
exit $rc
