#!/usr/bin/env bash
# round 5z6: hybrid (b) shadow rays without the light cone up to 16 / 64 objects (build/v_sc16,
# build/v_sc64, RT_SHADOW_CONE_MIN) vs production (the cone above 8 objects)
set -uo pipefail
O=gpurun_out/r05z6
mkdir -p $O
L=real_time_ray_tracer_amd/librtrt.so,build/v_sc16/librtrt.so,build/v_sc64/librtrt.so
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs $L --rounds 5 > $O/hybrid_b.txt 2>&1
rc=$?
tail -1 $O/hybrid_b.txt
exit $rc
