#!/usr/bin/env bash
# round 5z2: hybrid single-frame kernel with the object count requested together with the tile
# order (build/v_en, RT_HY_EARLY_NOBJ=1) vs production
set -uo pipefail
O=gpurun_out/r05z2
mkdir -p $O
L=real_time_ray_tracer_amd/librtrt.so,build/v_en/librtrt.so
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs $L --rounds 7 > $O/hybrid_b.txt 2>&1
rc=$?
tail -1 $O/hybrid_b.txt
exit $rc
