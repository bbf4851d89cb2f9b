#!/usr/bin/env bash
# round 5m: hybrid (b) without the per-block LDS table staging (v_nolt) vs production
set -uo pipefail
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs real_time_ray_tracer_amd/librtrt.so,build/v_nolt/librtrt.so --rounds 4 > $O/hybrid_nolt_b.txt 2>&1
rc=$?
tail -1 $O/hybrid_nolt_b.txt
exit $rc
