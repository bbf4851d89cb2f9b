#!/usr/bin/env bash
# round 5h: hybrid_kernel (config b) burst timings of the timing ablations, and the wave timeline
set -uo pipefail
O=gpurun_out/r05h
mkdir -p $O
RTRT_LIB=build/librtrt_ab.so timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --env RTRT_HY_ABL --variants 0,1,2,3,5,6 --rounds 3 > $O/hybrid_abl_b.txt 2>&1 &&
RTRT_LIB=build/librtrt_ab.so timeout -k 10 120 python -u tools/explore/wave_timeline.py b > $O/wave_timeline_b.txt 2>&1
rc=$?
cat $O/hybrid_abl_b.txt | tail -2; tail -30 $O/wave_timeline_b.txt
exit $rc
