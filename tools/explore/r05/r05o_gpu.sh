#!/usr/bin/env bash
# round 5o: hybrid (b) block shapes (1x1 .. 4x4 waves of 8x8 tiles), tables through the caches,
# row order for all (the schedule's tables are sized for 2x2 blocks)
set -uo pipefail
O=gpurun_out/r05o
mkdir -p $O
RTRT_LIB=build/librtrt_ab.so timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --env RTRT_HY_BLK --variants 22,11,21,41,42 --no-schedule --rounds 3 > $O/hybrid_blk_b.txt 2>&1
rc=$?
tail -1 $O/hybrid_blk_b.txt
exit $rc
