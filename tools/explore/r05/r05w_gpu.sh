#!/usr/bin/env bash
# round 5w: hybrid (b) timing ablations on the production table form (tables through the caches,
# schedule on): 0 production, 2 no scene tests (launch + directions + stores), 3 primary cull only,
# 1 no shadow rays, 5 no bounce segments
set -uo pipefail
O=gpurun_out/r05w
mkdir -p $O
RTRT_LIB=build/librtrt_ab.so timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --env RTRT_HY_ABL --variants 0,2,3,1,5 --rounds 3 > $O/hybrid_abl_b.txt 2>&1
rc=$?
tail -1 $O/hybrid_abl_b.txt
exit $rc
