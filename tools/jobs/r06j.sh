#!/usr/bin/env bash
# round 6 GPU job j: hybrid_kernel at (b), one segment per path (ABL 5) with and without the shading's
# per-lane table loads (ABL 9): how much of a wave's chain the shading loads are
set -uo pipefail
O=gpurun_out/r06j; mkdir -p $O
RTRT_LIB=build/librtrt_ab.so timeout -k 10 300 python -u tools/ab.py --config b --env RTRT_HY_ABL --variants 5,9,5,9 \
  --rounds 4 --frames 40 --allow-diff > $O/hybrid_shading_loads_b.txt 2>&1 || exit $?
tail -1 $O/hybrid_shading_loads_b.txt | cut -c 300-800
