#!/usr/bin/env bash
# round 6 GPU job o: the post-process's cost in the pipelined (d) frame: wall ms per pipelined frame
# with the production library, the A/B library, and the A/B library with the post-process skipped
set -uo pipefail
O=gpurun_out/r06o; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/explore/pipeline_floor.py --config d > $O/prod_$i.txt 2>&1 || exit $?
  RTRT_LIB=build/librtrt_ab.so timeout -k 10 120 python -u tools/explore/pipeline_floor.py --config d > $O/ab_$i.txt 2>&1 || exit $?
  RTRT_LIB=build/librtrt_ab.so RTRT_POST_SKIP=1 timeout -k 10 120 python -u tools/explore/pipeline_floor.py --config d > $O/ab_nopost_$i.txt 2>&1 || exit $?
  tail -1 $O/prod_$i.txt; tail -1 $O/ab_$i.txt; tail -1 $O/ab_nopost_$i.txt
done
