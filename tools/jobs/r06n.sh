#!/usr/bin/env bash
# round 6 GPU job n: hybrid_kernel with two pixels per lane (RT_HY_PX=2, 8x16-pixel wave tiles)
# against production: mode-4 parity + schedule + whole (b) frames on it, then per-launch bursts at (b)
set -uo pipefail
O=gpurun_out/r06n; mkdir -p $O
RTRT_LIB=build/v_px2/librtrt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_schedule.py tests/test_gpu_parity.py tests/test_golden.py -m gpu -k "schedule or mode_parity or golden or moving" \
  > $O/tests_px2.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_px2.txt; tail -2 $O/tests_px2.txt
[ $rc -ne 0 ] && exit $rc
RTRT_LIB=build/v_px2/librtrt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py -m gpu -k "whole_frame and b" > $O/tests_px2_fullsize.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_px2_fullsize.txt; tail -2 $O/tests_px2_fullsize.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/explore/r05/hybrid_burst.py --rounds 4 \
  --libs build/v_base/librtrt.so,build/v_px2/librtrt.so,build/v_px2m7/librtrt.so,build/v_px2m8/librtrt.so \
  > $O/hybrid_burst_b.txt 2>&1
rc=$?; tail -1 $O/hybrid_burst_b.txt; exit $rc
