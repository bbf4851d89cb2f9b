#!/usr/bin/env bash
# round 6 GPU job l: persistent hybrid blocks over the tile schedule (RT_HY_PERSIST blocks per CU)
# against production: mode-4 parity on one variant, then per-launch bursts at (b) for all
set -uo pipefail
O=gpurun_out/r06l; mkdir -p $O
RTRT_LIB=build/v_hyp7m7/librtrt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_schedule.py tests/test_gpu_parity.py tests/test_golden.py -m gpu -k "schedule or mode_parity or golden or moving" \
  > $O/tests_hyp7m7.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_hyp7m7.txt; tail -2 $O/tests_hyp7m7.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/explore/r05/hybrid_burst.py --rounds 4 \
  --libs build/v_base/librtrt.so,build/v_hyp7m7/librtrt.so,build/v_hyp6/librtrt.so,build/v_hyp7l/librtrt.so,build/v_hyp14m7/librtrt.so \
  > $O/hybrid_burst_b.txt 2>&1
rc=$?; tail -1 $O/hybrid_burst_b.txt; exit $rc
