#!/usr/bin/env bash
# round 6 GPU job t: config (e) (256 spheres) with the first bounce's pre-test rows one word at a
# time (RT_PT_WIDE=1) and with clusters of 16: per-launch A/B (images must be bit-identical), then
# the whole (e) frame against the oracle on the pre-test build
set -uo pipefail
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 400 python -u tools/ab.py --config e --rounds 3 --frames 3 \
  --libs real_time_ray_tracer_amd/librtrt.so,build/v_ptw/librtrt.so,build/v_cl16/librtrt.so > $O/ab_e.txt 2>&1
rc=$?; tail -1 $O/ab_e.txt; [ $rc -ne 0 ] && exit $rc
RTRT_LIB=build/v_ptw/librtrt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread \
  tests/test_gpu_fullsize.py -m gpu -k "whole_frame and e" > $O/tests_ptw_e.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_ptw_e.txt; tail -2 $O/tests_ptw_e.txt; exit $rc
