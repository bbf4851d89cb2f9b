#!/usr/bin/env bash
# round 5b: correctly rounded sin — exhaustive device sweep, goldens, cost A/B against round 4
set -uo pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_det_sin_exhaustive" "tests/test_gpu_parity.py::test_math_primitives_bitwise" \
  tests/test_golden.py tests/test_gpu_bench_launch.py -m gpu -s > $O/sin_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config d --libs build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so \
  --allow-diff --rounds 5 --frames 4 > $O/ab_sin_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so \
  --allow-diff --rounds 5 --frames 4 > $O/ab_sin_c.txt 2>&1
rc=$?
tail -5 $O/sin_tests.txt; tail -4 $O/ab_sin_d.txt; tail -4 $O/ab_sin_c.txt
exit $rc
