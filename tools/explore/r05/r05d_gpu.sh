#!/usr/bin/env bash
# round 5d: the N-wide sin (constants once per 2 / 3 hashes) vs the per-hash sin vs round 4
set -uo pipefail
O=gpurun_out/${TAG:-r05d}
mkdir -p $O
L=build/old/librtrt.so,build/c1/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --allow-diff --rounds 5 --frames 4 > $O/ab_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --allow-diff --rounds 5 --frames 4 > $O/ab_c.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_math_primitives_bitwise" "tests/test_gpu_parity.py::test_det_sin_exhaustive" tests/test_golden.py "tests/test_gpu_fullsize.py" -m gpu > $O/tests.txt 2>&1
rc=$?
tail -3 $O/ab_d.txt; tail -3 $O/ab_c.txt; tail -3 $O/tests.txt
exit $rc
