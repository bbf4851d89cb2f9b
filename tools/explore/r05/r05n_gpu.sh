#!/usr/bin/env bash
# round 5n: tables read through the caches instead of staged in LDS per block: hybrid (b) v_nolt,
# phong (a) v_phnolt; and hybrid at (b) with the GPU tests on v_nolt
set -uo pipefail
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs real_time_ray_tracer_amd/librtrt.so,build/v_nolt/librtrt.so --rounds 5 > $O/hybrid_nolt_b.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --config a --libs real_time_ray_tracer_amd/librtrt.so,build/v_phnolt/librtrt.so --rounds 5 --reps 400 > $O/phong_nolt_a.txt 2>&1 &&
RTRT_LIB=build/v_nolt/librtrt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py "tests/test_gpu_fullsize.py::test_whole_frame" tests/test_gpu_parity.py -m gpu > $O/tests_nolt.txt 2>&1
rc=$?
tail -1 $O/hybrid_nolt_b.txt; tail -1 $O/phong_nolt_a.txt; tail -2 $O/tests_nolt.txt
exit $rc
