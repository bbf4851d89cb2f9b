#!/usr/bin/env bash
# round 5k: hybrid (b) two tiles per block (longest + shortest of the schedule's order) vs one
set -uo pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs real_time_ray_tracer_amd/librtrt.so,build/v_hy2/librtrt.so --rounds 4 > $O/hybrid_tpb2_b.txt 2>&1 &&
RTRT_LIB=build/v_hy2/librtrt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py "tests/test_gpu_fullsize.py::test_whole_frame" -m gpu > $O/tests_hy2.txt 2>&1
rc=$?
tail -1 $O/hybrid_tpb2_b.txt; tail -2 $O/tests_hy2.txt
exit $rc
