#!/usr/bin/env bash
# round 6 GPU job a: the changed/new GPU tests, then the paired pre-test A/B at (d) and (c)
set -uo pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_faults.py \
  tests/test_gpu_bench_launch.py "tests/test_gpu_parity.py::test_sin_table_entries_are_ambiguous_on_this_device_build" \
  tests/test_gpu_group.py > $O/r06a_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> $O/r06a_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/ab.py --config d --libs real_time_ray_tracer_amd/librtrt.so,build/v_pairs/librtrt.so,build/v_quads/librtrt.so \
  --rounds 4 --frames 4 > $O/r06a_ab_pairs_d.txt 2>&1 || exit $?
timeout -k 10 240 python -u tools/ab.py --config c --libs real_time_ray_tracer_amd/librtrt.so,build/v_pairs/librtrt.so,build/v_quads/librtrt.so \
  --rounds 4 --frames 4 > $O/r06a_ab_pairs_c.txt 2>&1 || exit $?
exit $rc
