#!/usr/bin/env bash
# round 5p: hybrid one-wave workgroups with the schedule at 8x8 granularity (production) vs the
# 2x2 blocks (v_hy22); schedule + mode-4 parity tests
set -uo pipefail
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs build/v_hy22/librtrt.so,real_time_ray_tracer_amd/librtrt.so --rounds 5 > $O/hybrid_bw_b.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_whole_frame" tests/test_golden.py -m gpu > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config b --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err
rc=$?
tail -1 $O/hybrid_bw_b.txt; tail -2 $O/tests.txt
python3 -c "import json; d=json.load(open('$O/bench_b.json')); print('bench b', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('tile_schedule'))"
exit $rc
