#!/usr/bin/env bash
# round 5q: hybrid (b) with its tables and order as leading kernel arguments preloaded into SGPRs
# (production) vs the same code without the preload flag (v_nopre); mode-4 tests
set -uo pipefail
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs build/v_nopre/librtrt.so,real_time_ray_tracer_amd/librtrt.so --rounds 5 > $O/hybrid_preload_b.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_parity.py tests/test_golden.py -m gpu > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config b --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err
rc=$?
tail -1 $O/hybrid_preload_b.txt; tail -2 $O/tests.txt
python3 -c "import json; d=json.load(open('$O/bench_b.json')); print('bench b', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
exit $rc
