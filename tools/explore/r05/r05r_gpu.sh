#!/usr/bin/env bash
# round 5r: phong (a) and hybrid (b) with leading preloaded table arguments vs no preload flag
set -uo pipefail
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --config a --libs build/v_nopre/librtrt.so,real_time_ray_tracer_amd/librtrt.so --rounds 5 --reps 400 > $O/phong_preload_a.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs build/v_nopre/librtrt.so,real_time_ray_tracer_amd/librtrt.so --rounds 5 > $O/hybrid_preload_b.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_image.py -m gpu > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config a --no-cpu-baseline > $O/bench_a.json 2> $O/bench_a.err
rc=$?
tail -1 $O/phong_preload_a.txt; tail -1 $O/hybrid_preload_b.txt; tail -2 $O/tests.txt
python3 -c "import json; d=json.load(open('$O/bench_a.json')); print('bench a', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
exit $rc
