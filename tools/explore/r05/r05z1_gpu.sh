#!/usr/bin/env bash
# round 5z1: single-frame Phong/hybrid kernels request the lane's first-word sphere row before
# the tile order (the culls consume it) vs HEAD (build/v_h3); mode 3/4 parity, bursts, bench
set -uo pipefail
O=gpurun_out/r05z1
mkdir -p $O
L=build/v_h3/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_fullsize.py -m gpu -k "mode_parity or compute_frames or moving_camera or schedule or max_depth or degenerate or config_a or config_b or scene_sizes" > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs $L --rounds 5 > $O/hybrid_b.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --config a --libs $L --rounds 5 > $O/phong_a.txt 2>&1 &&
timeout -k 10 200 python -u bench.py --config b --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err &&
timeout -k 10 200 python -u bench.py --config a --no-cpu-baseline > $O/bench_a.json 2> $O/bench_a.err
rc=$?
tail -3 $O/tests.txt; tail -1 $O/hybrid_b.txt; tail -1 $O/phong_a.txt
for c in a b; do python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('bench $c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; done
exit $rc
