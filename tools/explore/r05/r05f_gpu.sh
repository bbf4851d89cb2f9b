#!/usr/bin/env bash
# round 5f: sin per call (v_sin1) vs N-wide (production) vs the first sin build (c1); the driver's bench
set -uo pipefail
O=gpurun_out/r05f
mkdir -p $O
L=build/c1/librtrt.so,build/v_sin1/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --allow-diff --rounds 7 --frames 4 > $O/ab_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --allow-diff --rounds 7 --frames 4 > $O/ab_c.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
tail -1 $O/ab_d.txt | cut -c1-600; tail -1 $O/ab_c.txt | cut -c1-600
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline_post']['kernel_ms'], d['cpu_baseline'].get('value'))"
exit $rc
