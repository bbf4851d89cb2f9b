#!/usr/bin/env bash
# round 5v: the AO pass's normal/depth stores non-temporal too (build/v_ntg, RT_NT_GBUF=1) vs
# production (colour stores non-temporal): AO (d) per launch and the driver's (d) command alternating
set -uo pipefail
O=gpurun_out/r05v
mkdir -p $O
L=real_time_ray_tracer_amd/librtrt.so,build/v_ntg/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 5 --frames 4 > $O/ab_d.txt 2>&1 &&
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_d_prod_$i.json 2> $O/bench_d_prod_$i.err &&
  RTRT_LIB=build/v_ntg/librtrt.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_d_ntg_$i.json 2> $O/bench_d_ntg_$i.err || exit 1
done
rc=$?
tail -1 $O/ab_d.txt
for f in $O/bench_d_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('roofline_post',{}).get('kernel_ms'))"; done
exit $rc
