#!/usr/bin/env bash
# round 5t: first-bounce candidate test on scalar masks (production) vs HEAD (build/prev)
set -uo pipefail
O=gpurun_out/r05t
mkdir -p $O
L=build/h1/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 7 --frames 4 > $O/ab_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --rounds 7 --frames 4 > $O/ab_c.txt 2>&1
rc=$?
python3 -c "
import json
for c in ('d','c'):
    d=json.loads(open('$O/ab_'+c+'.txt').read().strip().split('\n')[-1]); print(c, {k: round(v['median'],4) for k,v in d['ms'].items()})"
exit $rc
