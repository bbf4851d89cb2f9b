#!/usr/bin/env bash
# round 5i: AO kernel compiled for 6 / 7 (production) / 8 waves per SIMD with the binary64 sin
set -uo pipefail
O=gpurun_out/r05i
mkdir -p $O
L=build/v_w6/librtrt.so,real_time_ray_tracer_amd/librtrt.so,build/v_w8/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 5 --frames 4 > $O/ab_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --rounds 5 --frames 4 > $O/ab_c.txt 2>&1
rc=$?
tail -1 $O/ab_d.txt | cut -c 1-40; python3 -c "
import json
for c in ('d','c'):
    d=json.loads(open('$O/ab_'+c+'.txt').read().strip().split('\n')[-1]); print(c, {k: round(v['median'],4) for k,v in d['ms'].items()})"
exit $rc
