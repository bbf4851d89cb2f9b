#!/usr/bin/env bash
# round 5z8: the bounce rounds cluster cull as three ballots of single compares and scalar-select kept bits vs HEAD (build/v_h5)
# masks (build/v_def, RT_B1_DEFER=1; build/v_def2, two pending per lane) vs production: images identical (ab.py), AO (d)/(c) per launch
set -uo pipefail
O=gpurun_out/r05z8
mkdir -p $O
L=build/v_h5/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 5 --frames 4 > $O/ab_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --rounds 5 --frames 4 > $O/ab_c.txt 2>&1
rc=$?
[ $rc = 0 ] && timeout -k 10 300 python -u tools/ab.py --config e --libs $L --rounds 2 --frames 2 > $O/ab_e.txt 2>&1
python3 -c "
import json
for c in ('d','c'):
    try:
        d=json.loads(open('$O/ab_'+c+'.txt').read().strip().split('\n')[-1]); print(c, {k: round(v['median'],4) for k,v in d['ms'].items()})
    except Exception as e: print(c, 'n/a', e)"
tail -3 $O/ab_d.txt
exit $rc
