#!/usr/bin/env bash
# round 5zd: the first-bounce pre-test row read in C (no inline-asm boundary, no s_nop) vs HEAD (build/v_h9)
set -uo pipefail
O=gpurun_out/r05zd
mkdir -p $O
L=build/v_h9/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 5 --frames 4 > $O/ab_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --rounds 5 --frames 4 > $O/ab_c.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs $L --rounds 5 > $O/hybrid_b.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --config a --libs $L --rounds 5 > $O/phong_a.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_golden.py -m gpu > $O/tests.txt 2>&1
rc=$?
python3 -c "
import json
for c in ('d','c'):
    try:
        d=json.loads(open('$O/ab_'+c+'.txt').read().strip().split('\n')[-1]); print(c, {k: round(v['median'],4) for k,v in d['ms'].items()})
    except Exception as e: print(c, 'n/a', e)"
grep -c "identical=False" $O/ab_d.txt $O/ab_c.txt
tail -1 $O/hybrid_b.txt; tail -1 $O/phong_a.txt; tail -1 $O/tests.txt
exit $rc
