#!/usr/bin/env bash
# round 5l: tier-1 sin rounding by the 1.5*2^52 constant (production) vs rint + cvt (v_nomagic);
# hybrid (b) two tiles per block (v_hy2) vs one
set -uo pipefail
O=gpurun_out/r05l
mkdir -p $O
L=build/v_nomagic/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 5 --frames 4 > $O/ab_magic_d.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --rounds 5 --frames 4 > $O/ab_magic_c.txt 2>&1 &&
timeout -k 10 300 python -u tools/explore/r05/hybrid_burst.py --libs real_time_ray_tracer_amd/librtrt.so,build/v_hy2/librtrt.so --rounds 4 > $O/hybrid_tpb2_b.txt 2>&1 &&
RTRT_LIB=build/v_hy2/librtrt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py "tests/test_gpu_fullsize.py::test_whole_frame" -m gpu > $O/tests_hy2.txt 2>&1
rc=$?
python3 -c "
import json
for c in ('magic_d','magic_c'):
    d=json.loads(open('$O/ab_'+c+'.txt').read().strip().split('\n')[-1]); print(c, {k: round(v['median'],4) for k,v in d['ms'].items()})"
tail -1 $O/hybrid_tpb2_b.txt; tail -2 $O/tests_hy2.txt
exit $rc
