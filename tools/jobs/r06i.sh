#!/usr/bin/env bash
# round 6 GPU job i: the same sources under two other AMDGPU scheduler settings (AMDGPU register
# pressure trackers; max-memory-clause) against the production build, same process, bit-identical
set -uo pipefail
O=gpurun_out/r06i; mkdir -p $O
L=build/v_base/librtrt.so,build/v_trk/librtrt.so,build/v_memcl/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 4 --frames 4 > $O/ab_sched_d.txt 2>&1 || exit $?
tail -1 $O/ab_sched_d.txt | cut -c 300-700
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --rounds 4 --frames 4 > $O/ab_sched_c.txt 2>&1 || exit $?
tail -1 $O/ab_sched_c.txt | cut -c 250-700
for i in 1 2; do for v in base trk memcl; do
  RTRT_LIB=build/v_$v/librtrt.so timeout -k 10 120 python3 bench.py --config b --no-cpu-baseline --no-alt-dispatch > $O/b_${v}_$i.json 2>/dev/null || exit $?
  RTRT_LIB=build/v_$v/librtrt.so timeout -k 10 200 python3 bench.py --config d --no-cpu-baseline > $O/d_${v}_$i.json 2>/dev/null || exit $?
  python3 -c "import json
for c in 'bd':
  d=json.loads(open('$O/'+c+'_${v}_$i.json').read().strip().splitlines()[-1]); print(c, '$v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('roofline_post', {}).get('kernel_ms'))"
done; done
