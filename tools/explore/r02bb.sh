# A/B (libs): split-tail loop unrolled 2x + hybrid closest_hit unrolled 4x; configs d c b
O=gpurun_out/r02bb; mkdir -p $O
L=build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so
for k in 1 2; do
  timeout -k 10 250 python tools/ab.py --config d --libs $L --rounds 4 --frames 5 > $O/d$k.txt 2>&1 || exit $?
done
timeout -k 10 250 python tools/ab.py --config c --libs $L --rounds 5 --frames 5 > $O/c.txt 2>&1 || exit $?
timeout -k 10 250 python tools/ab.py --config b --libs $L --rounds 6 --frames 20 > $O/b.txt 2>&1 || exit $?
for f in d1 d2 c b; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k.split('/')[0]: round(v['median'], 5) for k, v in d['ms'].items()})"; done
