# A/B (same process): HEAD library vs uniform-branch hit tails + 4-sphere bounce groups, configs d c p b a
O=gpurun_out/r02ar; mkdir -p $O
L=build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so
for c in d c p; do
  timeout -k 10 250 python tools/ab.py --config $c --libs $L --rounds 4 --frames 5 > $O/$c.txt 2>&1 || exit $?
done
for c in; do
  timeout -k 10 250 python tools/ab.py --config $c --libs $L --rounds 6 --frames 20 > $O/$c.txt 2>&1 || exit $?
done
for c in d c p; do grep -h "^{" $O/$c.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$c', {k.split('/')[0]: round(v['median'], 5) for k, v in d['ms'].items()})"; grep -c "identical=True" $O/$c.txt; done
