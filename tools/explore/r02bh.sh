# A/B (libs): pop_lowest in the plane-mask, primary-cone, shadow-cone and unpretested first-bounce loops; configs b a p d
O=gpurun_out/r02bh; mkdir -p $O
L=build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so
for c in b a; do
  timeout -k 10 250 python tools/ab.py --config $c --libs $L --rounds 6 --frames 20 > $O/$c.txt 2>&1 || exit $?
done
for c in p d; do
  timeout -k 10 250 python tools/ab.py --config $c --libs $L --rounds 4 --frames 5 > $O/$c.txt 2>&1 || exit $?
done
for f in b a p d; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k.split('/')[0]: round(v['median'], 5) for k, v in d['ms'].items()})"; done
