# A/B (libs): first-bounce pre-test as a wave-uniform SGPR-mask skip; configs d c d
O=gpurun_out/r02bk; mkdir -p $O
L=build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 250 python tools/ab.py --config d --libs $L --rounds 4 --frames 5 > $O/d1.txt 2>&1 || exit $?
timeout -k 10 250 python tools/ab.py --config c --libs $L --rounds 4 --frames 5 > $O/c.txt 2>&1 || exit $?
timeout -k 10 250 python tools/ab.py --config d --libs $L --rounds 4 --frames 5 > $O/d2.txt 2>&1 || exit $?
for f in d1 c d2; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k.split('/')[0]: round(v['median'], 5) for k, v in d['ms'].items()})"; done
