# A/B: bounce-round group loop unrolled x2 (104) / x4 (105)
O=gpurun_out/r02az; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 250 python tools/ab.py --config d --variants 105,104,108,105,104,108 --rounds 3 --frames 5 > $O/d.txt 2>&1 || exit $?
timeout -k 10 250 python tools/ab.py --config c --variants 105,104,108 --rounds 4 --frames 5 > $O/c.txt 2>&1 || exit $?
for f in d c; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k: round(v['median'], 4) for k, v in d['ms'].items()})"; done
