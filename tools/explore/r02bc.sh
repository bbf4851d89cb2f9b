# A/B: shade's emissive / mirror cases as selects (109)
O=gpurun_out/r02bc; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 250 python tools/ab.py --config d --variants 7,109,7,109 --rounds 4 --frames 5 > $O/d.txt 2>&1 || exit $?
timeout -k 10 250 python tools/ab.py --config c --variants 7,109 --rounds 5 --frames 5 > $O/c.txt 2>&1 || exit $?
for f in d c; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k: round(v['median'], 4) for k, v in d['ms'].items()})"; done
