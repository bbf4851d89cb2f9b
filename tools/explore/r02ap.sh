# A/B: bounce rounds with 4-sphere scalar groups (104) instead of 2 (fewer loop SALU per test)
O=gpurun_out/r02ap; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/ab.py --config d --variants 7,104,105,7,104,105 --rounds 3 --frames 5 > $O/d.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config c --variants 7,104,105 --rounds 4 --frames 5 > $O/c.txt 2>&1 || exit $?
for f in d c; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k: round(v['median'], 4) for k, v in d['ms'].items()})"; done
