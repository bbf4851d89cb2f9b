# A/B: first-bounce pre-test rows by readlane + masked exact pass (98: streamed table, 99: plain loop)
O=gpurun_out/r02z5; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/ab.py --config d --variants 7,98,99 --rounds 4 --frames 5 > $O/d.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config c --variants 7,98,99 --rounds 4 --frames 5 > $O/c.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config e --variants 7,99 --rounds 2 --frames 2 > $O/e.txt 2>&1 || exit $?
for f in d c e; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k: round(v['median'], 4) for k, v in d['ms'].items()})"; done
