# A/B: odd pool interleaves (RTRT_POOL_ILV = K) and first-bounce survivor loads waited together (variant 95)
O=gpurun_out/r02z2; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/ab.py --config d --env RTRT_POOL_ILV --variants 0,3,5,15,0 --rounds 3 --frames 5 > $O/ilv_d.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config d --variants 7,95 --rounds 4 --frames 5 > $O/v95_d.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config c --variants 7,95 --rounds 4 --frames 5 > $O/v95_c.txt 2>&1 || exit $?
for f in ilv_d v95_d v95_c; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k: round(v['median'], 4) for k, v in d['ms'].items()})"; done
