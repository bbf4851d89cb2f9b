# A/B: pool interleave (RTRT_POOL_ILV = log2 K) and branchless bounce-round hit tails (variant 94)
O=gpurun_out/r02z; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/ab.py --config d --env RTRT_POOL_ILV --variants 0,2,4,6,0 --rounds 3 --frames 5 > $O/ilv_d.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config d --variants 7,94 --rounds 4 --frames 5 > $O/nb_d.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config c --env RTRT_POOL_ILV --variants 0,4 --rounds 4 --frames 5 > $O/ilv_c.txt 2>&1 || exit $?
for f in ilv_d nb_d ilv_c; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k: round(v['median'], 4) for k, v in d['ms'].items()})"; done
