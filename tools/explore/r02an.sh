# timing ablations: pools end after the cull (114), sky pools skip their stores (115)
O=gpurun_out/r02an; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/ab.py --config d --variants 7,114,115 --rounds 3 --frames 5 --allow-diff > $O/d.txt 2>&1 || exit $?
grep -h "^{" $O/d.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('d', {k: round(v['median'], 4) for k, v in d['ms'].items()})"
