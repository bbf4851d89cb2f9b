# LDS allocation granule probe: the AO launch's dynamic LDS (5504 B) plus 0 / 128 / 600 / 700 / 1200 bytes
O=gpurun_out/r02ah; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 250 python tools/ab.py --config d --env RTRT_LDS_EXTRA --variants 0,128,600,700,1200,0 --rounds 3 --frames 4 > $O/lds_d.txt 2>&1 || exit $?
grep -h "^{" $O/lds_d.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('lds', {k: round(v['median'], 4) for k, v in d['ms'].items()})"
