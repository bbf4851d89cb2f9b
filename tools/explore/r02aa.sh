# production build with XCD-balanced pool / tile order: GPU suite, A/B of the rotations, benches
set -o pipefail
O=gpurun_out/r02aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/ab.py --config b --env RTRT_TILE_ROT --variants 1,0 --rounds 5 --frames 6 > $O/tile_b.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config c --env RTRT_POOL_ROT --variants 1,0 --rounds 4 --frames 5 > $O/rot_c.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab.py --config d --env RTRT_POOL_ILV --variants 0,3 --rounds 3 --frames 5 > $O/rotilv_d.txt 2>&1 || exit $?
for f in tile_b rot_c rotilv_d; do grep -h "^{" $O/$f.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$f', {k: round(v['median'], 4) for k, v in d['ms'].items()})"; done
unset RTRT_LIB
for c in d c b a; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['ms_per_step_median'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
