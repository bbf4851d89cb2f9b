# XCD balance: rotate each row's pools by the row index (RTRT_POOL_ROT=1), with/without interleave 3
O=gpurun_out/r02z9; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/ab.py --config d --env RTRT_POOL_ROT --variants 0,1,0,1 --rounds 3 --frames 5 > $O/rot_d.txt 2>&1 || exit $?
for rot in 0 1; do
  RTRT_POOL_ROT=$rot timeout -k 10 250 python tools/strip_scaling.py --config d --n 8 --frames 24 --mode 2 --multi > $O/m2_multi_rot$rot.txt 2>&1 || exit $?
  RTRT_POOL_ROT=$rot timeout -k 10 250 python tools/strip_scaling.py --config d --n 8 --frames 24 > $O/m1_pipe_rot$rot.txt 2>&1 || exit $?
done
grep -h "^{" $O/rot_d.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('rot_d', {k: round(v['median'], 4) for k, v in d['ms'].items()})"
tail -n 3 $O/m2_multi_rot*.txt $O/m1_pipe_rot*.txt
