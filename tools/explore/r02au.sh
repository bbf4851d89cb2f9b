# A/B repeat at config d (HEAD vs working tree), 2 x 6 rounds
O=gpurun_out/r02au; mkdir -p $O
L=build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so
for k in 1 2; do
  timeout -k 10 250 python tools/ab.py --config d --libs $L --rounds 5 --frames 5 > $O/d$k.txt 2>&1 || exit $?
  grep -h "^{" $O/d$k.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('d', {k.split('/')[0]: round(v['median'], 5) for k, v in d['ms'].items()})"
done
timeout -k 10 250 python tools/ab.py --config c --libs $L --rounds 6 --frames 5 > $O/c.txt 2>&1 || exit $?
grep -h "^{" $O/c.txt | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('c', {k.split('/')[0]: round(v['median'], 5) for k, v in d['ms'].items()})"
