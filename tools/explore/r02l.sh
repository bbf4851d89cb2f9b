set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "phong or hybrid or mode_parity or golden or fullsize or image or max_depth or group" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in b a; do
  timeout -k 10 200 python tools/ab.py --config $c --libs build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so --rounds 5 --frames 40 > $O/ab_$c.txt 2>&1 || exit $?
  grep -o '"ms": {.*}}' $O/ab_$c.txt
done
