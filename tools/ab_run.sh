#!/usr/bin/env bash
# On the GPU box: full GPU suite, then interleaved A/B of build/old/librtrt.so (the previous
# build) against the current library at configs d and c.   tools/ab_run.sh <tag>
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/r01k
mkdir -p "$OUT"
timeout -k 10 250 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
rc=$?
tail -2 "$OUT/${TAG}_tests.log"
[ $rc -eq 0 ] || exit $rc
for c in d c; do
  timeout -k 10 200 python tools/ab.py --config $c --libs build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so --rounds 5 > "$OUT/ab_${TAG}_$c.txt" 2>&1 || exit $?
done
grep -h "^{" "$OUT/ab_${TAG}_d.txt" "$OUT/ab_${TAG}_c.txt" | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print(d['config'][:12], {k.split('/')[0]: round(v['median'], 4) for k, v in d['ms'].items()})"
echo "identical rounds: $(grep -c 'identical=True' "$OUT/ab_${TAG}_d.txt") (d) $(grep -c 'identical=True' "$OUT/ab_${TAG}_c.txt") (c)"
