#!/usr/bin/env bash
# A/B of an environment switch on the pipelined config-(d) bench: GPU suite with the switch
# on, then 3 interleaved bench runs each way.   tools/explore/ab_env.sh NAME=VALUE
set -o pipefail
KV=$1
O=gpurun_out/r01k/env; mkdir -p $O
env "$KV" timeout -k 10 250 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$? $(tail -1 $O/tests.log)"
for r in 1 2 3; do
  for on in 0 1; do
    if [ $on = 1 ]; then E="$KV"; else E="RTRT_NONE=0"; fi
    env "$E" timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > $O/b_${on}_$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/b_${on}_$r.json'));print('on=$on', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
