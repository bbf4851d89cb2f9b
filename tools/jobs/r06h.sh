#!/usr/bin/env bash
# round 6 GPU job h: gloo rehearsals of the gather-aware multi-rank path with more ranks (sharing the
# one GPU, every gathered frame verified) and a second box's driver command
set -uo pipefail
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 400 python bench.py --gpus 4 --backend gloo --config d --steps 10 --warmup 8 --warm-ms 100 --verify \
  --no-cpu-baseline --dist-timeout 300 > $O/gloo_rehearsal_d_n4.json 2> $O/gloo_rehearsal_d_n4.err || exit $?
python3 -c "import json; d=json.loads(open('$O/gloo_rehearsal_d_n4.json').read().strip().splitlines()[-1]); print('gloo n4', d['verify']['frames_checked'], d['verify']['mismatched'], d['gather']['root_strip'], d['config']['strips'], [r['strip'] for r in d['ranks']])"
timeout -k 10 400 python bench.py --gpus 3 --backend gloo --config c --steps 10 --warmup 8 --warm-ms 100 --verify \
  --no-cpu-baseline --no-alt-dispatch --dist-timeout 300 > $O/gloo_rehearsal_c_n3.json 2> $O/gloo_rehearsal_c_n3.err || exit $?
python3 -c "import json; d=json.loads(open('$O/gloo_rehearsal_c_n3.json').read().strip().splitlines()[-1]); print('gloo n3', d['verify']['frames_checked'], d['verify']['mismatched'], d['gather']['root_strip'], d['config']['strips'], [r['strip'] for r in d['ranks']])"
for i in 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_command_d_$i.json 2> $O/driver_command_d_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/driver_command_d_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('driver', $i, d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
