#!/usr/bin/env bash
# round 6, last source (6e9311b65f39: comment-only change from 4f72333e042d, the same ISA): smoke,
# the driver's command twice and the (e) bench line, with this build's counter files in profiles/
set -uo pipefail
O=gpurun_out/r06zg; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_command_d_$i.json 2> $O/driver_command_d_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/driver_command_d_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('driver', $i, d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic_on_this_build'), d['build'])"
done
timeout -k 10 600 python bench.py --config e > $O/bench_e.json 2> $O/bench_e.err || exit $?
python3 -c "import json; d=json.loads(open('$O/bench_e.json').read().strip().splitlines()[-1]); r=d['roofline']; print('e', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic_on_this_build'))"
