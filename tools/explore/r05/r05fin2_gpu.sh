#!/usr/bin/env bash
# round 5, final build: bench + rocprof for e ref p, then the driver's command three times
# (post-process spread) and smoke()
set -uo pipefail
O=gpurun_out/r05fin
mkdir -p $O
bash tools/round_profile.sh bench r05fin e ref p > gpurun_out/r05fin_bench_2.log 2>&1 &&
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_d_$i.json 2> $O/driver_d_$i.err || exit 1
done &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
rc=$?
tail -20 gpurun_out/r05fin_bench_2.log
for i in 1 2 3; do python3 -c "import json; d=json.loads(open('$O/driver_d_$i.json').read().strip().splitlines()[-1]); print('driver', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('roofline_post',{}).get('kernel_ms'))"; done
tail -2 $O/smoke.txt
exit $rc
