#!/usr/bin/env bash
# round 5, end-of-round build: bench + rocprof for e ref p, the driver's command three times
# (post-process spread), smoke() and the whole GPU suite
set -uo pipefail
O=gpurun_out/r05last
mkdir -p $O
bash tools/round_profile.sh bench r05last e ref p > gpurun_out/r05last_bench_2.log 2>&1 &&
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_d_$i.json 2> $O/driver_d_$i.err || exit 1
done &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=5 > $O/gpu_tests.txt 2>&1
rc=$?
tail -20 gpurun_out/r05last_bench_2.log
for i in 1 2 3; do python3 -c "import json; d=json.loads(open('$O/driver_d_$i.json').read().strip().splitlines()[-1]); print('driver', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('roofline_post',{}).get('kernel_ms'))"; done
tail -2 $O/smoke.txt
tail -2 $O/gpu_tests.txt
exit $rc
