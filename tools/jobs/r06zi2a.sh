#!/usr/bin/env bash
# round 6 final evidence (build with the pool-start priority), part 2a: the GPU suite, smoke, the driver's command three times, and the
# N = 2 gloo rehearsal of the multi-rank path (2 ranks on the one GPU, every gathered frame verified)
set -uo pipefail
O=gpurun_out/r06zi; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -12 $O/gpu_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
cat $O/smoke.txt | tail -2
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_command_d_$i.json 2> $O/driver_command_d_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/driver_command_d_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('driver', $i, d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic_on_this_build'), d.get('cpu_baseline', {}).get('value'))"
done
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --config d --steps 10 --warmup 8 --warm-ms 100 --verify \
  --no-cpu-baseline --dist-timeout 200 > $O/gloo_rehearsal_d_n2.json 2> $O/gloo_rehearsal_d_n2.err || exit $?
python3 -c "import json; d=json.loads(open('$O/gloo_rehearsal_d_n2.json').read().strip().splitlines()[-1]); print('gloo n2', d['value'], d['verify'], d['gather'])"
