#!/usr/bin/env bash
# round 6 final evidence (build with the pool-start priority), part 2b: every config's bench line with its CPU baseline, rocprof
# --kernel-trace --stats of the same command and the burst check; one-GPU strip estimates
set -uo pipefail
O=gpurun_out/r06zj; mkdir -p $O
timeout -k 10 900 bash tools/round_profile.sh bench r06zj d c b a p ref > $O/bench_all.log 2>&1 || { tail -20 $O/bench_all.log; exit 1; }
grep -v "^ \|amdgpu" $O/bench_all.log | tail -30
timeout -k 10 200 python -u tools/strip_scaling.py --config d --n 8 --frames 20 --calibrate --warm-ms 300 \
  --save-profile $O/strip_scaling_d_n8.json > $O/strip_scaling_d_n8_calibrated.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/strip_scaling.py --config d --n 4 --frames 20 --calibrate --warm-ms 300 \
  --save-profile $O/strip_scaling_d_n4.json > $O/strip_scaling_d_n4_calibrated.txt 2>&1 || exit $?
grep -v amdgpu $O/strip_scaling_d_n8_calibrated.txt | tail -4
grep -v amdgpu $O/strip_scaling_d_n4_calibrated.txt | tail -4
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --config d --steps 10 --warmup 8 --warm-ms 100 --verify \
  --no-cpu-baseline --dist-timeout 200 > $O/gloo_rehearsal_d_n2.json 2> $O/gloo_rehearsal_d_n2.err || exit $?
python3 -c "import json; d=json.loads(open('$O/gloo_rehearsal_d_n2.json').read().strip().splitlines()[-1]); print('gloo n2', d['value'], d['verify'], d['gather']['root_strip'])"
