#!/usr/bin/env bash
# round 5j: the driver's bench command (pipelined frames) on the 6-wave and 7-wave AO builds, alternating
set -uo pipefail
O=gpurun_out/r05j
mkdir -p $O
for i in 1 2; do
  for v in w7 w6; do
    if [ $v = w6 ]; then LIBV=build/v_w6/librtrt.so; else LIBV=real_time_ray_tracer_amd/librtrt.so; fi
    RTRT_LIB=$LIBV timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
