#!/usr/bin/env bash
# round 6 GPU job pm: wave issue priority (s_setprio 1) by phase of ao_batch_kernel (RT_PRIO_MODE
# 1 first bounce, 2 bounce rounds, 3 both, 4 all of prepare) against production: per-launch A/Bs
# at (d), (c), (e) (images must be identical), then pipelined (d) frames in alternating processes
set -uo pipefail
O=gpurun_out/r06px; mkdir -p $O
L=real_time_ray_tracer_amd/librtrt.so,build/v_px1/librtrt.so,build/v_px2/librtrt.so
for c in d c; do
  timeout -k 10 400 python -u tools/ab.py --config $c --rounds 3 --frames 3 --libs $L > $O/ab_$c.txt 2>&1 || exit $?
  tail -1 $O/ab_$c.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', {k.split('/')[-2]: round(v['median'],4) for k,v in d['ms'].items()})"
  echo "mismatches: $(grep -c identical=False $O/ab_$c.txt)"
done
for i in 1 2 3; do
  for v in prod px1 px2; do
    lib=build/v_$v/librtrt.so; [ $v = prod ] && lib=real_time_ray_tracer_amd/librtrt.so
    RTRT_LIB=$lib timeout -k 10 120 python -u tools/explore/pipeline_floor.py --config d > $O/pipe_${v}_$i.txt 2>&1 || exit $?
    echo "$v $i $(tail -1 $O/pipe_${v}_$i.txt)"
  done
done
