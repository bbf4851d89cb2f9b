set -uo pipefail
O=gpurun_out/r06pp; mkdir -p $O
for i in 1 2 3; do
  for v in prod pp1 pp2; do
    lib=build/v_$v/librtrt.so; [ $v = prod ] && lib=real_time_ray_tracer_amd/librtrt.so
    RTRT_LIB=$lib timeout -k 10 120 python -u tools/explore/pipeline_floor.py --config d > $O/pipe_${v}_$i.txt 2>&1 || exit $?
    echo "$v $i $(tail -1 $O/pipe_${v}_$i.txt)"
  done
done
