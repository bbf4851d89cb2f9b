# pipelined bench with the A/B library: pool interleave 0 vs 3 (alternating runs)
O=gpurun_out/r02z6; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
for i in 1 2 3; do
  for k in 0 3; do
    RTRT_POOL_ILV=$k timeout -k 10 200 python bench.py --steps 40 --warmup 8 --no-cpu-baseline > $O/b_${k}_$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/b_${k}_$i.json'));print('ilv $k', d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'])"
  done
done
