# r03m3: frame-level A/B of the driver's bench command (alternating processes on one box) and a
# same-process AO-kernel A/B: old (round 2) / tlc0 (normals planes, no clusters <= 128 spheres) /
# nrm4 (interleaved normals, clusters) / nrm4tlc0 (interleaved, no clusters <= 128) / in-tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03m3; mkdir -p $O
timeout -k 10 300 python -u tools/ab.py --config d --libs build/old/librtrt.so,build/tlc0/librtrt.so,build/nrm4/librtrt.so,build/nrm4tlc0/librtrt.so,real_time_ray_tracer_amd/librtrt.so --rounds 6 --frames 6 --time-from 1 > $O/ab_ao_d.txt 2>&1 || { tail -20 $O/ab_ao_d.txt; exit 1; }
tail -1 $O/ab_ao_d.txt
for i in 1 2; do
  for v in old tlc0 nrm4 nrm4tlc0 new; do
    if [ $v = new ]; then unset RTRT_LIB; else export RTRT_LIB=build/$v/librtrt.so; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
