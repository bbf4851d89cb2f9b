# r04d: HEAD (cheaper det_sin) GPU suite; AO A/B against the build before it (59678ff, outputs differ
# by design); post-process tile-shape variants; the driver's bench command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }; tail -6 $O/gpu_tests.txt
L=build/oldsin/librtrt.so,real_time_ray_tracer_amd/librtrt.so
for c in d c; do
  timeout -k 10 300 python -u tools/ab.py --config $c --libs $L --rounds 8 --frames 6 --allow-diff > $O/ab_sin_$c.txt 2>&1 || { tail -20 $O/ab_sin_$c.txt; exit 1; }
  tail -1 $O/ab_sin_$c.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', {k: round(v['median'],4) for k,v in d['ms'].items()})"
done
L=real_time_ray_tracer_amd/librtrt.so,build/v_post64x4/librtrt.so,build/v_post128x2/librtrt.so,build/v_post64x4r0/librtrt.so,build/v_post64x4r15/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --prog 2 --libs $L --rounds 6 --frames 10 --time-from 8 > $O/ab_post.txt 2>&1 || { tail -20 $O/ab_post.txt; exit 1; }
tail -1 $O/ab_post.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('post', {k: round(v['median'],4) for k,v in d['ms'].items()})"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_d.json 2> $O/bench_d.err || { tail $O/bench_d.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_d.json')); r=d['roofline']; print('bench d', d['value'], d['ms_per_step'], d['ms_per_step_median'], r['kernel_ms'], r['frac'], d['roofline_post']['kernel_ms'], d['cpu_baseline']['value'])"
L=real_time_ray_tracer_amd/librtrt.so,build/v_b1pipe/librtrt.so,build/v_b1rl/librtrt.so
for c in d c; do
  timeout -k 10 300 python -u tools/ab.py --config $c --libs $L --rounds 8 --frames 6 > $O/ab_b1pipe_$c.txt 2>&1 || { tail -20 $O/ab_b1pipe_$c.txt; exit 1; }
  tail -1 $O/ab_b1pipe_$c.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b1pipe $c', {k: round(v['median'],4) for k,v in d['ms'].items()})"
done
for i in 1 2 3; do
  for v in tree hytpb2 hytpb4; do
    if [ $v = tree ]; then unset RTRT_LIB; else export RTRT_LIB=build/v_$v/librtrt.so; fi
    timeout -k 10 200 python -u bench.py --config b --steps 400 --no-cpu-baseline > $O/bench_b_${v}_$i.json 2> $O/bench_b_${v}_$i.err || { tail $O/bench_b_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_b_${v}_$i.json')); print('b $v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
unset RTRT_LIB
