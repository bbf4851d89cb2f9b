# r03w: batched first bounce with the per-ray pre-test on the f32 MFMA (in-tree, min 8 survivors; m4 / m16) vs HEAD (old)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 60 build/mfma_pretest > $O/micro.txt 2>&1 || { cat $O/micro.txt; exit 1; }; tail -1 $O/micro.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adversarial.py -q -x --timeout 200 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }; tail -1 $O/t.txt
L=build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so,build/m4/librtrt.so,build/m16/librtrt.so
for c in d c; do
timeout -k 10 300 python -u tools/ab.py --config $c --libs $L --rounds 6 --frames 6 --time-from 1 > $O/ab_ao_$c.txt 2>&1 || { tail -20 $O/ab_ao_$c.txt; exit 1; }
tail -4 $O/ab_ao_$c.txt
done
for i in 1 2; do
  for v in old new; do
    if [ $v = new ]; then unset RTRT_LIB; else export RTRT_LIB=build/$v/librtrt.so; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
