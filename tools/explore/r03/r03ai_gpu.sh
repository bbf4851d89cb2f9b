# r03ai: the bounce-round A/B of r03ah (head = 6d4f894, c2, bg, new = in-tree 2f31c46) and the round's evidence
# set on the in-tree build (tools/round_profile.sh steps): suite, A/B, smoke, driver bench, rocprof, PMC, SQ,
# strip-scaling estimates, gloo N = 4 rehearsal, then the alternating bench pairs
set -o pipefail
export TMPDIR=/tmp
TAG=r03ai
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
L=build/head/librtrt.so,build/c2/librtrt.so,build/bg/librtrt.so,real_time_ray_tracer_amd/librtrt.so
for c in d c e; do
timeout -k 10 300 python -u tools/ab.py --config $c --libs $L --rounds $([ $c = e ] && echo 3 || echo 8) --frames $([ $c = e ] && echo 2 || echo 6) --time-from 1 > $O/ab_ao_$c.txt 2>&1 || { tail -20 $O/ab_ao_$c.txt; exit 1; }
tail -1 $O/ab_ao_$c.txt | cut -c1-400
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('driver bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline_post']['kernel_ms'])"
timeout -k 10 600 bash tools/profile_box.sh $TAG d 20 > $O/profile_box.txt 2>&1 || { tail -20 $O/profile_box.txt; exit 1; }
timeout -k 10 600 bash tools/pmc_config.sh $TAG d ao_batch > $O/sq_d.txt 2>&1 || { tail $O/sq_d.txt; exit 1; }
tail -2 $O/sq_d.txt
timeout -k 10 300 python -u tools/strip_scaling.py --config d --n 4 --frames 20 --calibrate --warm-ms 300 > $O/strip_scaling_n4_calibrated.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/strip_scaling.py --config d --n 8 --frames 20 --calibrate --warm-ms 300 > $O/strip_scaling_n8_calibrated.txt 2>&1 || exit 1
tail -1 $O/strip_scaling_n8_calibrated.txt
timeout -k 10 600 python -u tools/strip_scaling.py --config e --n 8 --frames 4 --calibrate --warm-ms 300 > $O/strip_scaling_e_n8_calibrated.txt 2>&1 || exit 1
tail -1 $O/strip_scaling_e_n8_calibrated.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 4 --backend gloo --steps 6 --warmup 8 --no-cpu-baseline > $O/gloo_n4.json 2> $O/gloo_n4.err || { tail -20 $O/gloo_n4.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/gloo_n4.json') if l.startswith('{')][-1]); print('gloo', d['value'], d['verify'], d['collective'], d['config']['strips'])"
for i in 1 2; do
  for v in head c2 bg new; do
    if [ $v = new ]; then unset RTRT_LIB; else export RTRT_LIB=build/$v/librtrt.so; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
