# Phong 4 frames per block, hybrid 1 without the frame loop: parity tests, then configs a/b against the previous build (old)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in old new; do
    L=real_time_ray_tracer_amd/librtrt.so; [ $v = new ] || L=build/$v/librtrt.so
    for c in a b; do
      RTRT_LIB=$L timeout -k 10 120 python bench.py --config $c --steps 800 --warmup 16 --no-cpu-baseline > $O/${c}_${v}_$r.json 2> $O/${c}_${v}_$r.err || exit $?
      python3 -c "
import json; d=json.loads(open('$O/${c}_${v}_$r.json').read().strip().splitlines()[-1])
print('$c $v $r', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['roofline'].get('kernel_ms'))"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_a -o run -- \
  python3 bench.py --config a --steps 80 --warmup 8 --no-cpu-baseline > $O/kt_bench_a.json 2> $O/kt_a.err || exit $?
