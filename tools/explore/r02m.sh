# A/B (libs, separate processes, alternating): Phong/hybrid multi-frame launches with 2 (new), 4, 8
# frames per block vs one frame per block (build/old); configs b and a; the parity tests run first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in old new fpb4 fpb8; do
    L=real_time_ray_tracer_amd/librtrt.so; [ $v = new ] || L=build/$v/librtrt.so
    for c in b a; do
      RTRT_LIB=$L timeout -k 10 120 python bench.py --config $c --steps 800 --warmup 16 --no-cpu-baseline > $O/${c}_${v}_$r.json 2> $O/${c}_${v}_$r.err || exit $?
      python3 -c "
import json; d=json.loads(open('$O/${c}_${v}_$r.json').read().strip().splitlines()[-1])
print('$c $v $r', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['roofline'].get('kernel_ms'))"
    done
  done
done
