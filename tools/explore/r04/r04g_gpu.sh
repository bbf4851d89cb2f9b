# r04g: hybrid longest-first tile schedule: its tests first, then the GPU suite; per-frame (b), (a)
# and a mode-4 scene with planes (p is mode 1) against row order (the previous build) and the
# reverse-order variant, alternating processes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedule.py -v -x --timeout 200 --timeout-method thread > $O/sched_tests.txt 2>&1 || { tail -40 $O/sched_tests.txt; exit 1; }; tail -4 $O/sched_tests.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }; tail -3 $O/gpu_tests.txt
for i in 1 2 3; do
  for v in old tree hyrev; do
    if [ $v = tree ]; then unset RTRT_LIB; elif [ $v = old ]; then export RTRT_LIB=build/old/librtrt.so; else export RTRT_LIB=build/v_$v/librtrt.so; fi
    for c in b; do
      timeout -k 10 200 python -u bench.py --config $c --steps 800 --no-cpu-baseline --no-alt-dispatch > $O/bench_${c}_${v}_$i.json 2> $O/bench_${c}_${v}_$i.err || { tail $O/bench_${c}_${v}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_${c}_${v}_$i.json')); print('$c $v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
unset RTRT_LIB
timeout -k 10 200 python -u bench.py --config b --frame-batch 8 --steps 800 --no-cpu-baseline --no-alt-dispatch > $O/bench_b_batched.json 2> $O/bench_b_batched.err && python3 -c "import json; d=json.load(open('$O/bench_b_batched.json')); print('b batched', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
