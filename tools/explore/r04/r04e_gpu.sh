# r04e: GPU suite on the tree (64x4 post tiles, distinct-table uploads); pipelined frame (d) and
# per-frame (a)/(b) against the previous build (build/old = 082bb5f), alternating processes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }; tail -3 $O/gpu_tests.txt
for i in 1 2 3; do
  for v in old tree; do
    if [ $v = tree ]; then unset RTRT_LIB; else export RTRT_LIB=build/old/librtrt.so; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_d_${v}_$i.json 2> $O/bench_d_${v}_$i.err || { tail $O/bench_d_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_d_${v}_$i.json')); print('d $v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
    for c in a b; do
      timeout -k 10 200 python -u bench.py --config $c --steps 400 --no-cpu-baseline > $O/bench_${c}_${v}_$i.json 2> $O/bench_${c}_${v}_$i.err || { tail $O/bench_${c}_${v}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_${c}_${v}_$i.json')); print('$c $v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('batched_dispatch', {}).get('value'))"
    done
  done
done
unset RTRT_LIB
