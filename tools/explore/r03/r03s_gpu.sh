# r03s: post-process history prefetch distance PF (1..3) and EARLY (first slots issued before the spatial filter) vs in-tree (old)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s; mkdir -p $O
for v in p1e0 p2e1 p3e0; do
RTRT_LIB=build/$v/librtrt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adversarial.py -q -x --timeout 200 --timeout-method thread > $O/t_$v.txt 2>&1 || { tail $O/t_$v.txt; exit 1; }; echo $v $(tail -1 $O/t_$v.txt)
done
for i in 1 2; do
  for v in old p1e0 p1e1 p2e0 p2e1 p3e0; do
    export RTRT_LIB=build/$v/librtrt.so
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
