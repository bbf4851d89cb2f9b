# r03u: post-process spatial stage with every neighbour requested in one round trip (p1s1) vs PF=1 only (p1e0) and in-tree (old)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03u; mkdir -p $O
for v in p1s1; do
RTRT_LIB=build/$v/librtrt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adversarial.py -q -x --timeout 200 --timeout-method thread > $O/t_$v.txt 2>&1 || { tail $O/t_$v.txt; exit 1; }; echo $v $(tail -1 $O/t_$v.txt)
done
for i in 1 2 3; do
  for v in old p1e0 p1s1; do
    export RTRT_LIB=build/$v/librtrt.so
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
