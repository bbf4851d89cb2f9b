# r03r: post-process history slot loads: colour with keys (pf1) / next slot prefetched (pf2) vs in-tree (old)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r; mkdir -p $O
RTRT_LIB=build/pf2/librtrt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "post or pipelined or mode1 or ring" > $O/t.txt 2>&1; tail -1 $O/t.txt
for i in 1 2; do
  for v in old pf1 pf2; do
    export RTRT_LIB=build/$v/librtrt.so
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
