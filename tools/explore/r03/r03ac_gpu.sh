# r03ac: post-process history slots in pairs (build/pp) vs in-tree: parity subset + frame A/B at d (3 rounds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ac; mkdir -p $O
RTRT_LIB=build/pp/librtrt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adversarial.py -q -x --timeout 200 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }; tail -1 $O/t.txt
for i in 1 2 3; do
  for v in new pp; do
    if [ $v = new ]; then unset RTRT_LIB; else export RTRT_LIB=build/$v/librtrt.so; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
