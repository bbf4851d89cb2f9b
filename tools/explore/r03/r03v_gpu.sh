# r03v: final post-process form (in-tree) — full GPU suite, smoke, frame A/B vs round-3 post (build/old)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }; tail -1 $O/t.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }; tail -1 $O/smoke.txt
for i in 1 2 3; do
  for v in old new; do
    if [ $v = new ]; then unset RTRT_LIB; else export RTRT_LIB=build/$v/librtrt.so; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print('$v', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
