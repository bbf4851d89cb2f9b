# r03k: GPU suite; configs a / b / c bench lines (batched + one launch per frame); SQ counters of
# hybrid_kernel at config b (tools/pmc_config.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for c in a b c; do
  st=400; [ $c = c ] && st=40
  timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 8 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d.get('per_frame_dispatch'), d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['hbm']['frac'])"
done
timeout -k 10 600 bash tools/pmc_config.sh r03k b hybrid_kernel > $O/sq_b.txt 2>&1 || { tail $O/sq_b.txt; exit 1; }
tail -3 $O/sq_b.txt
timeout -k 10 300 python -u bench.py --config ref --steps 200 --warmup 10 --no-cpu-baseline > $O/bench_ref.json 2> $O/bench_ref.err || { tail $O/bench_ref.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_ref.json')); print('ref', d['value'], d['ms_per_step'], d['ssbo_path'])"
