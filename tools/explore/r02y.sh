set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in c d; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['ms_per_step_median'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
