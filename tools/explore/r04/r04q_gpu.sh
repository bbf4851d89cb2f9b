# r04q: the driver's command three times on one box (final build): the headline's run-to-run spread
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { tail $O/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); r=d['roofline']; print('driver bench', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], r['kernel_ms'], r['frac'], d['roofline_post']['kernel_ms'], d['roofline_post']['traffic_over_model'], d['cpu_baseline']['value'])"
done
