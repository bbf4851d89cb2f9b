# r03ab: bench lines of the batched configs with the per-frame counter files attached (a, b: 400 frames)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab; mkdir -p $O
for cs in "a 400" "b 400" "c 100"; do set -- $cs
  timeout -k 10 300 python -u bench.py --config $1 --steps $2 > $O/bench_$1.json 2> $O/bench_$1.err || { tail $O/bench_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], d['ms_per_step_median'], r['kernel_ms'], r['frac'], r['hbm']['frac'], r['traffic'], r.get('valu_issue'), d.get('per_frame_dispatch',{}).get('ms_per_step'))"
done
