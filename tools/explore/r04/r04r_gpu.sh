# r04r: pipelined frame (d) with the post-process stream at a higher priority than the AO streams
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for i in 1 2 3; do
  for pr in 0 -1 -2; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --out-stream-priority=$pr > $O/d_p${pr}_$i.json 2> $O/d_p${pr}_$i.err || { tail $O/d_p${pr}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/d_p${pr}_$i.json')); print('d prio $pr', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
