#!/usr/bin/env bash
# round 6 GPU job d: hybrid_kernel at (b) with 4 tiles per block in sequence (a quarter of the waves)
# against production (schedule on) and production with the schedule off, alternating processes
set -uo pipefail
O=gpurun_out/r06d; mkdir -p $O
for i in 1 2; do
  for v in prod noschd tpb4; do
    case $v in
      prod) timeout -k 10 120 python3 bench.py --config b --no-cpu-baseline --no-alt-dispatch > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $? ;;
      noschd) timeout -k 10 120 python3 bench.py --config b --no-cpu-baseline --no-alt-dispatch --no-tile-schedule > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $? ;;
      tpb4) RTRT_LIB=build/v_hytpb4/librtrt.so timeout -k 10 120 python3 bench.py --config b --no-cpu-baseline --no-alt-dispatch > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $? ;;
    esac
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
