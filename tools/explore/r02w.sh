O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b20.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/b100.json 2>/dev/null || exit $?
for f in b20 b100; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['ms_per_step'], d['ms_per_step_median'], d['frame_intervals_ms'][:30])"; done
