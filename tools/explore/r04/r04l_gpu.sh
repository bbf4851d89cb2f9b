# r04l: on the final build: the driver's bench command, the one-GPU N = 8 strip estimates at (d)
# and (e), gloo rehearsals of the N > 1 path (N = 4 at (d); N = 2 at (b): strips with the
# hybrid tile schedule per rank), every gathered frame verified
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('driver bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline_post']['kernel_ms'], d['cpu_baseline']['value'])"
timeout -k 10 300 python -u tools/strip_scaling.py --config d --n 8 --frames 20 --calibrate --warm-ms 300 > $O/strip_scaling_n8_calibrated.txt 2>&1 || exit 1
tail -1 $O/strip_scaling_n8_calibrated.txt
timeout -k 10 500 python -u tools/strip_scaling.py --config e --n 8 --frames 4 --calibrate --warm-ms 300 > $O/strip_scaling_e_n8_calibrated.txt 2>&1 || exit 1
tail -1 $O/strip_scaling_e_n8_calibrated.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 4 --backend gloo --steps 6 --warmup 8 --no-cpu-baseline > $O/gloo_n4.json 2> $O/gloo_n4.err || { tail -20 $O/gloo_n4.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/gloo_n4.json') if l.startswith('{')][-1]); print('gloo d n4', d['value'], d['verify'], d['collective'], d['config']['strips'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 2 --config b --backend gloo --steps 40 --warmup 8 --no-cpu-baseline > $O/gloo_b_n2.json 2> $O/gloo_b_n2.err || { tail -20 $O/gloo_b_n2.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/gloo_b_n2.json') if l.startswith('{')][-1]); print('gloo b n2', d['value'], d['verify'], d['collective'], d['config']['strips'], d.get('tile_schedule'))"
