# r03ak: the evidence set on the final in-tree build (f0c6c623ef3b): smoke, the driver's bench command, rocprof
# kernel traces, PMC and SQ passes, the N = 8 strip estimate at (d), the gloo N = 4 rehearsal
set -o pipefail
export TMPDIR=/tmp
TAG=r03ak
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('driver bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline_post']['kernel_ms'])"
timeout -k 10 600 bash tools/profile_box.sh $TAG d 20 > $O/profile_box.txt 2>&1 || { tail -20 $O/profile_box.txt; exit 1; }
timeout -k 10 600 bash tools/pmc_config.sh $TAG d ao_batch > $O/sq_d.txt 2>&1 || { tail $O/sq_d.txt; exit 1; }
tail -2 $O/sq_d.txt | cut -c1-300
timeout -k 10 300 python -u tools/strip_scaling.py --config d --n 8 --frames 20 --calibrate --warm-ms 300 > $O/strip_scaling_n8_calibrated.txt 2>&1 || exit 1
tail -1 $O/strip_scaling_n8_calibrated.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 4 --backend gloo --steps 6 --warmup 8 --no-cpu-baseline > $O/gloo_n4.json 2> $O/gloo_n4.err || { tail -20 $O/gloo_n4.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/gloo_n4.json') if l.startswith('{')][-1]); print('gloo', d['value'], d['verify'], d['collective'], d['config']['strips'])"
