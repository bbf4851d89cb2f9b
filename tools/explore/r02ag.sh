# gloo rehearsal of the N=2 path with clock settling (2 ranks share the GPU), verify on; default bench d
set -o pipefail
O=gpurun_out/r02ag; mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 6 --warmup 3 --backend gloo --verify --no-cpu-baseline > $O/gloo_n2.json 2> $O/gloo_n2.err || exit $?
python3 -c "import json;d=json.load(open('$O/gloo_n2.json'));print('gloo n2', d['value'], d['settle_frames'], d['verify'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_d.json 2> $O/bench_d.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_d.json'));print('d',d['value'],d['ms_per_step'],d['ms_per_step_median'],d['settle_frames'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['cpu_baseline']['value'])"
