# the driver's N>1 launch shape (torchrun, one rank per strip) rehearsed on a one-GPU box with gloo:
# every gathered frame checked against a whole-frame render on rank 0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02l; mkdir -p $O
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 5 --backend gloo --verify \
    > $O/gloo_n$n.json 2> $O/gloo_n$n.err || exit $?
  tail -c 400 $O/gloo_n$n.json
done
