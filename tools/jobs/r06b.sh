#!/usr/bin/env bash
# round 6 GPU job b: can RCCL run 2 ranks on the box's one GPU? (then the nccl gather path can be tested)
set -uo pipefail
O=gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29531 tools/explore/r06/nccl_one_gpu.py > $O/r06b_nccl_one_gpu.txt 2>&1
echo "rc=$?" >> $O/r06b_nccl_one_gpu.txt
tail -20 $O/r06b_nccl_one_gpu.txt
