"""Can two ranks share the one GPU of the box over the nccl (RCCL) backend?  If so, bench.py's
RCCL gather path (batch_isend_irecv on the NCCL stream, the link probe, the per-frame gather
events) can run on the one-GPU box.  Run under torch.distributed.run --nproc-per-node 2."""
import os
import time

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
t0 = time.time()
dist.init_process_group("nccl", device_id=dev)
x = torch.full((4,), float(rank + 1), device=dev)
dist.all_reduce(x)
print(f"rank {rank}: all_reduce {x.tolist()} ({time.time() - t0:.1f} s)", flush=True)
n = 16 << 20
buf = torch.full((n // 4,), float(rank), device=dev)
for it in range(3):
    torch.cuda.synchronize()
    dist.barrier()
    t = time.perf_counter()
    if rank == 0:
        ops = [dist.P2POp(dist.irecv, buf, 1)]
    else:
        ops = [dist.P2POp(dist.isend, buf, 0)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"rank {rank}: p2p 16 MiB {dt * 1e3:.3f} ms ({n / dt / 1e9:.1f} GB/s), value {buf[0].item()}", flush=True)
dist.destroy_process_group()
