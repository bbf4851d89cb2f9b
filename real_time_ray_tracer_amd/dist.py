"""Multi-GPU row strips + gather of the image strips to rank 0.

SURVEY.md §8e: every trace pixel is independent, so a frame is cut into N contiguous row
strips, one per GPU (one process per GPU, torch.distributed over RCCL/xGMI).  Each rank
keeps its own g-buffer ring for its strip plus a 1-row halo (rendered redundantly, so the
post-process needs no exchange); the only collective is the per-frame gather of the final
image strips into rank 0.  Strip bounds are balanced by a per-row cost profile (work
estimates from the kernels' row counters), because sky rows are far cheaper than ground rows,
then calibrated once against each strip's measured kernel time and re-balanced.

The gather is pipelined: frame k's strip is gathered (async, RCCL stream) while frame k+1
renders into the other of two image buffers.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def equal_bounds(H: int, n: int) -> list[int]:
    return [round(i * H / n) for i in range(n + 1)]


def balanced_bounds(row_cost: np.ndarray, n: int, min_rows: int | None = None) -> list[int]:
    """Contiguous strips of (nearly) equal total cost, row_cost[y] >= 0 for every frame row:
    the C ABI's host-only planner (rt_plan_strips, no GPU call), shared with the one-process
    rt_group path, so both drivers split frames identically.  It needs librtrt.so built (it
    loads without a GPU).  min_rows is deprecated: every strip has at least one row, and a
    larger minimum is no longer supported (it raises rather than being ignored)."""
    from .host import plan_strips

    if min_rows is not None:
        import warnings

        warnings.warn("balanced_bounds(min_rows=...) is deprecated; strips have >= 1 row", DeprecationWarning,
                      stacklevel=2)
        if min_rows > 1:
            raise ValueError("min_rows > 1 is no longer supported by rt_plan_strips")
    return plan_strips(row_cost, n)


def strip_cost(bounds: list[int], row_cost: np.ndarray) -> list[float]:
    return [float(np.sum(row_cost[bounds[i]:bounds[i + 1]])) for i in range(len(bounds) - 1)]


def calibrate_row_cost(bounds: list[int], row_cost: np.ndarray, strip_time: list[float]) -> np.ndarray:
    """Rescale the modelled per-row cost so every strip's total equals its measured time
    (keeping the row shape inside each strip): corrects the cost model (setup vs test cost,
    per-rank overheads) before a second balancing pass (rt_calibrate_row_cost)."""
    from .host import calibrate_row_cost as _cal

    return _cal(bounds, row_cost, strip_time)


def imbalance(strip_time: list[float]) -> float:
    """max / mean - 1 of the per-strip times."""
    t = np.asarray(strip_time, np.float64)
    return float(t.max() / max(t.mean(), 1e-30) - 1.0)


@dataclass
class StripPlan:
    W: int
    H: int
    bounds: list[int]

    @property
    def n(self) -> int:
        return len(self.bounds) - 1

    def rows(self, rank: int) -> tuple[int, int]:
        return self.bounds[rank], self.bounds[rank + 1]

    @property
    def max_rows(self) -> int:
        return max(self.bounds[i + 1] - self.bounds[i] for i in range(self.n))

    def assemble(self, padded_strips: list) -> "np.ndarray | object":
        """Concatenate the gathered (padded) strips into the [H][W][4] frame."""
        parts = [padded_strips[i][: self.bounds[i + 1] - self.bounds[i]] for i in range(self.n)]
        if isinstance(parts[0], np.ndarray):
            return np.concatenate(parts, 0)
        import torch

        return torch.cat(parts, 0)


class StripGather:
    """Gathers every rank's image strip into rank 0's [H][W][4] frame with point-to-point
    transfers of exactly the strip's rows (torch.distributed batch_isend_irecv: grouped RCCL
    send/recv on GPUs, gloo on CPU).  Strip r lands directly in rows [bounds[r], bounds[r+1])
    of the frame, and rank 0 renders its own strip straight into its rows, so there is no
    padding and no assembly copy (cost-balanced strips differ in height by up to ~3x, and a
    padded gather would move max_rows for every rank)."""

    def __init__(self, plan: StripPlan, rank: int, device, nbuf: int = 2, root: int = 0, host_staging: bool = False):
        """host_staging: gather through host copies (gloo rehearsal of the GPU path)."""
        import torch

        self.plan, self.rank, self.root, self.nbuf = plan, rank, root, nbuf
        self.host_staging = host_staging
        self.device = device
        W = plan.W
        r0, r1 = plan.rows(rank)
        fdev = "cpu" if host_staging else device
        self.frames = []
        if rank == root:
            self.frames = [torch.zeros((plan.H, W, 4), dtype=torch.float32, device=fdev) for _ in range(nbuf)]
        if rank == root and not host_staging:
            self.strips = [f[r0:r1] for f in self.frames]  # contiguous rows of the frame
        else:
            self.strips = [torch.zeros((r1 - r0, W, 4), dtype=torch.float32, device=device) for _ in range(nbuf)]
        self.pending = [None] * nbuf

    def strip(self, k: int):
        """Image buffer frame k renders into (waits for the gather that last used it)."""
        i = k % self.nbuf
        self._wait(i)
        return self.strips[i]

    def _wait(self, i: int):
        if self.pending[i] is not None:
            for w in self.pending[i]:
                w.wait()
            self.pending[i] = None

    def gather(self, k: int):
        import torch.distributed as dist

        i = k % self.nbuf
        ops = []
        if self.rank == self.root:
            if self.host_staging:  # rank 0's own strip into the host frame
                r0, r1 = self.plan.rows(self.rank)
                self.frames[i][r0:r1].copy_(self.strips[i].cpu())
            for r in range(self.plan.n):
                if r != self.root:
                    a, b = self.plan.rows(r)
                    ops.append(dist.P2POp(dist.irecv, self.frames[i][a:b], r))
        else:
            src = self.strips[i].cpu() if self.host_staging else self.strips[i]
            ops.append(dist.P2POp(dist.isend, src, self.root))
        self.pending[i] = dist.batch_isend_irecv(ops) if ops else None

    def finish(self):
        for i in range(self.nbuf):
            self._wait(i)

    def frame(self, k: int):
        """Rank 0: the [H][W][4] frame of frame k (after finish())."""
        if self.rank != self.root:
            return None
        return self.frames[k % self.nbuf]


def init_process_group(backend: str, device=None, timeout_s: float = 300.0) -> None:
    """torch.distributed.init_process_group with a finite timeout: every later collective of a
    rank whose peer has died raises after timeout_s (gloo: the collective's own timeout; NCCL:
    the watchdog), instead of blocking until an outside time limit kills the job."""
    from datetime import timedelta

    import torch.distributed as dist

    kw = {"timeout": timedelta(seconds=timeout_s)}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)


def run_rank(fn, *args, **kwargs):
    """Run one rank's body; on any exception print the rank and the error to stderr and exit
    the process with status 1 at once (os._exit: no atexit / process-group teardown that could
    block on dead peers).  The other ranks then fail at their next collective, within the
    process group's timeout, and exit the same way, so a failed multi-GPU run ends with every
    rank non-zero and the failing rank named."""
    import os
    import sys
    import traceback

    try:
        return fn(*args, **kwargs)
    except BaseException as e:  # noqa: BLE001 - every failure must end the rank loudly
        if isinstance(e, SystemExit) and not e.code:
            raise
        rank = os.environ.get("RANK", "0")
        world = os.environ.get("WORLD_SIZE", "1")
        print(f"[rank {rank}/{world}] failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        traceback.print_exc(file=sys.stderr)
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)
