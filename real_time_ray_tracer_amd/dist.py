"""Multi-GPU row strips + gather of the image strips to rank 0.

SURVEY.md §8e: every trace pixel is independent, so a frame is cut into N contiguous row
strips, one per GPU (one process per GPU, torch.distributed over RCCL/xGMI).  Each rank
keeps its own g-buffer ring for its strip plus a 1-row halo (rendered redundantly, so the
post-process needs no exchange); the only collective is the per-frame gather of the final
image strips into rank 0.  Strip bounds are balanced by a per-row cost profile (work
estimates from the kernels' row counters), because sky rows are far cheaper than ground rows,
then calibrated once against each strip's measured kernel time and re-balanced.

The gather is part of the plan: every non-root strip crosses one xGMI link into rank 0 each
frame, so the planner (rt_plan_strips_gather) chooses the bounds AND which strip rank 0 owns
(the root strip, rendered in place, never sent) to minimise max(render, per-link copy, root
ingest).  At config (d) that puts the large, cheap sky strip on rank 0.  Rank r > 0 renders the
r-th of the other strips in row order.

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


def gather_bounds(row_ms: np.ndarray, n: int, W: int, link_gbps: float, ingest_gbps: float):
    """rt_plan_strips_gather: (bounds, root strip, predicted {bound, render, link, ingest} ms) for a
    per-row cost profile in ms (calibrate_row_cost's output)."""
    from .host import plan_strips_gather

    return plan_strips_gather(row_ms, n, W, link_gbps, ingest_gbps)


def gather_bound(row_ms: np.ndarray, bounds: list[int], root_strip: int, W: int, link_gbps: float,
                 ingest_gbps: float) -> dict:
    from .host import strip_gather_bound

    return strip_gather_bound(row_ms, bounds, root_strip, W, link_gbps, ingest_gbps)


@dataclass
class StripPlan:
    """Row strips [bounds[i], bounds[i+1]) and their owners: rank 0 (the gather's root) owns
    strip root_strip, rank r > 0 the r-th of the others in row order."""
    W: int
    H: int
    bounds: list[int]
    root_strip: int = 0

    def __post_init__(self):
        if not 0 <= self.root_strip < self.n:
            raise ValueError(f"root strip {self.root_strip} outside 0..{self.n - 1}")

    @property
    def n(self) -> int:
        return len(self.bounds) - 1

    def strip_of(self, rank: int) -> int:
        """the strip index rank renders"""
        if rank == 0:
            return self.root_strip
        return rank - 1 if rank - 1 < self.root_strip else rank

    def rank_of(self, strip: int) -> int:
        if strip == self.root_strip:
            return 0
        return strip + 1 if strip < self.root_strip else strip

    def rows(self, rank: int) -> tuple[int, int]:
        i = self.strip_of(rank)
        return self.bounds[i], self.bounds[i + 1]

    def strip_bytes(self, rank: int) -> int:
        """bytes of rank's image strip (rgba32f rows): what it sends to rank 0 per frame (0 for rank 0)"""
        if rank == 0:
            return 0
        a, b = self.rows(rank)
        return (b - a) * self.W * 16

    @property
    def max_rows(self) -> int:
        return max(self.bounds[i + 1] - self.bounds[i] for i in range(self.n))

    def assemble(self, padded_strips: list) -> "np.ndarray | object":
        """Concatenate the gathered (padded) strips, indexed by rank, into the [H][W][4] frame."""
        parts = [padded_strips[self.rank_of(i)][: self.bounds[i + 1] - self.bounds[i]] for i in range(self.n)]
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

    def __init__(self, plan: StripPlan, rank: int, device, nbuf: int = 2, host_staging: bool = False,
                 timing: bool = False):
        """host_staging: gather through host copies (gloo rehearsal of the GPU path).  timing (GPU
        ranks): events around every gather (gather_ms)."""
        import torch

        self.plan, self.rank, self.root, self.nbuf = plan, rank, 0, nbuf
        self.host_staging = host_staging
        self.device = device
        W = plan.W
        r0, r1 = plan.rows(rank)
        fdev = "cpu" if host_staging else device
        self.frames = []
        if rank == self.root:
            self.frames = [torch.zeros((plan.H, W, 4), dtype=torch.float32, device=fdev) for _ in range(nbuf)]
        if rank == self.root and not host_staging:
            self.strips = [f[r0:r1] for f in self.frames]  # contiguous rows of the frame
        else:
            self.strips = [torch.zeros((r1 - r0, W, 4), dtype=torch.float32, device=device) for _ in range(nbuf)]
        self.pending = [None] * nbuf
        # timing: per gather, an event on the output stream before the sends / receives (the
        # strip is rendered) and one on a side stream made to wait for the transfers' completion
        self.timing = timing and not host_staging
        self.side = torch.cuda.Stream(device) if self.timing else None
        self.marks: list = []

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
        e0 = None
        if self.timing:
            import torch

            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        self.pending[i] = dist.batch_isend_irecv(ops) if ops else None
        if self.timing and self.pending[i]:
            import torch

            # Work.wait() orders the current stream after the transfers (no host block): the
            # side stream's event marks when this rank's sends / receives have completed
            e1 = torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(self.side):
                for w in self.pending[i]:
                    w.wait()
                e1.record()
            self.marks.append((e0, e1))

    def gather_ms(self, reset: bool = True) -> list[float]:
        """ms from 'strip rendered on this rank' to 'this rank's transfers complete', per gather
        since the last reset (synchronises).  Rank 0: until every strip has landed in its frame."""
        import torch

        torch.cuda.synchronize()
        out = [a.elapsed_time(b) for a, b in self.marks]
        if reset:
            self.marks = []
        return out

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


def probe_links(rank: int, world: int, device, nbytes: int, host_staging: bool = False, reps: int = 4) -> dict:
    """One-way transfer rates into rank 0 over the gather's own path (batch_isend_irecv: RCCL
    send/recv over xGMI on GPUs, gloo through host with host_staging): every rank alone (the
    slowest is the per-link rate) and all ranks at once (the root's ingest rate).  Timed on rank 0
    by wall clock over `reps` transfers after one warm-up, each case behind a barrier; every rank
    returns rank 0's figures."""
    import time

    import torch
    import torch.distributed as dist

    n_el = max(1, nbytes // 4)
    dev = "cpu" if host_staging else device
    bufs = [torch.empty(n_el, dtype=torch.float32, device=dev) for _ in range(world)] if rank == 0 else None
    src = torch.ones(n_el, dtype=torch.float32, device=dev) if rank != 0 else None

    def sync():
        if not host_staging:
            torch.cuda.synchronize()

    def xfer(senders):
        if rank == 0:
            ops = [dist.P2POp(dist.irecv, bufs[r], r) for r in senders]
        else:
            ops = [dist.P2POp(dist.isend, src, 0)] if rank in senders else []
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()

    def timed(senders):
        xfer(senders)
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            xfer(senders)
        sync()
        return (time.perf_counter() - t0) / reps

    per = [timed([r]) for r in range(1, world)]
    both = timed(list(range(1, world)))
    out = torch.zeros(world + 1, dtype=torch.float64, device="cpu" if host_staging else device)
    if rank == 0:
        out[1:world] = torch.tensor(per, dtype=torch.float64)
        out[world] = both
    dist.all_reduce(out)
    per_ms = [float(x) * 1e3 for x in out[1:world].tolist()]
    all_ms = float(out[world].item()) * 1e3
    rates = [nbytes / (ms * 1e6) for ms in per_ms]
    return {"link_gbps": min(rates), "ingest_gbps": (world - 1) * nbytes / (all_ms * 1e6),
            "per_link_gbps": [round(r, 2) for r in rates], "bytes": nbytes, "reps": reps,
            "per_link_ms": [round(m, 4) for m in per_ms], "all_at_once_ms": round(all_ms, 4),
            "path": "gloo through host (rehearsal)" if host_staging else "RCCL send/recv (batch_isend_irecv)"}
