#!/usr/bin/env python
"""Benchmark: Mrays/s + ms/frame of the per-pixel ray-scene hot path (BASELINE.json metric).

Workload (default, BASELINE.json configs[3] = SURVEY §8d config (d)): 3840x2160, 64 spheres,
AO 16 spp + temporal/spatial post-process (mode 1 = aop_compute + aop_postprocessing),
synthetic seeded scene (scene seed 1234+3, per-frame rand_buffer seed 7000+k).

One step = one frame: host header update (fill_rand_buffer, mode.y) -> upload -> AO pass ->
post-process pass (-> on N>1, gather of the image strips into rank 0 over RCCL, pipelined).
N GPUs split the SAME frame into cost-balanced row strips (strong scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config b|c|d|e]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

--gpus N means N ranks.  Without a launcher (WORLD_SIZE unset) and N > 1, bench.py starts
torch.distributed.run with N processes on 127.0.0.1 itself, before anything touches the GPU, and
exits with its status; under a launcher, WORLD_SIZE must equal N or the run exits non-zero.

Rank 0 prints one JSON line.  Mrays/s = W*H*spp*K / time (primary samples, whole job).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

# Pipelined frames keep three streams busy (two AO streams + the output stream) beside
# RCCL's: with HIP's default of 4 hardware queues per process two of them can land on one
# queue and serialise.  8 queues (must be set before the HIP runtime starts; <= 32).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

CONFIGS = {
    # name: (W, H, spheres, spp, mode, description)
    "a": (640, 480, 4, 1, 3, "config (a): 640x480, 4 spheres, Phong (mode 3), 1 spp"),
    "b": (1920, 1080, 16, 1, 4, "config (b): 1920x1080, 16 spheres, Phong + reflections (mode 4, <=20 bounces), 1 spp"),
    "c": (1920, 1080, 64, 16, 2, "config (c): 1920x1080, 64 spheres, AO 16 spp (mode 2)"),
    "d": (3840, 2160, 64, 16, 1, "config (d): 3840x2160, 64 spheres, AO 16 spp + temporal/spatial post-process (mode 1)"),
    "e": (7680, 4320, 256, 64, 2, "config (e): 7680x4320, 256 spheres, AO 64 spp (mode 2)"),
    # scenes with planes (not BASELINE configs: the plane path's own measurement)
    "p": (3840, 2160, 65, 16, 1, "config (d) + one ground plane (64 spheres + 1 plane = 65 objects), AO 16 spp + "
                                 "post-process (mode 1)"),
    # diagnostic twin of "p": the plane replaced by a sphere of radius 1e4 tangent to it (same
    # workload shape, all spheres): isolates what the plane path itself costs
    "q": (3840, 2160, 65, 16, 1, "config p with its plane replaced by a radius-1e4 sphere tangent to it (65 spheres), "
                                 "AO 16 spp + post-process (mode 1)"),
    "s1": (3840, 2160, 10, 16, 1, "the reference's scene1 (4 spheres + 1 plane, src/scene.h:15-65) at 3840x2160, "
                                  "AO 16 spp + post-process (mode 1)"),
    # the reference's own instance (src/main.cpp:29-36, 146, 309): 440x330, NUM_SHAPES 10, AA 4,
    # scene1 (4 spheres + 1 plane), lighting 1 = aop_compute + aop_postprocessing
    "ref": (440, 330, 10, 4, 1, "the reference's own instance: 440x330, NUM_SHAPES 10, AA 4, scene1 (4 spheres + 1 plane), "
                                "lighting 1 = AO + post-process (src/main.cpp:29-36, 146, 309)"),
}
CONFIG_INDEX = {"a": 0, "b": 1, "c": 2, "d": 3, "e": 4, "p": 3, "q": 3, "s1": 3, "ref": 3}


def config_header(name: str):
    """The seeded scene of a config: synthetic spheres (seed 1234 + config index);
    "p" adds a ground plane y = -2.5 to config (d)'s scene; "s1" is the reference's scene1."""
    from real_time_ray_tracer_amd import Header, aspect_for

    W, H, S, spp, _, _ = CONFIGS[name]
    if name in ("s1", "ref"):
        return Header.builtin(1, spp, aspect_for(W, H), num_shapes=S)
    if name in ("p", "q"):
        h = Header.synthetic(S - 1, spp, 1234 + CONFIG_INDEX[name], aspect_for(W, H), num_shapes=S)
        if name == "p":
            h.pack_plane(S - 1, (0.0, 1.0, 0.0), -2.5, (0.45, 0.4, 0.35), reflectivity=1.0)
        else:
            h.pack_sphere(S - 1, (0.0, -10002.5, 0.0), 10000.0, (0.45, 0.4, 0.35), reflectivity=1.0)
        h.set_mode(0, S)
        return h
    return Header.synthetic(S, spp, 1234 + CONFIG_INDEX[name], aspect_for(W, H))

FLOP_PER_TEST = 20          # ~20 FLOP per ray-sphere test (FMA = 2 FLOP)
PEAK_FP32_TFLOPS = 157.3    # MI355X_MICROARCH.md: peak FP32 vector (spec)
PEAK_HBM_GBPS = 8000.0      # MI355X_MICROARCH.md: HBM3E peak (spec)
# algorithmic HBM bytes per pixel per launch: mode-1 pass 1 writes raw colour +
# normal + depth (48 B); mode 2 also the image (64 B); modes 3/4 pixel + image (32 B).  The
# post-process (pass 2, aop_postprocessing.glsl:57-208) needs, at minimum: per pixel its raw
# colour (16 B) and its normal's hit flag w (4 B), and writes pixel + image (32 B); per filtered
# pixel (a primary hit) also its normal xyz (12 B) and depth.xy (8 B: .z/.w are never read);
# per history slot it examines the slot's normal xyz + depth.xy (20 B), and per slot it accepts
# the slot's colour (16 B).  The 4 neighbours are other pixels' bytes.  Counted per launch from
# the kernel's counters ([5] filtered pixels, [6] slots read, [7] slots accepted).
BYTES_PER_PIXEL = {1: 48, 3: 64, 4: 32, 5: 32}
POST_BYTES_PIXEL, POST_BYTES_FILTERED, POST_BYTES_SLOT_READ, POST_BYTES_SLOT_ACCEPTED = 52, 20, 20, 16


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpus() -> dict:
    """The CPUs this process may use: the affinity mask, the cgroup CPU quota (the GPU box's
    lease is 16 CPUs of a 256-CPU host: affinity shows all 256, the quota 16), and the thread
    count the CPU baseline uses = min(affinity, quota)."""
    import math
    import shutil
    import subprocess

    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    nproc = None
    if shutil.which("nproc"):
        try:  # GNU nproc honours OMP_NUM_THREADS; --all is the host's count
            nproc = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
        except ValueError:
            pass
    usable = aff if quota is None else max(1, min(aff, math.floor(quota + 1e-9)))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "nproc": nproc, "os_cpu_count": os.cpu_count(),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "usable": usable, "cpu": model}


def cpu_baseline(cfg_name: str, target_s: float) -> dict:
    """The CPU oracle (oracle/rt_oracle.c, OpenMP over pixels, one thread per usable CPU) on a
    bounded, evenly spread sample of 4-row bands of the same frame.  Mode 1 is timed in steady
    state: each band renders RING frames in a row (its 8-slot history ring fills), the AO pass
    is timed in every frame and the post-process only once 7 history slots hold frames (the
    temporal filter of aop_postprocessing.glsl:177-201 then examines up to 7 slots, as in the
    GPU's timed frames); a frame costs the mean AO pass + the mean steady-state post-process."""
    import oracle

    oracle.select_native()
    W, H, S, spp, mode, _ = CONFIGS[cfg_name]
    cpus = host_cpus()
    threads = cpus["usable"]
    h = config_header(cfg_name)
    progs = {1: [oracle.AOP_COMPUTE, oracle.AOP_POSTPROCESSING], 2: [oracle.AO_COMPUTE],
             3: [oracle.P_COMPUTE], 4: [oracle.H_COMPUTE]}[mode]
    # rows per band: 4 in mode 1 (vertical neighbours for the post-process); modes 2-4 have no
    # neighbour reads, and 32-row bands keep OpenMP's per-call cost out of a small frame's time
    BAND = 4 if mode == 1 else 32
    FR = 9 if mode == 1 else 2    # frames per band: mode 1 -> frames 7 and 8 have 7 history slots
    STEADY = 7                    # first steady-state frame of the post-process

    def run_band(y):
        """One band's FR frames: (trace s, trace passes, steady post s, steady post passes)."""
        t_trace = t_post = 0.0
        n_trace = n_post = 0
        gh = min(BAND, H - int(y))
        d = oracle.dims(W, H, S, spp, gy0=int(y), gh=gh)
        buf = np.zeros(h.data.size + 3 * 8 * W * gh * 4, np.float32)
        hh = h.copy()
        for k in range(FR):
            if mode in (1, 2):
                hh.fill_rand_buffer(7000 + k)
            else:
                hh.moving_light(False)
            slot = k % 8
            hh.set_mode(slot, hh.num_objects)
            buf[:hh.data.size] = hh.data
            t0 = time.perf_counter()
            oracle.run_program(buf, d, progs[0], slot, None, nthreads=threads)
            t_trace += time.perf_counter() - t0
            n_trace += 1
            if mode == 1:
                t0 = time.perf_counter()
                oracle.run_program(buf, d, progs[1], slot, None, nthreads=threads)
                if k >= STEADY:
                    t_post += time.perf_counter() - t0
                    n_post += 1
        return t_trace, n_trace, t_post, n_post

    # bands in van der Corput order over the frame's H / BAND bands (every prefix is spread
    # evenly over the rows, sky and ground alike) until target_s of CPU work has run
    nb = H // BAND
    order, seen = [], set()
    bits = max(1, (nb - 1).bit_length())
    for i in range(1 << bits):
        j = int(format(i, f"0{bits}b")[::-1], 2)
        if j < nb and j not in seen:
            seen.add(j)
            order.append(j)
    t_trace = t_post = 0.0
    n_trace = n_post = n = 0
    tw = time.perf_counter()
    # (a small frame is swept again until target_s: config (b)'s whole frame is ~16 ms of CPU work)
    while True:
        j = order[n % len(order)]
        a, b_, c_, d_ = run_band(j * BAND)
        t_trace, n_trace, t_post, n_post, n = t_trace + a, n_trace + b_, t_post + c_, n_post + d_, n + 1
        if time.perf_counter() - tw >= target_s and n >= 2:
            break
    wall = time.perf_counter() - tw
    per_band_frame = t_trace / n_trace + (t_post / n_post if n_post else 0.0)  # seconds per band per frame
    rays = BAND * W * (spp if mode in (1, 2) else 1)                          # per band per frame
    names = {1: "aop_compute", 2: "aop_postprocessing", 3: "ao_compute", 4: "p_compute", 5: "h_compute"}
    return {"value": round(rays / per_band_frame / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "cpu": cpus["cpu"], "host_cpus": cpus,
            "cores_note": ("threads = min(affinity CPUs, cgroup CPU quota): the lease's CPU share; more threads "
                           "than the quota only time-slice"),
            "build": oracle.lib_name(),
            "sample": f"{n} bands of {BAND} rows (evenly spread; {n * BAND / H:.2f} passes over the {H} rows) x {W} px x "
                      f"{spp if mode in (1, 2) else 1} spp, {FR} frames per band"
                      + (f" (post-process timed in frames {STEADY}-{FR - 1}, full history ring)" if mode == 1 else "")
                      + f", {'+'.join(names[p] for p in progs)}, oracle/rt_oracle.c with {threads} OpenMP threads, "
                      f"{wall:.1f} s; ms/frame extrapolated {per_band_frame * H / BAND * 1e3:.0f}"}


def ssbo_path(cfg_name: str, gpu: int, frames: int = 30) -> dict:
    """The reference's own call shape, timed: every frame copies the whole host SSBO in, runs the
    program(s) and copies the whole SSBO (and the image) back (compute_one_shader /
    compute_two_shaders, src/main.cpp:580-671), through rt_compute_one/two_shaders.  PCIe-inclusive;
    never the headline value (that one keeps the inputs resident in HBM)."""
    from real_time_ray_tracer_amd import (AO_COMPUTE, AOP_COMPUTE, AOP_POSTPROCESSING, H_COMPUTE, P_COMPUTE, SSBO,
                                          Renderer)

    W, H, S, spp, mode, _ = CONFIGS[cfg_name]
    h = config_header(cfg_name)
    s = SSBO(h, W, H)
    img = np.zeros((H, W, 4), np.float32)
    r = Renderer(W, H, S, spp, device=gpu)
    f = 0

    def one(k, f):
        if mode in (1, 2):
            h.fill_rand_buffer(7000 + k)
        else:
            h.moving_light(False)
        s.set_header(h)
        if mode == 1:
            return r.compute_two_shaders(s, f, AOP_COMPUTE, AOP_POSTPROCESSING, img)
        return r.compute_one_shader(s, f, {2: AO_COMPUTE, 3: P_COMPUTE, 4: H_COMPUTE}[mode], img)

    for k in range(4):
        f = one(k, f)
    t0 = time.perf_counter()
    for k in range(4, 4 + frames):
        f = one(k, f)
    dt = (time.perf_counter() - t0) / frames
    r.close()
    nbytes = s.data.nbytes
    return {"ms_per_frame": round(dt * 1e3, 4), "mrays_per_s": round(W * H * (spp if mode in (1, 2) else 1) / dt / 1e6, 2),
            "frames": frames, "ssbo_bytes": nbytes, "pcie_bytes_per_frame": 2 * nbytes + img.nbytes,
            "call": "rt_compute_two_shaders (whole SSBO in and out, src/main.cpp:622-671)" if mode == 1
            else "rt_compute_one_shader (whole SSBO in and out, src/main.cpp:580-620)"}


VALU_FMA_RATE = 116.7e12 / 128  # wave64 v_fma_f32 instructions/s a dense stream sustains (profiles/r01g_valu_rate.txt)


def load_sq(cfg_name: str, src_sha1):
    """SQ counters per dispatch (profiles/*_sq_<cfg>.json, tools/pmc_config.sh), preferring this build's."""
    found = []
    for p in sorted(ROOT.glob(f"profiles/*_sq_{cfg_name}.json"), reverse=True):
        try:
            found.append((json.loads(p.read_text()), p.name))
        except Exception:
            continue
    for data, name in found:
        if src_sha1 and data.get("src_sha1") == src_sha1:
            return data, name
    return found[0] if found else (None, None)


def build_info() -> dict:
    """The library's source hash and commit (written by `make lib` next to librtrt.so)."""
    try:
        return json.loads((ROOT / "real_time_ray_tracer_amd" / "BUILD_INFO").read_text())
    except Exception:
        return {"src_sha1": None, "commit": None}


def load_traffic(cfg_name: str, src_sha1, root: Path | None = None):
    """HBM bytes per launch measured with rocprofv3 PMC passes (tools/pmc_summary.py): files named
    profiles/*_pmc_<cfg>.json (as load_sq's *_sq_<cfg>.json) or the older profiles/*_pmc.json whose
    "config" is this config; the newest by name, preferring one taken on this library build (same
    source hash)."""
    found = []
    prof = (root or ROOT) / "profiles"
    paths = set(prof.glob(f"*_pmc_{cfg_name}.json")) | set(prof.glob("*_pmc.json"))
    for p in sorted(paths, key=lambda q: q.name, reverse=True):
        try:
            data = json.loads(p.read_text())
        except Exception:
            continue
        if data.get("config", cfg_name) == cfg_name:
            found.append((data, p.name))
    for data, name in found:
        if src_sha1 and data.get("src_sha1") == src_sha1:
            return data, name
    return found[0] if found else (None, None)


def rank_devices(world, rank, gpu, cdev):
    """every rank's (device index, PCI bus) on every rank: a world x 2 all-reduce"""
    import torch
    import torch.distributed as dist

    props = torch.cuda.get_device_properties(gpu)
    t = torch.zeros(world, 2, dtype=torch.float64, device=cdev)
    t[rank, 0] = gpu
    t[rank, 1] = getattr(props, "pci_bus_id", -1)
    if world > 1:
        dist.all_reduce(t)
    return [{"device": int(t[i, 0].item()), "pci_bus": int(t[i, 1].item())} for i in range(world)]


def launch_report(args, world, rank, local_rank):
    """--launch-check: the ranks are up and agree; rank 0 reports who runs where"""
    import torch
    import torch.distributed as dist

    # (NCCL has no CPU tensors: the report's tensor lives on the rank's GPU under nccl)
    tdev = torch.device("cuda", local_rank) if args.backend == "nccl" and world > 1 else "cpu"
    t = torch.zeros(world, 3, dtype=torch.float64, device=tdev)
    t[rank] = torch.tensor([local_rank, os.getpid(), 1.0], dtype=torch.float64, device=tdev)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "gpus_arg": args.gpus, "backend": args.backend,
                          "launched_by": os.environ.get("RTRT_BENCH_LAUNCHER", "external launcher"),
                          "ranks": [{"rank": i, "local_rank": int(t[i, 0].item()), "pid": int(t[i, 1].item())}
                                    for i in range(world)],
                          "ranks_up": int(t[:, 2].sum().item())}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def launch_ranks(argv) -> int | None:
    """--gpus N > 1 without a launcher: run this script as N ranks under torch.distributed.run
    (one process per GPU, 127.0.0.1 rendezvous on a free port) and return its exit status (None:
    nothing launched, this process is the rank).  Called
    before anything initialises HIP in this process (nothing here touches the GPU), so the ranks
    are children of a clean parent; the parent never execs."""
    import socket
    import subprocess

    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args(argv)[0].gpus
    if n <= 1 or "WORLD_SIZE" in os.environ:
        return None
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RTRT_BENCH_LAUNCHER=f"bench.py --gpus {n}: torch.distributed.run, {n} ranks")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + list(argv)
    print(f"bench.py: starting {n} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed frames (default 20; configs (a) and (b), whose frames are 7-26 us, 1000 and 400 "
                         "so the timed region is >= 7 ms)")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="d", choices=sorted(CONFIGS))
    ap.add_argument("--no-balance", action="store_true", help="equal strips instead of cost-balanced")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="mode 1: run each frame's post-process after its AO pass on one stream, instead of "
                         "overlapping frame k's post-process with frame k+1's AO pass")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--warm-ms", type=float, default=300.0,
                    help="after the warm-up frames, keep rendering (chunks of 8 frames) until this much wall "
                         "time has passed on every rank, so the timed frames run at settled GPU clocks: the "
                         "clock ramps over ~10 ms of load (DVFS), longer than 20 strip frames at N = 8")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 also renders every frame whole and checks the gathered frames bit for bit "
                         "(without it, N > 1 still checks the first 2 gathered frames, before the timed region)")
    ap.add_argument("--frame-batch", type=int, default=1,
                    help="modes 2-4: most frames per launch in the C++ frame loop (rt_set_frame_batch).  1 (the "
                         "default) = the reference's dispatch shape, one launch and one image write per frame "
                         "(src/main.cpp:604): `value`.  >1: multi-frame launches (only the launch's last frame "
                         "writes the image) are timed instead; either way the other shape is reported beside it")
    ap.add_argument("--link-gbps", type=float, default=0.0,
                    help="N>1: the gather planner's per-link rate (GB/s one way into rank 0); 0 (default) = "
                         "measured over the gather's own path before planning (dist.probe_links)")
    ap.add_argument("--ingest-gbps", type=float, default=0.0,
                    help="N>1 with --link-gbps: the root's ingest rate over all links (default min(N-1, 7) x link)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearsal of the N>1 path with ranks sharing GPUs, gather staged through host")
    ap.add_argument("--out-stream-priority", type=int, default=0,
                    help="mode 1 pipelined: torch priority of the post-process (output) stream (lower = higher)")
    ap.add_argument("--no-tile-schedule", action="store_true",
                    help="workgroups in the plain order (rt_set_tile_schedule(0)) instead of longest first")
    ap.add_argument("--no-alt-dispatch", action="store_true",
                    help="modes 2-4: skip timing the other dispatch shape (counter runs: every dispatch then has "
                         "the timed shape, so per-dispatch counters are per frame)")
    ap.add_argument("--dist-timeout", type=float, default=600.0,
                    help="N>1: seconds a collective may wait for a peer before it raises (a rank that died "
                         "takes the others down within this time instead of hanging the job)")
    ap.add_argument("--inject-failure", type=int, default=-1, metavar="RANK",
                    help="test hook: this rank raises right after the process group is up")
    ap.add_argument("--launch-check", action="store_true",
                    help="stop after the start-up check: rank 0 prints one JSON line with the world size and each "
                         "rank's device (the N-rank launch without a frame; runs on the CPU with --backend gloo)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = {"a": 1000, "b": 400}.get(args.config, 20)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:  # (launch_ranks starts the ranks when no launcher did)
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: a run asked for N GPUs must run N ranks")
    import torch
    import torch.distributed as dist

    from real_time_ray_tracer_amd import Header, Renderer, aspect_for
    from real_time_ray_tracer_amd.dist import (StripGather, StripPlan, balanced_bounds, calibrate_row_cost, equal_bounds,
                                               gather_bound, gather_bounds, imbalance, probe_links)

    from real_time_ray_tracer_amd.dist import init_process_group

    # the process group first for gloo (no GPU call before its start-up check), after the
    # device for RCCL (device_id binds the communicator); every collective times out after
    # --dist-timeout, and run_rank (bottom) turns any exception into a named, non-zero exit
    if world > 1 and args.backend == "gloo":
        init_process_group("gloo", timeout_s=args.dist_timeout)
    if world > 1 and args.backend == "nccl":
        torch.cuda.set_device(local_rank)
        init_process_group("nccl", torch.device("cuda", local_rank), timeout_s=args.dist_timeout)
    if world > 1:
        if rank == args.inject_failure:
            raise RuntimeError(f"injected failure on rank {rank} (--inject-failure)")
        # start-up check: every rank is alive and agrees on the run before any GPU work
        chk = torch.tensor([1.0, float(args.steps)], dtype=torch.float64,
                           device=torch.device("cuda", local_rank) if args.backend == "nccl" else "cpu")
        dist.all_reduce(chk)
        if int(chk[0].item()) != world or int(chk[1].item()) != world * args.steps:
            raise RuntimeError(f"ranks disagree at start-up: {chk.tolist()} (world {world}, steps {args.steps})")
    if args.launch_check:
        return launch_report(args, world, rank, local_rank)
    gpu = local_rank if args.backend == "nccl" else local_rank % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # collective tensors
    devices = rank_devices(world, rank, gpu, cdev)

    W, H, S, spp, mode, desc = CONFIGS[args.config]
    header = config_header(args.config)
    nobj = header.num_objects
    # a dedicated stream: the renderer, the gather and torch's copies are all ordered on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    # ---- strip plan: cost-balanced from the kernels' per-row work counters, calibrated against
    # each strip's measured render time, and planned WITH the gather: the root strip (rank 0's,
    # rendered in place) and the bounds minimise max(render, per-link copy, root ingest) on the
    # link rates measured here (rt_plan_strips_gather); best of three measured plans ------------
    bounds = equal_bounds(H, world)
    root_strip = 0
    balance_info = None
    links = None
    if world > 1 and not args.no_balance:
        piped = mode == 1 and not args.no_pipeline

        def strip_run(sp, frames, counters):
            """counters: one frame's row-counter profile.  Otherwise the strip's time per frame as
            the timed run will render it: pipelined mode 1 by wall clock over 16 frames after 8,
            else the kernels' HIP-event times of the last 3 of `frames` frames."""
            r = Renderer(W, H, S, spp, device=gpu, rows=sp.rows(rank))
            r.set_stream(stream)
            if counters:
                r.enable_counters(totals=False, rows=True)
            timed_wall = piped and not counters
            if timed_wall:
                r.enable_pipelining(True)
                frames = 24
            f = 0
            t0 = 0.0
            if not counters:  # settled clocks for the measurement (see --warm-ms)
                tw, k = time.perf_counter(), 0
                while (time.perf_counter() - tw) * 1e3 < min(args.warm_ms, 100.0):
                    header.fill_rand_buffer(7000 + k) if mode in (1, 2) else header.moving_light(False)
                    header.set_mode(f, nobj)
                    r.upload_header(header)
                    f = r.dispatch(mode, f)
                    k += 1
                    if k % 8 == 0:
                        r.synchronize()
            for k in range(frames):
                header.fill_rand_buffer(7000 + k) if mode in (1, 2) else header.moving_light(False)
                header.set_mode(f, nobj)
                r.upload_header(header)
                if timed_wall and k == 8:
                    r.synchronize()
                    t0 = time.perf_counter()
                if k == frames - 3 and not counters and not timed_wall:  # time the last 3 frames
                    r.enable_timing(True)
                    r.reset_stats()
                f = r.dispatch(mode, f)
            out = r.read_row_counters().astype(np.float64) if counters else None
            ms = 0.0
            if timed_wall:
                r.synchronize()
                ms = (time.perf_counter() - t0) / (frames - 8) * 1e3
            elif not counters:
                for p in {1: [1, 2], 2: [3], 3: [4], 4: [5]}[mode]:
                    n_l, tot = r.kernel_stats(p)
                    ms += tot / max(n_l, 1)
            r.close()
            return out, ms

        sp0 = StripPlan(W, H, bounds)
        mine, _ = strip_run(sp0, 1, True)
        full = torch.zeros(H, dtype=torch.float64, device=cdev)
        full[bounds[rank]:bounds[rank + 1]] = torch.from_numpy(mine).to(cdev)
        dist.all_reduce(full)
        row_cost = full.cpu().numpy()
        bounds = balanced_bounds(row_cost, world)
        # the link model: measured over the gather's own path (a strip's worth of bytes per
        # transfer), unless --link-gbps states it
        if args.link_gbps > 0:
            links = {"link_gbps": args.link_gbps, "ingest_gbps": args.ingest_gbps if args.ingest_gbps > 0
                     else min(world - 1, 7) * args.link_gbps, "source": "stated (--link-gbps / --ingest-gbps)"}
        else:
            links = probe_links(rank, world, dev, (H // world) * W * 16 if args.backend == "nccl" else 4 << 20,
                                host_staging=args.backend == "gloo")
            links["source"] = "measured before the plan (dist.probe_links)"
        # calibration: time each strip's render, rescale the profile so every strip's total is its
        # measured time (ms per row), re-plan with the gather; keep the measured plan whose bound
        # max(measured render, link model) is smallest (3 measurements)
        measured = []
        for it in range(3):
            sp = StripPlan(W, H, bounds, root_strip)
            _, ms = strip_run(sp, 6 if mode in (1, 2) else 3, False)
            tt = torch.zeros(world, dtype=torch.float64, device=cdev)
            tt[sp.strip_of(rank)] = ms
            dist.all_reduce(tt)
            t1 = tt.cpu().tolist()  # per strip, in row order
            per_row = np.concatenate([np.full(bounds[i + 1] - bounds[i], t1[i] / (bounds[i + 1] - bounds[i]))
                                      for i in range(world)])
            pred = gather_bound(per_row, bounds, root_strip, W, links["link_gbps"], links["ingest_gbps"])
            measured.append((pred["bound_ms"], list(bounds), root_strip, t1, pred))
            if it < 2:
                row_cost = calibrate_row_cost(bounds, row_cost, t1)
                bounds, root_strip, _ = gather_bounds(row_cost, world, W, links["link_gbps"], links["ingest_gbps"])
        best = min(measured, key=lambda m: m[0])
        bounds, root_strip = best[1], best[2]
        balance_info = {"model_bounds": measured[0][1], "model_strip_ms": [round(t, 4) for t in measured[0][3]],
                        "model_imbalance": round(imbalance(measured[0][3]), 4),
                        "calibrated_max_ms": [round(max(m[3]), 4) for m in measured],
                        "plans": [{"bounds": m[1], "root_strip": m[2], "strip_ms": [round(t, 4) for t in m[3]],
                                   "predicted_ms": {k: round(v, 4) for k, v in m[4].items()}} for m in measured],
                        "root_strip": root_strip,
                        "predicted_frame_ms": {k: round(v, 4) for k, v in best[4].items()},
                        "predicted_basis": ("max(render: each strip's measured render time, link: the largest "
                                            "non-root strip's bytes / link_gbps, ingest: all non-root bytes / "
                                            "ingest_gbps); rt_strip_gather_bound"),
                        "link_model": links}
    plan = StripPlan(W, H, bounds, root_strip)
    r0, r1 = plan.rows(rank)
    rend = Renderer(W, H, S, spp, device=gpu, rows=(r0, r1))
    if args.frame_batch > 0:
        rend.set_frame_batch(args.frame_batch)
    if args.no_tile_schedule:
        rend.set_tile_schedule(False)
    rend.set_stream(stream)
    # pipelined mode 1: post-process (and the image consumers: the gather) on a second stream
    pipeline = mode == 1 and not args.no_pipeline
    out_stream = torch.cuda.Stream(dev, priority=args.out_stream_priority) if pipeline else stream
    if pipeline:
        rend.enable_pipelining(True, out_stream)
    streams = {"out": out_stream}
    gather = (StripGather(plan, rank, dev, host_staging=args.backend == "gloo", timing=args.backend == "nccl")
              if world > 1 else None)
    state = {"frame": 0, "ref_frame": 0, "mismatch": 0, "checked": 0, "verify_on": True, "phase": "warm-up"}
    ref = None
    # rank 0 checks gathered frames against a whole-frame render of its own: every frame with
    # --verify, otherwise (N > 1) the first VERIFY_FIRST frames, during the warm-up, so every
    # multi-GPU line carries correctness evidence without touching the timed region
    VERIFY_FIRST = 2
    if (args.verify or world > 1) and rank == 0:
        ref = Renderer(W, H, S, spp, device=gpu)
        ref.set_stream(stream)

    def verify(k: int):
        # rank 0: the gathered frame of frame k must equal the whole-frame render, bit for bit
        import torch as _t
        ref.upload_header(header)
        state["ref_frame"] = ref.dispatch(mode, state["ref_frame"])
        if gather is None:
            got = rend.image()
        else:
            gather.finish()
            got = gather.frame(k).cpu().numpy()[:H]
        want = ref.image()
        state["checked"] += 1
        bad = np.any(got.view(np.uint32) != want.view(np.uint32), axis=2)
        if bad.any():
            state["mismatch"] += 1
            ys = np.nonzero(bad.any(axis=1))[0]
            state.setdefault("diag", []).append({"frame": k, "phase": state["phase"], "pixels": int(bad.sum()),
                                                 "rows": [int(ys.min()), int(ys.max())], "nrows": int(len(ys))})
        _t.cuda.synchronize()

    def step(k: int):
        if mode in (1, 2):
            header.fill_rand_buffer(7000 + k)
        else:
            header.moving_light(False)
        header.set_mode(state["frame"], nobj)
        rend.upload_header(header)
        if gather is not None:
            with torch.cuda.stream(streams["out"]):  # the post-process writes the strip buffer there
                buf = gather.strip(k)
            rend.bind_image(buf.data_ptr())
        state["frame"] = rend.dispatch(mode, state["frame"])
        if gather is not None:
            with torch.cuda.stream(streams["out"]):
                gather.gather(k)
        if ref is not None and state["verify_on"] and (args.verify or k < VERIFY_FIRST):
            verify(k)

    # One GPU, sequential modes: the frame loop runs in C++ (rt_compute_frames, the render loop of
    # src/main.cpp:763-781): same frames as step(), without the per-frame Python and ctypes cost
    # that makes the small configs host-bound.  Pipelined mode 1 and N > 1 keep step().
    host_loop = world == 1 and ref is None and not pipeline
    # the 8-slot history ring is full before timing whatever --warmup says (>= 8
    # warm-up frames so the mode-1 temporal filter reads a full ring)
    ring_fill = max(0, rend.F - args.warmup)
    warm = args.warmup + ring_fill
    tw = time.perf_counter()
    if host_loop:
        state["frame"] = rend.compute_frames(header, mode, state["frame"], warm, 7000, False)
    else:
        for k in range(warm):
            step(k)
    # settle the clock: chunks of 8 more frames until warm_ms has passed on every rank (the
    # ranks agree on the chunk count, so the per-frame gathers stay matched)
    settle = 0
    while True:
        torch.cuda.synchronize()
        left = torch.tensor([args.warm_ms - (time.perf_counter() - tw) * 1e3], dtype=torch.float64, device=cdev)
        if world > 1:
            dist.all_reduce(left, op=dist.ReduceOp.MAX)
        if float(left.item()) <= 0.0:
            break
        if host_loop:
            state["frame"] = rend.compute_frames(header, mode, state["frame"], 8, 7000 + warm + settle, False)
        else:
            for k in range(warm + settle, warm + settle + 8):
                step(k)
        settle += 8
    warm += settle
    if gather is not None:
        gather.finish()
        gather.gather_ms(reset=True)  # the timed frames' gathers only
    torch.cuda.synchronize()

    # ---- timed region -----------------------------------------------------------------------
    state["phase"] = "timed"
    # per-launch HIP events only where the timed launches are the kernel durations (sequential);
    # pipelined, the roofline uses the standalone launches below and the events are host cost
    rend.enable_timing(not pipeline and not host_loop)
    rend.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0  # host time inside step() (enqueue + back-pressure waits)
    frame_ev = []  # per-frame completion events (the frame's last stream): median frame interval
    if host_loop:
        # chunks of the C++ loop, each bracketed by an event: the median chunk's ms per frame;
        # chunks of F frames (a multi-frame launch of modes 2-4 never spans two chunks)
        F = rend.F
        sizes = [min(F, args.steps - i) for i in range(0, args.steps, F)]
        k0 = warm
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        frame_ev.append((ev, 0))
        for n_ in sizes:
            th = time.perf_counter()
            state["frame"] = rend.compute_frames(header, mode, state["frame"], n_, 7000 + k0, False)
            host_s += time.perf_counter() - th
            k0 += n_
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            frame_ev.append((ev, n_))
    else:
        for k in range(warm, warm + args.steps):
            th = time.perf_counter()
            step(k)
            host_s += time.perf_counter() - th
            if world == 1:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(streams["out"])
                frame_ev.append((ev, 1))
    if gather is not None:
        gather.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gms = gather.gather_ms(reset=True) if gather is not None and gather.timing else []
    host_wait_ms, host_waits = rend.host_stats()
    intervals = [frame_ev[i][0].elapsed_time(frame_ev[i + 1][0]) / frame_ev[i + 1][1]
                 for i in range(len(frame_ev) - 1)] if frame_ev else []
    rend.enable_timing(False)
    progs = {1: [1, 2], 2: [3], 3: [4], 4: [5]}[mode]
    kstats = {p: rend.kernel_stats(p) for p in progs}

    # ---- the other dispatch shape of modes 2-4, the same frames through the same C++ loop, wall
    # clock: batched (up to F frames per launch, the image by each launch's last frame) beside
    # the reference's one launch + one image write per frame, or the other way round --------
    fb_timed = args.frame_batch
    fb_other = 32 if fb_timed == 1 else 1
    frames_per_launch = lambda fb: min(32, fb, rend.F)  # rt_compute_frames: min(kMaxBatch, batch, F)
    other = None
    if host_loop and mode in (2, 3, 4) and not args.no_alt_dispatch:
        rend.set_frame_batch(fb_other)
        # warm the other path first (its kernel instantiation's first launches)
        state["frame"] = rend.compute_frames(header, mode, state["frame"], 16, 7000 + warm, False)
        torch.cuda.synchronize()
        t0p = time.perf_counter()
        state["frame"] = rend.compute_frames(header, mode, state["frame"], args.steps, 7000 + warm, False)
        torch.cuda.synchronize()
        pf_s = (time.perf_counter() - t0p) / args.steps
        rend.set_frame_batch(fb_timed)
        other = {"ms_per_step": round(pf_s * 1e3, 4),
                 "value": round(W * H * (spp if mode in (1, 2) else 1) / pf_s / 1e6, 2),
                 "frames_per_launch": frames_per_launch(fb_other),
                 "dispatch": ("batched: up to %d frames per launch, each frame writing its own ring slot and the "
                              "launch's last frame the image" % frames_per_launch(fb_other)) if fb_other > 1 else
                             "one launch and one image write per frame (the reference's shape, src/main.cpp:604)",
                 "measured": "C++ frame loop (rt_compute_frames), wall clock over the same number of frames"}

    # ---- standalone kernel times (two frames, not overlapped) and work counters (two more,
    # un-timed) on the timed frames' inputs -------------------------------------------------
    if gather is not None:
        gather.finish()
    state["phase"] = "standalone"
    if pipeline:
        rend.enable_pipelining(False)
        streams["out"] = stream
    rend.enable_timing(True)
    rend.reset_stats()
    if host_loop:  # events recorded inside the C++ loop: no host submission gap in the bracket;
        # F frames = one multi-frame launch for modes 3/4, as in the timed region
        state["frame"] = rend.compute_frames(header, mode, state["frame"], rend.F, 7000 + warm, False)
    else:
        for k in range(warm, warm + 2):
            step(k)
    if gather is not None:
        gather.finish()
    solo = {p: rend.kernel_stats(p) for p in progs}
    rend.enable_timing(False)
    # kernel durations the way rocprof's sequential run sees them: a BURST of back-to-back
    # launches of one program on the stream, two events around the burst (no per-launch event,
    # no other program between; a per-launch event pair adds ~7 us, 20% of a config (b) frame),
    # the last rendered slot re-rendered with its own header (a trace pass rewrites identical
    # values; a post-process re-filters its previous output: the same flag-, history- and
    # byte-pattern, since those follow the normals and depth)
    # the bursts below re-run the last slot's programs in place (a post-process re-filters its own
    # output), so the ring no longer holds the frames the whole-frame reference renders: the
    # gathered frames are checked up to here (warm-up, timed and standalone frames), not after
    state["verify_on"] = False
    burst = {}
    if True:
        slot = (state["frame"] - 1) % rend.F
        # ~12 ms of launches per burst (AO at (d): 6, post: 24 ... hybrid at (b): 200)
        reps_for = lambda p: int(min(400, max(6, 12.0 / max(solo[p][1] / max(solo[p][0], 1), 0.01))))
        for prog in progs:
            reps = reps_for(prog)
            rend.run_program(prog, slot)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                rend.run_program(prog, slot)
            e1.record(stream)
            e1.synchronize()
            burst[prog] = (e0.elapsed_time(e1) / reps, reps)
    rend.enable_counters(True)
    rend.read_counters(reset=True)
    ncount = 2
    for k in range(warm, warm + ncount):
        step(k)
    if gather is not None:
        gather.finish()
    counts = rend.read_counters(reset=True)
    rend.enable_counters(False)

    t_max = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    host_max = torch.tensor([host_s], dtype=torch.float64, device=cdev)
    strip_ms = torch.zeros(world, dtype=torch.float64, device=cdev)
    strip_ms[plan.strip_of(rank)] = sum(tot / max(n_l, 1) for n_l, tot in solo.values())  # standalone kernel ms
    # per rank: median and mean ms from "strip rendered" to "its gather transfers complete"
    g_ms = torch.zeros(world, 2, dtype=torch.float64, device=cdev)
    if gms:
        g_ms[rank, 0] = float(np.median(gms))
        g_ms[rank, 1] = float(np.mean(gms))
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(host_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(strip_ms)
        dist.all_reduce(g_ms)
    elapsed = float(t_max.item())

    if rank == 0:
        rays_per_frame = W * H * (spp if mode in (1, 2) else 1)
        value = rays_per_frame * args.steps / elapsed / 1e6
        ms = elapsed / args.steps * 1e3
        dom = progs[0]
        # Kernel duration for the roofline: the HIP-event span of a launch.  Without pipelining
        # that is the timed region's average.  Pipelined, consecutive AO launches overlap (frame
        # k+1's AO fills frame k's tail), so a timed span is not a duration: the standalone
        # launches after the timed region are used, and the sustained rate (per frame) is given
        # beside it.
        n_l, tot = kstats[dom]
        timed_ms = tot / max(n_l, 1)
        solo_ms = solo[dom][1] / max(solo[dom][0], 1)
        avg_ms = burst[dom][0]
        tests = counts["tests"] / ncount
        exec_tests = counts["executed_lane_tests"] / ncount
        eff_tflops = FLOP_PER_TEST * tests / (avg_ms * 1e-3) / 1e12
        exec_tflops = FLOP_PER_TEST * exec_tests / (avg_ms * 1e-3) / 1e12
        sustained = FLOP_PER_TEST * tests / (elapsed / args.steps) / 1e12
        band_px = (r1 - r0 + (2 if mode in (1, 2) and world > 1 else 0)) * W
        hbm_alg = BYTES_PER_PIXEL[dom] * band_px / (avg_ms * 1e-3) / 1e9
        binfo = build_info()
        # the committed PMC / SQ files are whole-frame launches: attached only at N = 1
        traffic_data, traffic_src = load_traffic(args.config, binfo.get("src_sha1")) if world == 1 else (None, None)
        # a counter run's values are per dispatch: with multi-frame launches (modes 2-4 in the C++
        # loop) a dispatch holds up to F frames, so only runs taken one frame per dispatch
        # (--frame-batch 1, recorded as frames_per_dispatch) are comparable with a per-frame kernel_ms
        per_frame_launches = not host_loop or fb_timed == 1
        per_dispatch_ok = lambda d: d is not None and per_frame_launches and (
            not host_loop or d.get("frames_per_dispatch") == 1)
        hw_note = None
        if traffic_data is not None and not per_dispatch_ok(traffic_data):
            hw_note = f"{traffic_src}: per multi-frame dispatch, not per frame; omitted"
            traffic_data, traffic_src = None, None
        # the hardware's view: VALU wave-instructions the kernel issues per launch (SQ_INSTS_VALU,
        # committed counter run of this library build) over what the launch could issue at the
        # spec rate (one wave64 FP32 FMA, 128 FLOP, per 2 clocks per SIMD: the peak) and at the
        # rate a dense v_fma_f32 stream sustains on this GPU
        sq, sq_src = load_sq(args.config, binfo.get("src_sha1")) if world == 1 else (None, None)
        if sq is not None and not per_dispatch_ok(sq):
            hw_note = (hw_note + "; " if hw_note else "") + f"{sq_src}: per multi-frame dispatch, not per frame; omitted"
            sq, sq_src = None, None
        valu = None
        if sq:
            # the dominant program's kernel; of its instantiations the one with the most dispatches
            # (the timed form, not the counted one) where the file records dispatch counts
            sub = {1: "ao_", 3: "ao_", 4: "phong", 5: "hybrid"}[dom]
            names = [k for k in sq["kernels"] if sub in k] or list(sq["kernels"])
            disp = sq.get("dispatches", {})
            kern = sq["kernels"][max(names, key=lambda k: disp.get(k, 0))]
            insts = kern.get("SQ_INSTS_VALU")
            if insts:
                spec = PEAK_FP32_TFLOPS * 1e12 / 128 * avg_ms * 1e-3
                valu = {"insts_per_launch": insts, "frac_of_spec_issue": round(insts / spec, 4),
                        "frac_of_sustained_fma_issue": round(insts / (VALU_FMA_RATE * avg_ms * 1e-3), 4),
                        "salu_insts_per_launch": kern.get("SQ_INSTS_SALU"),
                        "source": sq_src, "on_this_build": sq.get("src_sha1") == binfo.get("src_sha1")}
        # roofline on EXECUTED work: the VALU issue fraction of this build's counters (each wave64
        # VALU instruction counted as one FMA's 128 FLOP, i.e. issue slots); without them, the
        # lane-tests the kernel executes x 20 FLOP (a lower bound: per-sample setup, hashes and
        # shading are not counted).  The reference's brute-force count is `effective_*`.
        if valu and valu["on_this_build"]:
            achieved = valu["insts_per_launch"] * 128 / (avg_ms * 1e-3) / 1e12
            basis = ("executed: SQ_INSTS_VALU per launch (rocprofv3 --pmc run of this library build, %s) x 128 FLOP "
                     "(one wave64 FMA per instruction = one issue slot) per kernel second; frac = VALU issue "
                     "fraction of the spec peak" % sq_src)
        else:
            achieved = exec_tflops
            basis = ("executed: lane-tests the kernel runs (work counters) x 20 FLOP per kernel second (no SQ "
                     "counters of this build; a lower bound on executed work)")
        roof = {
            "bound": "valu",
            "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "basis": basis,
            "traffic": traffic_data.get(str(dom)) if traffic_data else None,
            "kernel": {1: "aop_compute (ao_kernel)", 3: "ao_compute (ao_kernel)", 4: "p_compute (phong_kernel)",
                       5: "h_compute (hybrid_kernel)"}[dom],
            "kernel_ms": round(avg_ms, 4),
            "kernel_ms_measured": ("%d back-to-back launches between two events after the timed region (the shape of "
                                   "rocprof's sequential run; tools/burst_check.py compares the two)" % burst[dom][1]),
            "burst_launches": burst[dom][1],
            "kernel_ms_timed_span": None if pipeline or host_loop else round(timed_ms, 4),
            "kernel_ms_standalone_events": round(solo_ms, 4),
            "executed_test_tflops": round(exec_tflops, 2),
            "executed_lane_tests_per_launch": exec_tests,
            "effective_tflops": round(eff_tflops, 2),
            "effective_frac": round(eff_tflops / PEAK_FP32_TFLOPS, 4),
            "effective_basis": ("the reference's brute-force ray-shape tests (every segment tests every shape, 20 FLOP "
                                "each) per kernel second: work the culled kernel does NOT execute "
                                "(useful_test_ratio = brute-force / executed lane-tests), so it can exceed the peak"),
            "sustained_effective_tflops_per_frame": round(sustained, 2),
            "flop_per_launch_brute_force": FLOP_PER_TEST * tests,
            "tests_per_launch": tests,
            "segments_per_sample": round(counts["segments"] / max(counts["samples"], 1), 4),
            "useful_test_ratio": round(counts["tests"] / max(counts["executed_lane_tests"], 1), 4),
            "hbm": {"achieved": round(hbm_alg, 2), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                    "frac": round(hbm_alg / PEAK_HBM_GBPS, 6),
                    "bytes_per_launch": BYTES_PER_PIXEL[dom] * band_px},
            "traffic_source": traffic_src,
            # the PMC run's library build vs this one: equal source hashes = measured on this kernel code
            "traffic_src_sha1": traffic_data.get("src_sha1") if traffic_data else None,
            "traffic_on_this_build": bool(traffic_data and traffic_data.get("src_sha1") == binfo.get("src_sha1")),
        }
        if hw_note:
            roof["hardware_counters_note"] = hw_note
        if valu:
            roof["valu_issue"] = valu
        out = {
            "metric": "Mrays/s + ms/frame at 3840x2160, 16 AO samples, 64 spheres; 1/2/4/8 GPU",
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ring_fill_frames": ring_fill, "settle_frames": settle,
            "settle_ms": args.warm_ms, "ms_per_step": round(ms, 4),
            "ms_per_step_median": round(float(np.median(intervals)), 4) if intervals else None,
            "ms_per_step_median_of": ("per-frame completion intervals (events on the output stream)" if not host_loop
                                      else f"{len(intervals)} chunks of the C++ frame loop") if intervals else None,
            "frame_intervals_ms": [round(v, 3) for v in intervals] if not host_loop else None,
            "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": desc, "width": W, "height": H, "spheres": S, "spp": spp, "mode": mode,
                       "max_depth": 20, "strips": plan.bounds,
                       "parallelism": f"{world} row strip(s), cost-balanced" + ((", RCCL gather to rank 0" if args.backend == "nccl" else ", gloo gather to rank 0 (host-staged rehearsal)") if world > 1 else "")
                       + (", pipelined frames: consecutive AO passes on 2 alternating streams, post-process on a 3rd"
                          if pipeline else "")
                       + (", frame loop in C++ (rt_compute_frames)" if host_loop else "")
                       + ((", one launch per frame" if fb_timed == 1 else
                           ", up to %d frames per launch (each writes its colour slot; the image by the launch's "
                           "last frame)" % frames_per_launch(fb_timed)) if host_loop and mode in (2, 3, 4) else "")},
            "roofline": roof,
            # host time per frame inside the frame calls = enqueue + waits for a free staging
            # buffer (back-pressure: the host runs up to 8 uploads ahead of the GPU)
            "host_enqueue_ms_per_step": round(max(0.0, host_s * 1e3 - host_wait_ms) / args.steps, 4),
            "host_backpressure_ms_per_step": round(host_wait_ms / args.steps, 4),
            "build": binfo,
            "tile_schedule": ("off: workgroups in the plain order" if args.no_tile_schedule else
                              "longest first (rt_set_tile_schedule: mode-4 tiles by the bounce rounds of recent "
                              "frames; state %d)" % rend.tile_schedule_state()),
        }
        if host_loop and mode in (2, 3, 4):
            out["dispatch"] = (("one launch and one image write per frame (rt_set_frame_batch(1)): the reference's "
                                "dispatch shape (src/main.cpp:604)") if fb_timed == 1 else
                               ("batched: up to %d frames per launch, each frame writing its own ring slot and the "
                                "launch's last frame the image" % frames_per_launch(fb_timed)))
            out["frames_per_launch"] = frames_per_launch(fb_timed)
            if other is not None:
                out["batched_dispatch" if fb_other > 1 else "per_frame_dispatch"] = other
        if balance_info is not None:
            sm = strip_ms.cpu().tolist()
            balance_info.update({"strip_ms": [round(t, 4) for t in sm], "imbalance": round(imbalance(sm), 4)})
            out["config"]["balance"] = balance_info
        if ref is not None:
            out["verify"] = {"frames_checked": state["checked"], "mismatched": state["mismatch"],
                             "what": ("every frame up to the kernel-time bursts (warm-up, settle, timed and standalone "
                                      "frames)" if args.verify else f"the first {VERIFY_FIRST} frames (warm-up)")
                             + ": the gathered frame vs a whole-frame render on rank 0, bit for bit",
                             "diag": state.get("diag", [])[:6]}
        if world > 1:
            out["collective"] = {"backend": args.backend if args.backend == "gloo" else "nccl (RCCL)",
                                 "world_size": dist.get_world_size(), "op": "batch_isend_irecv strip gather to rank 0"}
            gm = g_ms.cpu().tolist()
            out["ranks"] = [{"rank": i, "device": devices[i]["device"], "pci_bus": devices[i]["pci_bus"],
                             "strip": plan.strip_of(i), "rows": list(plan.rows(i)),
                             "gather_bytes_per_frame": plan.strip_bytes(i),
                             "gather_ms_median": round(gm[i][0], 4) if gms else None,
                             "gather_ms_mean": round(gm[i][1], 4) if gms else None} for i in range(world)]
            tot_b = sum(plan.strip_bytes(i) for i in range(world))
            out["gather"] = {
                "root_strip": plan.root_strip, "bytes_per_frame": tot_b,
                "max_rank_bytes_per_frame": max(plan.strip_bytes(i) for i in range(world)),
                "root_gather_ms_median": round(gm[0][0], 4) if gms else None,
                "root_gather_ms_mean": round(gm[0][1], 4) if gms else None,
                "measured": ("events per timed frame (nccl): on each rank's output stream before its "
                             "batch_isend_irecv (the strip is rendered) and on a side stream ordered after the "
                             "transfers' completion (Work.wait); rank 0's span ends when every strip has landed, "
                             "so it includes waiting for the slowest rank's render" if gms else
                             "not timed (gloo rehearsal: host-staged)"),
                "link_model": links,
                "predicted_frame_ms": balance_info["predicted_frame_ms"] if balance_info else None}
            out["launched_by"] = os.environ.get("RTRT_BENCH_LAUNCHER", "external launcher")
        if mode == 1:
            # standalone launches: in the pipelined timed region the post-process shares the GPU
            # with the next frame's AO pass, so its event span is not a kernel duration
            pms = burst[2][0]
            n_p, tot_p = solo[2]
            post_px = (r1 - r0) * W * ncount  # every pixel of the strip, per counted launch
            post_bytes = (POST_BYTES_PIXEL * post_px + POST_BYTES_FILTERED * counts["filtered_pixels"]
                          + POST_BYTES_SLOT_READ * counts["history_read"]
                          + POST_BYTES_SLOT_ACCEPTED * counts["history_accepted"]) / ncount
            pbw = post_bytes / (pms * 1e-3) / 1e9
            out["roofline_post"] = {"bound": "hbm", "achieved": round(pbw, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                                    "frac": round(pbw / PEAK_HBM_GBPS, 4), "kernel": "aop_postprocessing (post_kernel)",
                                    "kernel_ms": round(pms, 4),
                                    "measured": ("%d back-to-back launches between two events after the timed region "
                                                 "(the shape of rocprof's sequential run)" % burst[2][1]),
                                    "burst_launches": burst[2][1],
                                    "kernel_ms_standalone_events": round(tot_p / max(n_p, 1), 4),
                                    "bytes_per_launch": round(post_bytes),
                                    "byte_model": "52 B/pixel + 20 B/filtered pixel + 20 B/history slot read + 16 B/slot accepted",
                                    "filtered_fraction": round(counts["filtered_pixels"] / max(post_px, 1), 4),
                                    "history_slots_read_per_filtered_pixel": round(counts["history_read"] / max(counts["filtered_pixels"], 1), 3),
                                    "traffic": traffic_data.get("2") if traffic_data else None,
                                    "traffic_over_model": (round(traffic_data["2"] / post_bytes, 3)
                                                           if traffic_data and traffic_data.get("2") else None)}
        if world == 1 and args.config in ("ref", "a"):
            out["ssbo_path"] = ssbo_path(args.config, gpu)
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
            except Exception as e:  # the checker must not take the GPU number down with it
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    rend.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    rc = launch_ranks(sys.argv[1:])
    if rc is not None:  # the launcher's status; killed by a signal (rc < 0): 128 + signal
        sys.exit(rc if rc >= 0 else 128 - rc)
    from real_time_ray_tracer_amd.dist import run_rank

    run_rank(main)
