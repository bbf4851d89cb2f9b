#!/usr/bin/env python
"""How far rounds 1-4's binary32 polynomial sin in random() moved the frames away from the
mathematical sin ("measure first").  TEST/MEASUREMENT TOOL (CPU only).

Renders configs (b), (c) and (d) (3 frames each, the bench's scene and per-frame rand_buffer
seeds) with two builds of the CPU oracle:
  * round 4's oracle (git 9329488: rto_sin = a binary32 reduction by 2 pi and a degree-11
    polynomial, the kernels' sin of that round), compiled here from that commit's source;
  * this round's oracle (rto_sin = the correctly rounded sin, which a plain re-execution
    (float)sin((double)x) reproduces except at double-rounding inputs; none in 84 M floats of the
    configs' binades, tests/test_sin_cpu.py);
and reports the fraction of image channels within the north-star tolerance
(|a - b| <= 1e-4 max(|a|, |b|) + 1e-6) and of depth / normal values that are bit-identical.

    python tools/sin_change_effect.py [--configs b,c,d] [--frames 3] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OLD = "9329488"


def build_old(tmp: Path) -> Path:
    for f in ("oracle/rt_oracle.c", "oracle/rt_oracle.h", "include/rt/layout.h"):
        dst = tmp / f
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_bytes(subprocess.run(["git", "show", f"{OLD}:{f}"], cwd=ROOT, check=True,
                                       capture_output=True).stdout)
    so = tmp / "librt_oracle_r4.so"
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-ffp-contract=off", "-fopenmp", "-fPIC", "-std=c99", "-shared",
                    "-o", str(so), str(tmp / "oracle/rt_oracle.c"), "-lm"], check=True)
    return so


def render(lib_path: str, cfg: str, frames: int, threads: int) -> dict:
    """one oracle build, in a child process (the oracle module loads one library per process)"""
    code = f"""
import sys, numpy as np
sys.path.insert(0, {str(ROOT)!r})
import oracle
if {lib_path!r}:
    from pathlib import Path
    oracle.LIB_PATH = Path({lib_path!r})
from bench import CONFIGS, config_header
from real_time_ray_tracer_amd import SSBO
W, H, S, spp, mode, _ = CONFIGS[{cfg!r}]
h = config_header({cfg!r})
s = SSBO(h, W, H)
d = oracle.dims(W, H, h.S, h.AA)
img = np.zeros((H, W, 4), np.float32)
f = 0
for k in range({frames}):
    if mode in (1, 2):
        h.fill_rand_buffer(7000 + k)
    else:
        h.moving_light(False)
    h.set_mode(f, h.num_objects)
    s.set_header(h)
    f = oracle.dispatch(s.data, d, mode, f, img, nthreads={threads})
slot = (f - 1) % 8
np.savez(sys.argv[1], image=img, depth=s.depth[slot], normals=s.normals[slot])
"""
    with tempfile.NamedTemporaryFile(suffix=".npz") as out:
        subprocess.run([sys.executable, "-c", code, out.name], check=True)
        z = np.load(out.name)
        return {k: z[k] for k in z.files}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="b,c,d")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    res = {}
    with tempfile.TemporaryDirectory() as td:
        old_so = build_old(Path(td))
        for cfg in a.configs.split(","):
            o = render(str(old_so), cfg, a.frames, a.threads)
            n = render("", cfg, a.frames, a.threads)
            x, y = o["image"][..., :3], n["image"][..., :3]
            close = np.abs(x - y) <= 1e-4 * np.maximum(np.abs(x), np.abs(y)) + 1e-6
            same_d = np.all(o["depth"].view(np.uint32) == n["depth"].view(np.uint32), axis=-1)
            same_n = np.all(o["normals"].view(np.uint32) == n["normals"].view(np.uint32), axis=-1)
            res[cfg] = {"frames": a.frames, "image_channels_within_1e-4": round(float(close.mean()), 6),
                        "pixels_all_channels_within_1e-4": round(float(close.all(axis=-1).mean()), 6),
                        "max_abs_diff": float(np.abs(x - y).max()),
                        "depth_bit_identical": round(float(same_d.mean()), 6),
                        "normals_bit_identical": round(float(same_n.mean()), 6)}
            print(cfg, json.dumps(res[cfg]), flush=True)
    print(json.dumps({"round4_sin_vs_math_sin": res}))


if __name__ == "__main__":
    main()
