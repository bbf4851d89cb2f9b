#!/usr/bin/env python
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads
exactly 1/2 of the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Median over launches (warm-up, timed and
counted frames alike).  Keys are RT_PROG ids: 1 aop_compute, 2 aop_postprocessing,
3 ao_compute, 4 p_compute, 5 h_compute.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <config> <out.json>
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = {"post_kernel": "2", "phong_kernel": "4", "hybrid_kernel": "5"}


def kernel_key(name, mode_cfg):
    for k, v in KERNELS.items():
        if k in name:
            return v
    if "ao_" in name:  # the AO trace kernels serve aop_compute (mode 1) or ao_compute (mode 2)
        return "1" if mode_cfg == 1 else "3"
    return None


def collect(d, counter, mode_cfg):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = kernel_key(r["Kernel_Name"], mode_cfg)
            if k:
                vals.setdefault(k, []).append(float(r["Counter_Value"]))
    return vals


def frames_per_dispatch(mode_cfg, bench_args):
    """1 when every dispatch renders one frame: mode 1 always; modes 2-4 unless bench.py ran
    with --frame-batch > 1 (its default, 1, is one launch per frame).  None otherwise."""
    import shlex
    fb = 1
    a = shlex.split(bench_args)
    for i, x in enumerate(a):
        if x == "--frame-batch" and i + 1 < len(a):
            fb = int(a[i + 1])
        elif x.startswith("--frame-batch="):
            fb = int(x.split("=", 1)[1])
    return 1 if mode_cfg == 1 or fb == 1 else None


def main():
    fetch_dir, write_dir, cfg, out = sys.argv[1:5]
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import CONFIGS
    mode_cfg = CONFIGS[cfg][4]
    fe = collect(fetch_dir, "FETCH_SIZE", mode_cfg)
    wr = collect(write_dir, "WRITE_SIZE", mode_cfg)
    res = {"config": cfg, "units": "bytes per launch (FETCH_SIZE*2*1024 + WRITE_SIZE*1024, median)",
           "bench_args": os.environ.get("BENCH_ARGS", ""),
           "frames_per_dispatch": frames_per_dispatch(mode_cfg, os.environ.get("BENCH_ARGS", ""))}
    try:  # the library build the counters were taken on (make lib writes BUILD_INFO)
        info = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                           "real_time_ray_tracer_amd", "BUILD_INFO")))
        res["src_sha1"], res["commit"] = info.get("src_sha1"), info.get("commit")
    except Exception:
        res["src_sha1"] = res["commit"] = None
    for k in sorted(set(fe) | set(wr)):
        f = statistics.median(fe.get(k, [0.0])) * 2 * 1024
        w = statistics.median(wr.get(k, [0.0])) * 1024
        res[k] = round(f + w)
        res[k + "_read"] = round(f)
        res[k + "_write"] = round(w)
        res[k + "_launches"] = len(wr.get(k, []))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
