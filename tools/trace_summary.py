#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace of `bench.py --warmup W --steps K` for profiles/:
per-launch durations of the renderer's kernels in dispatch order and the mean over the timed
launches (W warm-up first, then K timed, then 2 standalone frames (not overlapped), then the 2
counted frames), to compare with the bench line's live HIP-event kernel_ms and
kernel_ms_standalone.  In pipelined mode 1 the timed post-process launches overlap the next
frame's AO pass, so their spans are not kernel durations; the standalone ones are.

    python tools/trace_summary.py gpurun_out/<tag>/kt/run_kernel_trace.csv 8 10 "<command>"
"""
import csv
import sys


def main():
    path, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    cmd = sys.argv[4] if len(sys.argv) > 4 else ""
    launches = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            for key in ("ao_batch_kernel", "ao_kernel", "post_kernel", "phong_kernel", "hybrid_kernel"):
                if key + "<" in name or key + "(" in name:
                    d = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
                    # one entry per instantiation (template arguments included): the counted
                    # frames run the counter-enabled instantiation, with its own registers
                    inst = name.split("(rt::FrameParams")[0].replace("void rt::(anonymous namespace)::", "")
                    inst = inst.replace("rt::(anonymous namespace)::", "")
                    launches.setdefault(key, []).append((int(row["Dispatch_Id"]), d, row["VGPR_Count"],
                                                         row["SGPR_Count"], row["LDS_Block_Size"], inst))
    if cmd:
        print(cmd)
    print(f"per-launch durations (ms), in dispatch order: {warm} warm-up, {steps} timed, 2 standalone, "
          f"2 counted (work counters on)")
    print("rocprof's VGPR_Count is about half the compiler's VGPR count (tools/resource_usage.py: the production "
          "AO kernel 72 -> 36, post_kernel 56 -> 28) and LDS_Block_Size counts static LDS only")
    for key, ls in launches.items():
        ls.sort()
        ds = [d for _, d, *_ in ls]
        timed = ds[warm:warm + steps]
        insts = {}
        for _, _, v, sg, lds, inst in ls:
            insts.setdefault(inst, (v, sg, lds, 0))
            insts[inst] = insts[inst][:3] + (insts[inst][3] + 1,)
        for inst, (v, sg, lds, n) in insts.items():
            print(f"{key}: {inst}: {n} launches, vgpr={v} sgpr={sg} lds(static)={lds}")
        if len(ds) <= 40:
            print(f"  all={[round(d, 3) for d in ds]}")
        else:  # long warm-up (bench.py settles the clock first): the launches after it
            print(f"  {len(ds)} launches; after the {warm} warm-up: {[round(d, 3) for d in ds[warm:]]}")
        if timed:
            print(f"  timed mean={sum(timed) / len(timed):.4f} ms")
        solo = ds[warm + steps:warm + steps + 2]
        if solo:
            print(f"  standalone mean={sum(solo) / len(solo):.4f} ms")


if __name__ == "__main__":
    main()
