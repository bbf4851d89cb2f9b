#!/usr/bin/env python
"""The bench line's kernel_ms against rocprof's own durations of the same launches, from a
rocprofv3 --kernel-trace CSV of `bench.py ... --no-cpu-baseline` and that run's JSON line.

bench.py times each program of the frame (mode 1: the AO pass, then the post-process) as a burst
after the timed region: 1 warm-up launch + `burst_launches` back-to-back launches between two
events (kernel_ms = the span / launches); the 2 counted frames follow.

    python tools/burst_check.py <run_kernel_trace.csv> <bench.json>
"""
import csv
import json
import statistics
import sys

KEYS = {1: ("ao_batch_kernel", "post_kernel"), 2: ("ao_batch_kernel",), 3: ("phong_kernel",), 4: ("hybrid_kernel",)}



def main():
    path, bench = sys.argv[1], sys.argv[2]
    line = json.loads([l for l in open(bench) if l.startswith("{")][-1])
    mode = line["config"]["mode"]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    print(f"{path}\nbench line: {bench} (config {line['config']['workload'][:60]}...)")
    counted = 2  # launches per program after the bursts (the counted frames)
    for i, key in enumerate(KEYS[mode]):
        ds = [(b - a) / 1e6 for a, b, n in rows if key + "<" in n or key + "(" in n]
        rl = line["roofline"] if i == 0 else line["roofline_post"]
        reps = rl["burst_launches"]
        # mode 1: the post-process burst runs after the AO burst, so the AO launches after the AO
        # burst are only the counted ones; the same holds for the post-process
        sel = ds[-(reps + 1 + counted):-counted]
        m = statistics.mean(sel[1:])
        print(f"{key}: burst of {reps} (+1 warm-up) launches: median {statistics.median(sel[1:]):.4f}, "
              f"min {min(sel[1:]):.4f}, max {max(sel[1:]):.4f} ms")
        print(f"  rocprof mean {m:.4f} ms; bench kernel_ms {rl['kernel_ms']:.4f} ms; bench / rocprof = "
              f"{rl['kernel_ms'] / m:.4f}")

if __name__ == "__main__":
    main()
