#!/usr/bin/env python
"""Per-launch durations and the idle gaps between consecutive launches in a rocprofv3 kernel
trace (--kernel-trace --output-format csv): where a one-launch-per-frame loop loses its time.

    python tools/kernel_gaps.py <run_kernel_trace.csv> [kernel-substring ...]
"""
import csv
import statistics as st
import sys


def main():
    path = sys.argv[1]
    subs = sys.argv[2:] or ["kernel"]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    short = lambda n: n.replace("void ", "").replace("rt::(anonymous namespace)::", "").split("(rt::")[0][:90]
    for sub in subs:
        sel = [(a, b, n) for a, b, n in rows if sub in n]
        if not sel:
            continue
        durs = [(b - a) / 1e3 for a, b, _ in sel]
        print(f"{sub}: {len(sel)} launches, duration us: median {st.median(durs):.2f}, mean {st.mean(durs):.2f}, "
              f"min {min(durs):.2f}, max {max(durs):.2f}")
        names = {}
        for a, b, n in sel:
            names.setdefault(short(n), []).append((b - a) / 1e3)
        for n, d in names.items():
            print(f"   {len(d):5d} x {st.median(d):9.2f} us median  {n}")
    # gaps between consecutive launches (any kernel), and what ran before each
    gaps = [(rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
    if gaps:
        print(f"all kernels: {len(rows)} launches, gap to the next launch us: median {st.median(gaps):.2f}, "
              f"p10 {sorted(gaps)[len(gaps) // 10]:.2f}, p90 {sorted(gaps)[9 * len(gaps) // 10]:.2f}")
        sub = subs[0]
        seq = [i for i in range(len(rows) - 1) if sub in rows[i][2] and sub in rows[i + 1][2]]
        if seq:
            g = [gaps[i] for i in seq]
            print(f"{sub} -> {sub}: {len(g)} consecutive pairs, gap us: median {st.median(g):.2f}, "
                  f"p10 {sorted(g)[len(g) // 10]:.2f}, p90 {sorted(g)[9 * len(g) // 10]:.2f}; "
                  f"period (start to start) median {st.median([(rows[i + 1][0] - rows[i][0]) / 1e3 for i in seq]):.2f}")


if __name__ == "__main__":
    main()
