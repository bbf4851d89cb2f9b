#!/usr/bin/env python
"""GPU occupancy timeline of a rocprofv3 kernel trace: busy fraction (any renderer kernel
running), overlap between kernels, and idle gaps between consecutive frames.

    python tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [skip_first_n_launches]
"""
import csv
import sys


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            if "ao_batch_kernel" in n or "post_kernel" in n or "ao_kernel" in n:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "ao" if "ao_" in n else "post"))
    rows.sort()
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = rows[skip:]
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    # busy = union of intervals
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    ao = [(s, e) for s, e, k in rows if k == "ao"]
    ov = sum(max(0, min(ao[i][1], ao[i + 1][1]) - ao[i + 1][0]) for i in range(len(ao) - 1))
    span = t1 - t0
    print(f"launches {len(rows)} span {span / 1e6:.3f} ms busy {busy / span:.3f} gaps {len(gaps)} "
          f"total gap {sum(gaps) / 1e6:.3f} ms max gap {max(gaps, default=0) / 1e3:.1f} us; "
          f"AO-AO overlap {ov / 1e6:.3f} ms over {len(ao) - 1} pairs; mean AO span "
          f"{sum(e - s for s, e in ao) / len(ao) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
