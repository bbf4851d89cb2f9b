#!/usr/bin/env python
"""Per-kernel register / LDS / occupancy table of the production library, from the compiler's
kernel-resource-usage remarks (hipcc -Rpass-analysis=kernel-resource-usage, device pass only).

    python tools/resource_usage.py [--ab] [VFLAGS ...] [> profiles/rNN_resource_usage.txt]

The rocprofv3 kernel trace reports the same VGPR/SGPR/LDS fields per dispatch (its VGPR count
is in allocation granules: arch VGPRs rounded up to 8); this table is what DESIGN.md's
occupancy statements cite.
"""
from __future__ import annotations

import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "real_time_ray_tracer_amd/csrc/rt_kernels.hip"
AB_SRC = ROOT / "tools/ab/rt_kernels_ab.hip"  # the A/B tools library's launcher (make ablib)
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", f"-I{ROOT / 'include'}",
         f"-I{ROOT / 'real_time_ray_tracer_amd/csrc'}"]
FIELDS = ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill",
          "VGPRs Spill", "LDS Size [bytes/block]")


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def main():
    ab = "--ab" in sys.argv
    defines = [a for a in sys.argv[1:] if a != "--ab"]  # a variant's VFLAGS (-D..., -mllvm ...)
    cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *defines, "-x", "hip", "-c", str(AB_SRC if ab else SRC),
           "-o", "/dev/null", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"]
    text = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark: (.*) \[-Rpass-analysis", line)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in body:
            k, v = body.rsplit(":", 1)
            if k.strip() in FIELDS:
                cur[k.strip()] = v.strip()
    names = demangle([r["name"] for r in rows])
    short = [re.sub(r"\(anonymous namespace\)::|rt::|HIP_vector_type<float, 4u>", "", n) for n in names]
    short = [re.sub(r"\(.*\)$", "", n) for n in short]
    w = max(len(s) for s in short) if short else 10
    hdr = ["VGPR", "SGPR", "scratch", "waves/SIMD", "SGPR spill", "VGPR spill", "LDS(static)"]
    print(f"{'kernel':<{w}}  " + "  ".join(f"{h:>10}" for h in hdr))
    for s, r in sorted(zip(short, rows)):
        vals = [r.get(k, "?") for k in ("VGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
                                        "SGPRs Spill", "VGPRs Spill", "LDS Size [bytes/block]")]
        print(f"{s:<{w}}  " + "  ".join(f"{v:>10}" for v in vals))


if __name__ == "__main__":
    main()
