"""bench.py --gpus N without a launcher renders on N ranks, on the GPU box:
2 ranks share its one GPU (--backend gloo: the host-staged gather rehearsal), split config (c)
into row strips, and rank 0 checks the gathered frames against its own whole-frame render bit
for bit (the first 2 frames, outside the timed region).  The CPU test of the launch itself is
tests/test_dist_gloo.py::test_bench_gpus_n_starts_n_ranks_without_a_launcher."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_bench_gpus_2_renders_on_2_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "2", "--backend", "gloo", "--config", "c",
                        "--steps", "4", "--warmup", "2", "--warm-ms", "50", "--no-cpu-baseline", "--no-alt-dispatch",
                        "--dist-timeout", "100"], capture_output=True, text=True, timeout=110, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    print(json.dumps({k: out.get(k) for k in ("n_gpus", "value", "ms_per_step", "verify", "ranks", "launched_by")}))
    assert out["n_gpus"] == 2
    assert out["verify"]["frames_checked"] >= 2 and out["verify"]["mismatched"] == 0, out["verify"]
    assert [q["rank"] for q in out["ranks"]] == [0, 1]
    # the two strips partition the frame; rank 0 owns the plan's root strip (gather-aware plan,
    # dist.probe_links measured the host-staged gloo path here) and sends nothing
    spans = sorted(tuple(q["rows"]) for q in out["ranks"])
    assert spans[0][0] == 0 and spans[0][1] == spans[1][0] and spans[1][1] == 1080
    g = out["gather"]
    assert out["ranks"][0]["strip"] == g["root_strip"] and out["ranks"][0]["gather_bytes_per_frame"] == 0
    r1 = out["ranks"][1]["rows"]
    assert out["ranks"][1]["gather_bytes_per_frame"] == (r1[1] - r1[0]) * 1920 * 16
    assert g["link_model"]["link_gbps"] > 0 and g["predicted_frame_ms"]["bound_ms"] > 0
    assert out["launched_by"].startswith("bench.py --gpus 2")
