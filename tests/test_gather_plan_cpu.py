"""The gather-aware strip planner (rt_plan_strips_gather, host-only C ABI) on the CPU.

The reference blits one whole frame (src/main.cpp:783-797) rendered by one
glDispatchCompute(WIDTH, HEIGHT, 1) (src/main.cpp:604); split over N GPUs, every strip but the
root's crosses one xGMI link into rank 0 each frame.  VERDICT r5 item 1: the root must own the
strip with the most bytes, and the plan must bound max(render, per-link copy, root ingest)."""
import itertools
import re

import numpy as np
import pytest

from conftest import ROOT

W_D = 3840  # config (d)
ROW_BYTES = W_D * 16


def _r05last_profile(n: int) -> np.ndarray:
    """The committed round-5 (d) calibrated strip profile (tools/strip_scaling.py output): the
    kept plan's bounds and per-strip ms, spread evenly over each strip's rows (ms per row)."""
    txt = (ROOT / "profiles" / f"r05last_strip_scaling_d_n{n}_calibrated.txt").read_text()
    plans = re.findall(r"calibration plan \d+: \[([\d, ]+)\] strip ms \[([\d., ]+)\]", txt)
    b, t = plans[-1]
    b = [int(x) for x in b.split(",")]
    t = [float(x) for x in t.split(",")]
    assert len(b) == n + 1 and b[-1] == 2160
    return np.concatenate([np.full(b[i + 1] - b[i], t[i] / (b[i + 1] - b[i])) for i in range(n)]), b


def _bound(row_ms, bounds, root, W, link, ingest):
    """numpy restatement of rt_strip_gather_bound"""
    n = len(bounds) - 1
    render = max(row_ms[bounds[i]:bounds[i + 1]].sum() for i in range(n))
    nb = [(bounds[i + 1] - bounds[i]) * W * 16 for i in range(n) if i != root]
    link_ms = max(nb) / (link * 1e6) if nb and link > 0 else 0.0
    ing = sum(nb) / (ingest * 1e6) if ingest > 0 else 0.0
    return max(render, link_ms, ing)


def test_r05last_d_n8_root_owns_the_sky_strip_and_links_fit():
    """At N = 8 on the round-5 (d) profile with the MI355X's 153.6 GB/s xGMI links (76.8 GB/s each
    way) the root owns the largest strip, every non-root strip is <= 21 MB, and the frame bound is
    the render bound (the old plan, root = bottom strip, was link-bound at 0.45 ms)."""
    from real_time_ray_tracer_amd.dist import gather_bound, gather_bounds

    row, old = _r05last_profile(8)
    link = 76.8
    b, root, pred = gather_bounds(row, 8, W_D, link, 7 * link)
    rows = np.diff(b)
    assert rows[root] == rows.max()
    nonroot = [rows[i] * ROW_BYTES for i in range(8) if i != root]
    assert max(nonroot) <= 21e6, max(nonroot)
    assert pred["bound_ms"] == pytest.approx(pred["render_ms"], rel=1e-9)
    assert pred["link_ms"] < pred["render_ms"] and pred["ingest_ms"] < pred["render_ms"]
    assert pred["render_ms"] < row.sum() / 8 * 1.03  # within 3% of an even split of the render
    oldp = gather_bound(row, old, 0, W_D, link, 7 * link)  # round 5's plan: rank 0 = bottom strip
    assert oldp["link_ms"] > 0.44 and oldp["bound_ms"] > 1.5 * pred["bound_ms"]
    assert pred["bound_ms"] == pytest.approx(_bound(row, b, root, W_D, link, 7 * link), rel=1e-12)


def test_r05last_d_n4_bound():
    from real_time_ray_tracer_amd.dist import gather_bounds

    row, _ = _r05last_profile(4)
    b, root, pred = gather_bounds(row, 4, W_D, 76.8, 3 * 76.8)
    rows = np.diff(b)
    assert rows[root] == rows.max()
    assert pred["bound_ms"] < row.sum() / 4 * 1.03


def test_slower_links_move_rows_onto_the_root():
    """The lower the link rate, the more rows the root keeps and the smaller the largest sent strip."""
    from real_time_ray_tracer_amd.dist import gather_bounds

    row, _ = _r05last_profile(8)
    prev_root_rows, prev_sent = 0, 1 << 62
    for link in (200.0, 76.8, 50.0, 30.0, 15.0):
        b, root, pred = gather_bounds(row, 8, W_D, link, 7 * link)
        rows = np.diff(b)
        sent = max(rows[i] for i in range(8) if i != root)
        assert rows[root] >= prev_root_rows and sent <= prev_sent
        assert pred["link_ms"] <= pred["bound_ms"] * (1 + 1e-9)
        prev_root_rows, prev_sent = rows[root], sent


def _brute(row, n, W, link, ingest):
    H = len(row)
    best = None
    for cuts in itertools.combinations(range(1, H), n - 1):
        b = [0, *cuts, H]
        for root in range(n):
            t = _bound(row, b, root, W, link, ingest)
            best = t if best is None else min(best, t)
    return best


@pytest.mark.parametrize("seed", range(12))
def test_planner_is_optimal_on_small_frames(seed):
    """Against exhaustive search over every contiguous split and root (H <= 13 rows, n <= 4)."""
    from real_time_ray_tracer_amd.dist import gather_bounds

    rng = np.random.default_rng(seed)
    H = int(rng.integers(4, 14))
    n = int(rng.integers(1, min(4, H) + 1))
    row = rng.gamma(0.8, 1.0, H) * (rng.random(H) > 0.15)
    W = int(rng.integers(1, 5)) * 64
    link = float(rng.uniform(0.002, 0.05))     # GB/s: per-row link time comparable with a row's cost
    ingest = float(rng.choice([0.0, link * rng.uniform(1.0, 3.0)]))
    b, root, pred = gather_bounds(row, n, W, link, ingest)
    assert b[0] == 0 and b[-1] == H and all(b[i + 1] > b[i] for i in range(n)) and 0 <= root < n
    got = _bound(row, b, root, W, link, ingest)
    assert got == pytest.approx(pred["bound_ms"], rel=1e-12, abs=1e-15)
    assert got <= _brute(row, n, W, link, ingest) * (1 + 1e-9) + 1e-15


def test_planner_rejects_bad_input():
    from real_time_ray_tracer_amd import RtError
    from real_time_ray_tracer_amd.host import plan_strips_gather, strip_gather_bound

    for args in [(np.ones(4), 5, 64, 1.0, 1.0), (np.r_[1.0, -1.0, 1.0], 2, 64, 1.0, 1.0),
                 (np.r_[1.0, np.nan], 1, 64, 1.0, 1.0), (np.ones(4), 0, 64, 1.0, 1.0), (np.ones(4), 2, 0, 1.0, 1.0),
                 (np.r_[1.0, np.inf], 1, 64, 1.0, 1.0), (np.ones(4), 2, 64, float("nan"), 1.0)]:
        with pytest.raises(RtError):
            plan_strips_gather(*args)
    with pytest.raises(RtError):
        strip_gather_bound(np.ones(4), [0, 2, 2, 4], 0, 64, 1.0, 1.0)
    with pytest.raises(RtError):
        strip_gather_bound(np.ones(4), [0, 2, 4], 2, 64, 1.0, 1.0)


def test_no_link_terms_is_a_min_max_render_split():
    """Without link terms the plan is the optimal min-max split of the render cost, root = the
    strip with the most rows."""
    from real_time_ray_tracer_amd.dist import gather_bounds

    row = np.r_[np.full(1000, 0.01), np.full(1160, 0.09)]
    b, root, pred = gather_bounds(row, 8, W_D, 0.0, 0.0)
    rows = np.diff(b)
    assert rows[root] == rows.max() and pred["link_ms"] == 0.0 and pred["ingest_ms"] == 0.0
    assert pred["render_ms"] <= row.sum() / 8 + row.max() + 1e-12


def test_strip_plan_rank_mapping():
    from real_time_ray_tracer_amd.dist import StripPlan

    p = StripPlan(8, 10, [0, 2, 5, 7, 10], root_strip=2)
    assert [p.strip_of(r) for r in range(4)] == [2, 0, 1, 3]
    assert [p.rank_of(p.strip_of(r)) for r in range(4)] == [0, 1, 2, 3]
    assert p.rows(0) == (5, 7) and p.rows(1) == (0, 2) and p.rows(3) == (7, 10)
    assert p.strip_bytes(0) == 0 and p.strip_bytes(3) == 3 * 8 * 16
    with pytest.raises(ValueError):
        StripPlan(8, 10, [0, 5, 10], root_strip=2)
