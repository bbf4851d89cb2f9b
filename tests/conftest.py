import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU test")
    # the checker: on the GPU box's AMD EPYC (AVX-512) the oracle's Zen build, the same C source
    # with 16-wide sphere scans (bit-identical to the portable AVX2 build; tests/test_oracle_cpu.py)
    import oracle
    oracle.select_native()


def pytest_terminal_summary(terminalreporter):
    """Durations of the long parity tests (whole frames, full strips), always printed."""
    rows = []
    for rep in terminalreporter.stats.get("passed", []) + terminalreporter.stats.get("failed", []):
        if getattr(rep, "when", "") == "call" and rep.duration >= 5.0:
            rows.append((rep.duration, rep.nodeid, rep.outcome))
    if rows:
        terminalreporter.write_line(f"tests over 5 s ({len(rows)}):")
        for dur, nid, out in sorted(rows, reverse=True):
            terminalreporter.write_line(f"  {dur:7.1f} s  {out:6s} {nid}")


def close(g, c, rel=1e-4, abs_=1e-6):
    """North-star tolerance per channel: |g-c| <= rel*max(|g|,|c|) + abs; NaN == NaN."""
    g = np.asarray(g, np.float32)
    c = np.asarray(c, np.float32)
    both_nan = np.isnan(g) & np.isnan(c)
    with np.errstate(invalid="ignore"):
        ok = np.abs(g - c) <= rel * np.maximum(np.abs(g), np.abs(c)) + abs_
    return ok | both_nan


def assert_close(g, c, what="", rel=1e-4, abs_=1e-6):
    ok = close(g, c, rel, abs_)
    if not ok.all():
        bad = np.argwhere(~ok)
        i = tuple(bad[0])
        raise AssertionError(f"{what}: {(~ok).sum()} of {ok.size} values out of tolerance; first at {i}: "
                             f"gpu={np.asarray(g)[i]!r} cpu={np.asarray(c)[i]!r}")


def assert_bitwise(g, c, what=""):
    g = np.asarray(g, np.float32)
    c = np.asarray(c, np.float32)
    same = (g.view(np.uint32) == c.view(np.uint32)) | (np.isnan(g) & np.isnan(c))
    if not same.all():
        bad = np.argwhere(~same)
        i = tuple(bad[0])
        raise AssertionError(f"{what}: {(~same).sum()} of {same.size} values differ bitwise; first at {i}: "
                             f"{g[i]!r} vs {c[i]!r}")


@pytest.fixture(scope="session")
def gpu_available():
    import torch  # device count does not initialise HIP on this image
    return torch.cuda.device_count() > 0
