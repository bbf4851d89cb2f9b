"""bench.py / profiling-tool host logic (CPU only): the CPU baseline's core count, and the
per-dispatch labelling of counter runs ('--frame-batch 16' must not read as 1)."""
import builtins
import importlib.util
import io

from conftest import ROOT

import bench


def _load_tool(name):
    spec = importlib.util.spec_from_file_location(name, ROOT / "tools" / f"{name}.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_host_cpus_uses_the_cgroup_quota(monkeypatch):
    real_open = builtins.open

    def fake_open(path, *a, **k):
        if str(path) == "/sys/fs/cgroup/cpu.max":
            return io.StringIO("1600000 100000\n")
        return real_open(path, *a, **k)

    monkeypatch.setattr(builtins, "open", fake_open)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(256)))
    c = bench.host_cpus()
    assert c["affinity_cpus"] == 256 and c["cgroup_cpu_quota"] == 16.0 and c["usable"] == 16


def test_host_cpus_without_quota(monkeypatch):
    real_open = builtins.open

    def fake_open(path, *a, **k):
        if str(path) == "/sys/fs/cgroup/cpu.max":
            return io.StringIO("max 100000\n")
        return real_open(path, *a, **k)

    monkeypatch.setattr(builtins, "open", fake_open)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(12)))
    c = bench.host_cpus()
    assert c["cgroup_cpu_quota"] is None and c["usable"] == 12


def test_counter_runs_are_labelled_per_frame_only_when_they_are():
    pmc = _load_tool("pmc_summary")
    f = pmc.frames_per_dispatch
    assert f(1, "") == 1                      # mode 1: one frame per dispatch always
    assert f(4, "") == 1                      # bench.py's default: one launch per frame
    assert f(4, "--frame-batch 1") == 1
    assert f(4, "--frame-batch=1") == 1
    assert f(4, "--frame-batch 16") is None   # not 'contains --frame-batch 1'
    assert f(2, "--steps 10 --frame-batch 8") is None
