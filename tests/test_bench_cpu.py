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


def test_load_traffic_finds_both_pmc_namings(tmp_path):
    """load_traffic reads profiles/*_pmc_<cfg>.json (tools/round_profile.sh's
    naming since round 5, as load_sq reads *_sq_<cfg>.json) as well as the older *_pmc.json, and
    prefers the file taken on this library build."""
    import json

    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r04p_d_pmc.json").write_text(json.dumps({"config": "d", "src_sha1": "old", "1": 1}))
    (prof / "r05last_pmc_d.json").write_text(json.dumps({"config": "d", "src_sha1": "new", "1": 2}))
    (prof / "r05last_pmc_c.json").write_text(json.dumps({"config": "c", "src_sha1": "new", "1": 3}))
    (prof / "r06x_pmc_d.json").write_text(json.dumps({"src_sha1": "other", "1": 4}))  # no "config": by name
    assert bench.load_traffic("d", "new", root=tmp_path) == ({"config": "d", "src_sha1": "new", "1": 2},
                                                             "r05last_pmc_d.json")
    assert bench.load_traffic("d", "old", root=tmp_path)[1] == "r04p_d_pmc.json"
    assert bench.load_traffic("d", "other", root=tmp_path)[1] == "r06x_pmc_d.json"
    assert bench.load_traffic("d", "none", root=tmp_path)[1] == "r06x_pmc_d.json"  # newest by name
    assert bench.load_traffic("c", "new", root=tmp_path)[0]["1"] == 3
    assert bench.load_traffic("e", "new", root=tmp_path) == (None, None)
    # the committed round-5 file on its own build (the bench line's traffic, 408 MB per AO launch)
    data, name = bench.load_traffic("d", "38d1c896a956")
    assert name == "r05last_pmc_d.json" and data["1"] == 408074496


def test_launch_ranks_returns_none_when_not_launching(monkeypatch):
    """no launch is None (a killed launcher's negative status is not 'not launched')."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.launch_ranks(["--gpus", "1"]) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.launch_ranks(["--gpus", "2"]) is None
