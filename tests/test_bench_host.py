"""bench.py's host-core accounting (verdict r03 item 2): the CPU baseline runs on every usable core, where
usable = the affinity mask capped by the cgroup CPU quota (the GPU box: 256 CPUs in the mask, 16 granted)."""
import builtins
import io
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _fake_open(files):
    real = builtins.open

    def op(path, *a, **k):
        if path in files:
            if files[path] is None:
                raise FileNotFoundError(path)
            return io.StringIO(files[path])
        return real(path, *a, **k)
    return op


def test_quota_caps_affinity(monkeypatch):
    monkeypatch.setattr(builtins, "open", _fake_open({"/sys/fs/cgroup/cpu.max": "1600000 100000\n"}))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    threads, usable, _, how = bench.host_cores()
    assert threads == usable == 16
    assert how == {"affinity": 256, "cgroup_cpu_quota": 16.0}


def test_unlimited_quota_uses_affinity(monkeypatch):
    monkeypatch.setattr(builtins, "open", _fake_open({"/sys/fs/cgroup/cpu.max": "max 100000\n"}))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(12)))
    assert bench.host_cores()[:2] == (12, 12)


def test_fractional_quota_rounds_up_and_v1_fallback(monkeypatch):
    monkeypatch.setattr(builtins, "open", _fake_open({"/sys/fs/cgroup/cpu.max": None,
                                                      "/sys/fs/cgroup/cpu/cpu.cfs_quota_us": "250000\n",
                                                      "/sys/fs/cgroup/cpu/cpu.cfs_period_us": "100000\n"}))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(64)))
    assert bench.host_cores()[:2] == (3, 3)
