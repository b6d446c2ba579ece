"""hic3defdr_amd.numa: the cpulist parser and the no-device behaviour (the
binding itself is exercised by bench.py on the GPU box)."""
import os

from hic3defdr_amd import numa


def test_cpulist_ranges_and_singles():
    assert numa._cpulist('0-3,8,10-11\n') == {0, 1, 2, 3, 8, 10, 11}
    assert numa._cpulist('') == set()


def test_no_device_binds_nothing(monkeypatch):
    monkeypatch.setattr(numa, 'gpu_node', lambda device=0: None)
    before = os.sched_getaffinity(0)
    assert numa.bind(0) is None
    monkeypatch.setenv('H3D_NUMA_BIND', '1')
    assert numa.maybe_bind(0) is None
    assert os.sched_getaffinity(0) == before


def test_opt_in(monkeypatch):
    calls = []
    monkeypatch.setattr(numa, 'bind', lambda device=0: calls.append(device))
    monkeypatch.delenv('H3D_NUMA_BIND', raising=False)
    numa.maybe_bind(0)
    assert calls == []
    numa.maybe_bind(0, default=True)
    assert calls == [0]
    monkeypatch.setenv('H3D_NUMA_BIND', '0')
    numa.maybe_bind(0, default=True)
    assert calls == [0]
