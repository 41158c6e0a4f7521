"""CPU tests of bench.py's measurement bookkeeping (SURVEY.md §8 d): the roofline's two bases,
its nulls, and the PMC traffic that may only come from a summary of the same library build."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

GB = 1e9


def test_roofline_two_bases():
    L, read = 68_719_476_736, 63_476_596_736
    r = bench.roofline(L, read, 10.0, 0.02, 0.15, 64.5 * GB, 'x', 'id')
    assert r['achieved'] == pytest.approx(L / 10e-3 / GB, abs=0.1)
    assert r['frac'] == pytest.approx(L / 10e-3 / GB / bench.HBM_PEAK_GBS, abs=1e-4)
    assert r['frac_read'] == pytest.approx(read / 10e-3 / GB / bench.HBM_PEAK_GBS, abs=1e-4)
    assert r['frac_read'] < r['frac'] <= 1.0
    assert r['traffic'] == round(64.5 * GB) and r['bound'] == 'hbm'


def test_roofline_null_when_nothing_is_read():
    """config 3 (i): every stream cut by the tail rule alone -- no roofline, not a 1000x frac."""
    r = bench.roofline(68_719_476_736, 0, 0.005, 0.005, 0.12, None, 'x', 'id')
    assert r['achieved'] is None and r['frac'] is None and r['frac_read'] is None
    assert 'tail rule' in r['note']


def test_roofline_null_above_peak():
    r = bench.roofline(10 * GB, 10 * GB, 1.0, 0.0, 0.0, None, 'x', 'id')  # 10 TB/s
    assert r['frac'] is None and r['note'] == 'not a measurement'


def test_pmc_traffic_same_build_only(tmp_path, monkeypatch):
    d = tmp_path / 'profiles' / 'r09'
    d.mkdir(parents=True)
    (d / 'pmc_summary.json').write_text(json.dumps({
        'workload': 'config2', 'build_id': 'aaaa',
        'rc_tile_kernel': {'hbm_read_bytes_corrected': 64e9, 'hbm_write_bytes': 1e8}}))
    monkeypatch.setattr(bench, 'ROOT', str(tmp_path))
    got, src = bench.pmc_traffic('config2', 'aaaa')
    assert got == pytest.approx(64.1e9) and 'pmc_summary.json' in src
    got, why = bench.pmc_traffic('config2', 'bbbb')
    assert got is None and 'aaaa' in why and 'bbbb' in why
    assert bench.pmc_traffic('config4', 'aaaa')[0] is None
    assert bench.pmc_traffic(None, 'aaaa')[0] is None


def test_pmc_traffic_per_workload(tmp_path, monkeypatch):
    """Round 5: one summary holds every workload; the newest round with the line's build wins."""
    old = tmp_path / 'profiles' / 'r04'
    new = tmp_path / 'profiles' / 'r05'
    old.mkdir(parents=True)
    new.mkdir(parents=True)
    (old / 'pmc_summary.json').write_text(json.dumps({
        'workload': 'config2', 'build_id': 'aaaa',
        'rc_tile_kernel': {'hbm_read_bytes_corrected': 64e9}}))
    (new / 'pmc_summary.json').write_text(json.dumps({'build_id': 'cccc', 'workloads': {
        'harness': {'rc_tile_kernel': {'hbm_read_bytes_corrected': 5.2e9, 'hbm_write_bytes': 1e6}},
        'config2': {'rc_tile_kernel': {'hbm_read_bytes_corrected': 65e9}}}}))
    monkeypatch.setattr(bench, 'ROOT', str(tmp_path))
    got, src = bench.pmc_traffic('harness', 'cccc')
    assert got == pytest.approx(5.201e9) and src.endswith('[harness]') and 'r05' in src
    assert bench.pmc_traffic('config2', 'cccc')[0] == pytest.approx(65e9)
    assert bench.pmc_traffic('config2', 'aaaa')[0] == pytest.approx(64e9)  # the older build's
    got, why = bench.pmc_traffic('harness', 'aaaa')
    assert got is None and 'cccc' in why


def test_workload_keys():
    a = bench.parse(['--config', '2'])
    assert bench.workload_key(a, 1024, 64 << 20, False, None) == 'config2'
    a = bench.parse(['--config', '2', '--key', 'seeded'])
    assert bench.workload_key(a, 1024, 64 << 20, False, None) == 'config2_seeded'
    a = bench.parse(['--config', '2', '--streams', '8'])
    assert bench.workload_key(a, 8, 64 << 20, False, None) is None
    a = bench.parse(['--config', 'harness'])
    assert bench.workload_key(a, 1, 5_120_000_000, False, None) == 'harness'
    a = bench.parse(['--config', '3i'])
    assert bench.workload_key(a, 65536, 1 << 20, False, None) is None
    a = bench.parse(['--config', '3iii', '--min-length', '4'])
    assert bench.workload_key(a, 65536, 1 << 20, True, None) is None


def test_cpu_share_caps_at_the_box_share(monkeypatch):
    monkeypatch.setattr(os, 'sched_getaffinity', lambda pid: set(range(256)))
    monkeypatch.setenv('OMP_NUM_THREADS', '16')
    assert bench.cpu_share() == (16, 256)
    monkeypatch.delenv('OMP_NUM_THREADS')
    assert bench.cpu_share() == (256, 256)


def test_default_warmup_per_config():
    """2 warm-up steps by default (the driver's contract), 50 for the sub-millisecond
    configurations (the harness, 3 i: the GPU clock still ramps after the host-side setup);
    an explicit --warmup is always honoured."""
    import bench
    assert bench.parse([]).warmup == 2
    assert bench.parse(['--config', '3iii']).warmup == 2
    assert bench.parse(['--config', 'harness']).warmup == bench.WARMUP_SHORT == 50
    assert bench.parse(['--config', '3i']).warmup == 50
    assert bench.parse(['--config', 'harness', '--warmup', '3']).warmup == 3
    assert bench.parse(['--warmup', '0']).warmup == 0
