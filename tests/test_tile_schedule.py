"""The tile kernel's work units (kernels.hip tile_units / TileUnits.range, through the host-only
rc_tile_schedule): every schedule -- fully static, or a static share plus dynamic units -- must
hand out each tile of the launch exactly once, in address order, in units of at most the
promised size.  CPU only (no device)."""
import ctypes

import numpy as np
import pytest

from replicat_amd import _lib


def units(n_tiles, waves, permille=100, chunk=12, dyn_min=128):
    n = ctypes.c_uint64()
    assert _lib.lib().rc_tile_schedule(n_tiles, waves, permille, chunk, dyn_min, None, 0,
                                       ctypes.byref(n)) == 0
    r = np.zeros(2 * n.value, dtype=np.uint32)
    assert _lib.lib().rc_tile_schedule(n_tiles, waves, permille, chunk, dyn_min, r.ctypes.data,
                                       n.value, ctypes.byref(n)) == 0
    return r.reshape(-1, 2).astype(np.int64)


CASES = [
    # config 2 on 256 / 224 CUs (3.87 M tiles), config 4, 3 (iii), the harness (static), tiny
    (3_874_000, 4096), (3_874_000, 3584), (8_388_000, 4096), (3_875_000, 4096),
    (312_188, 4096), (312_188, 3584), (100, 4096), (0, 4096), (600_000, 4096), (1 << 20, 64),
]


@pytest.mark.parametrize('n_tiles,waves', CASES)
@pytest.mark.parametrize('permille,chunk', [(100, 12), (250, 32), (0, 7), (0, 2), (900, 3),
                                            (1000, 12), (100, 4)])
def test_units_partition_the_tiles(n_tiles, waves, permille, chunk):
    r = units(n_tiles, waves, permille, chunk, 128)
    static, dyn = r[:waves], r[waves:]
    # static units: contiguous equal shares from tile 0; then the dynamic units in order
    assert ((0 <= r[:, 0]) & (r[:, 0] <= r[:, 1]) & (r[:, 1] <= n_tiles)).all()
    diff = np.zeros(n_tiles + 1, dtype=np.int64)
    np.add.at(diff, r[:, 0], 1)
    np.add.at(diff, r[:, 1], -1)
    assert (np.cumsum(diff)[:n_tiles] == 1).all()  # every tile in exactly one unit
    nonempty = r[r[:, 1] > r[:, 0]]
    assert (nonempty[1:, 0] == nonempty[:-1, 1]).all(), 'units out of address order'
    if len(dyn):
        sizes = dyn[:, 1] - dyn[:, 0]
        assert sizes.max() <= max(chunk, 2)
        # ~4 dynamic units per wave at least (a unit is the granularity of the launch's tail)
        assert len(dyn) >= min(4 * waves, (n_tiles - static[:, 1].max()) // max(chunk, 2))


def test_static_below_the_dynamic_minimum():
    """Fewer than 128 tiles per wave (the harness: 76): one static unit per wave."""
    r = units(312_188, 4096)
    assert len(r) == 4096 and (r[:, 1] - r[:, 0]).max() == 77
