"""The N>1 path of bench.py on the CPU: world size 2 over gloo (the GPU run uses RCCL with
the same calls).  Ranks shard streams with no data-path collective; only the timing is
reduced (max over ranks)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    ranks = bench.Ranks()  # bench.py's gloo group
    ids = bench.shard_ids('2', rank, 4)
    ids4 = bench.shard_ids('4', rank, 16)
    mx = ranks.max([1.0 + rank, 10.0 - rank])
    ranks.barrier()
    q.put((rank, ids, ids4, mx))
    ranks.close()


def test_two_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, ids0, c40, m0), (r1, ids1, c41, m1) = res
    assert not set(ids0) & set(ids1)                       # disjoint shards
    assert ids0 == [0, 1, 2, 3] and ids1 == [4, 5, 6, 7]
    assert c40 == list(range(0, 128, 8)) and c41 == list(range(1, 128, 8))  # round-robin
    assert m0 == m1 == [2.0, 10.0]                         # max over ranks


@pytest.mark.parametrize('rank', [0, 3, 7])
def test_config4_round_robin(rank):
    ids = bench.shard_ids('4', rank, 16)
    assert all(i % 8 == rank for i in ids) and len(set(ids)) == 16
