"""The N>1 DB-shard protocol of `--mode shard` on CPU, world size 2 over gloo:
every rank takes its tile-strided shard of the DB rows (ia_shard_tiles), finds its local exact
winner per query (numpy fp64 here, the certified K3/K4 winner on the GPU), the (distance, row)
pairs are all-gathered, and ia_merge_winners picks the global winner in the same order on every
rank.  The result must equal the single-process exact NN with lowest-index ties, identically on
both ranks."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, n, d, nq, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import ia_amd  # noqa: F401
    from ia_amd import _native
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    rs = np.random.RandomState(0)
    pts = np.round(rs.rand(n, d) * 4) / 4          # coarse values: many exact ties across shards
    q = np.round(rs.rand(nq, d) * 4) / 4
    rows = _native.shard_rows(n, world, rank)
    dd = ((pts[rows][None, :, :] - q[:, None, :]) ** 2).sum(axis=2)
    k = dd.argmin(axis=1)                          # lowest local index among ties = lowest row (rows sorted)
    loc_d = dd[np.arange(nq), k]
    loc_r = rows[k].astype(np.int64)
    gd = [torch.zeros(nq, dtype=torch.float64) for _ in range(world)]
    gr = [torch.zeros(nq, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gd, torch.from_numpy(loc_d))
    dist.all_gather(gr, torch.from_numpy(loc_r))
    wd, wr = _native.merge_winners(np.stack([x.numpy() for x in gd]), np.stack([x.numpy() for x in gr]))
    np.savez(os.path.join(out_dir, 'rank%d.npz' % rank), d=wd, r=wr, rows=rows)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('n', [64 * 32 * 2 + 37, 70001])
def test_db_shard_exchange_world2_gloo(tmp_path, n):
    world, d, nq = 2, 9, 40
    mp.spawn(_rank_main, args=(world, _free_port(), n, d, nq, str(tmp_path)), nprocs=world, join=True)
    res = [np.load(os.path.join(str(tmp_path), 'rank%d.npz' % r)) for r in range(world)]
    rs = np.random.RandomState(0)
    pts = np.round(rs.rand(n, d) * 4) / 4
    q = np.round(rs.rand(nq, d) * 4) / 4
    full = ((pts[None, :, :] - q[:, None, :]) ** 2).sum(axis=2)
    assert len(res[0]['rows']) < n                   # the level really is sharded
    for z in res:
        assert np.array_equal(z['r'], full.argmin(axis=1))
        assert np.array_equal(z['d'], full.min(axis=1))
    assert np.array_equal(res[0]['r'], res[1]['r']) and np.array_equal(res[0]['d'], res[1]['d'])
