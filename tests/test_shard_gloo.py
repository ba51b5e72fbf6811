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


def _rank_pruned(rank, world, port, n_rows, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import ia_amd  # noqa: F401
    from ia_amd import _native
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    nt = (n_rows + 31) // 32
    t0, t1 = _native.shard_tiles_pruned(n_rows, world, rank)
    mine = torch.tensor([_native.shard_morton_tile(t, nt, world) for t in range(t0, t1)], dtype=torch.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([len(mine)]))
    mx = int(max(x.item() for x in sizes))
    buf = [torch.full((mx,), -1, dtype=torch.int64) for _ in range(world)]
    pad = torch.full((mx,), -1, dtype=torch.int64)
    pad[:len(mine)] = mine
    dist.all_gather(buf, pad)
    np.savez(os.path.join(out_dir, 'p%d.npz' % rank), t0=t0, t1=t1,
             tiles=np.concatenate([b.numpy()[:int(s.item())] for b, s in zip(buf, sizes)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,n_rows', [(2, 64 * 32 * 2 + 5), (2, 1048576), (4, 262144 + 96)])
def test_pruned_shard_layout_gloo(tmp_path, world, n_rows):
    """Pruned levels: shard r = Morton tiles r, r + W, ... stored contiguously.
    Over the ranks, the storage ranges tile [0, NT) in order, every Morton tile is owned exactly
    once, by rank m mod W, and shard sizes differ by at most one tile (balanced pruned work)."""
    mp.spawn(_rank_pruned, args=(world, _free_port(), n_rows, str(tmp_path)), nprocs=world, join=True)
    nt = (n_rows + 31) // 32
    res = [np.load(os.path.join(str(tmp_path), 'p%d.npz' % r)) for r in range(world)]
    assert res[0]['t0'] == 0 and res[-1]['t1'] == nt
    for r in range(world - 1):
        assert res[r]['t1'] == res[r + 1]['t0']
    sizes = [int(z['t1'] - z['t0']) for z in res]
    assert max(sizes) - min(sizes) <= 1
    for z in res:   # every rank gathered the same full map
        assert np.array_equal(np.sort(z['tiles']), np.arange(nt))
    owner = {}
    for r, z in enumerate(res):
        for t in range(int(z['t0']), int(z['t1'])):
            owner[t] = r
    full = res[0]['tiles']
    for ts, m in enumerate(full):
        assert m % world == owner[ts]


def test_merge_winners_skips_empty_shards():
    """a pruned shard that contracted nothing for a query reports no winner (DBL_MAX, INT64_MAX);
    the merge must pick the other shards' winner"""
    import ia_amd  # noqa: F401
    from ia_amd import _native
    big = np.finfo(np.float64).max
    d = np.array([[big, 0.5, 0.25], [0.75, big, 0.25]])
    r = np.array([[2 ** 63 - 1, 7, 9], [3, 2 ** 63 - 1, 4]], dtype=np.int64)
    wd, wr = _native.merge_winners(d, r)
    assert list(wd) == [0.75, 0.5, 0.25] and list(wr) == [3, 7, 4]
