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


def _rank_xchg(rank, world, port, out_dir):
    """Context.xchg_init's handle exchange over gloo with a stand-in libia (no GPU here): every
    rank's 64-byte handle must reach ia_xchg_open on every rank, in rank order."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import ia_amd  # noqa: F401
    from ia_amd import _native
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    seen = {}

    class FakeLib(object):
        def ia_xchg_alloc(self, h, w, buf):
            seen['alloc_world'] = w
            buf.raw = bytes([rank + 1]) * 64
            return 0

        def ia_xchg_open(self, h, r, w, handles):
            seen['open'] = (r, w, bytes(handles))
            return 0

    _native._lib = FakeLib()
    ctx = object.__new__(_native.Context)
    ctx._h = None

    def all_gather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out
    ctx.xchg_init(rank, world, all_gather)
    r, w, hs = seen['open']
    np.savez(os.path.join(out_dir, 'x%d.npz' % rank), r=r, w=w, alloc=seen['alloc_world'],
             hs=np.frombuffer(hs, dtype=np.uint8))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_xchg_handle_exchange_gloo(tmp_path, world):
    mp.spawn(_rank_xchg, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = np.concatenate([np.full(64, r + 1, dtype=np.uint8) for r in range(world)])
    for r in range(world):
        z = np.load(os.path.join(str(tmp_path), 'x%d.npz' % r))
        assert int(z['r']) == r and int(z['w']) == world and int(z['alloc']) == world
        assert np.array_equal(z['hs'], want)


def test_xchg_slot_protocol_two_parities_suffice():
    """The peer-write exchange's slot discipline (ia_internal.h XSlot / ia_xslot, k_merge_xchg)
    simulated with one thread per rank and random delays: a rank publishes its step-t winner
    into slot (t & 1, rank, m) of every rank's buffer, then waits for the W slots of step t in
    its own buffer and takes the lexicographic (d, row) minimum.  With two parities no slot is
    overwritten before its reader consumed it (a rank is never two steps ahead of a peer), every
    rank reads exactly step t's values, and all ranks agree on every winner."""
    import threading
    import time
    rs = np.random.RandomState(1)
    W, steps, M = 4, 60, 5
    vals = rs.randint(0, 7, size=(steps, W, M)).astype(np.float64) / 4   # many exact ties
    rows = rs.randint(0, 1000, size=(steps, W, M))
    bufs = [dict() for _ in range(W)]          # (parity, rank, m) -> (d, row, seq)
    consumed = [dict() for _ in range(W)]      # (parity, rank, m) -> seq its reader took
    lock = threading.Lock()
    got = np.zeros((W, steps, M, 2))
    errors = []

    def rank_main(r):
        try:
            rng = np.random.RandomState(100 + r)
            for t in range(steps):
                seq = t + 1
                time.sleep(rng.rand() * 1e-3)
                for p in range(W):               # publish into every peer (d, row, then seq)
                    for m in range(M):
                        with lock:
                            old = bufs[p].get((seq & 1, r, m))
                            if old is not None and consumed[p].get((seq & 1, r, m)) != old[2]:
                                errors.append(('overwrote an unread slot', r, p, t, old[2]))
                            bufs[p][(seq & 1, r, m)] = (vals[t, r, m], rows[t, r, m], seq)
                deadline = time.time() + 10
                for m in range(M):
                    best = (np.inf, 2 ** 62)
                    for p in range(W):           # poll own buffer
                        while True:
                            with lock:
                                x = bufs[r].get((seq & 1, p, m))
                            if x is not None and x[2] == seq:
                                with lock:
                                    consumed[r][(seq & 1, p, m)] = seq
                                break
                            if time.time() > deadline:
                                raise RuntimeError('rank %d timed out at step %d' % (r, t))
                            time.sleep(1e-5)
                        best = min(best, (x[0], x[1]))
                    got[r, t, m] = best
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(W)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:3]
    for t in range(steps):
        for m in range(M):
            want = min(zip(vals[t, :, m], rows[t, :, m]))
            for r in range(W):
                assert tuple(got[r, t, m]) == want
