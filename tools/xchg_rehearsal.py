"""Two-process rehearsal of the peer-write winner exchange (include/ia.h ia_xchg_*) on ONE GPU:
both ranks open each other's exchange buffer through real HIP IPC handles and run a sharded
synthesis whose every wavefront step publishes / polls across the process boundary.  Each rank
checks its B', s, im replica against the golden reference run (g256, every level pruned) and
against an unsharded run of a 1024^2 job (cfg3, pruned 1024^2 level) made by its own second
context.  Launch (from the repo root, gloo carries only the 64-byte handles):
  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/xchg_rehearsal.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def run(ctx, z, prune_all):
    from ia_amd import _native
    L, k = z['L'], float(z['k'])
    Bp = [x.copy() for x in z['Bp_init']]
    st = _native.Stats()
    out = {}
    ctx.set_option('prune_min_rows', 1 if prune_all else 524288)
    for level in range(1, L):
        out[level] = ctx.synthesize_level(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                          [p[level - 1] for p in z['Ap_pyr']], z['B_pyr'][level], z['B_pyr'][level - 1],
                                          Bp[level - 1], Bp[level], z['weights'], 1 + 2.0 ** (level - L) * k, st)
    return out, Bp, st


def main():
    import torch
    import torch.distributed as dist
    import ia_amd  # noqa: F401
    from ia_amd import _native, synth
    from golden_util import load_e2e
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    # both ranks share ONE GPU here: each context's stream gets its own CU slice, so a kernel
    # waiting for the peer's exchange never holds the CUs the peer's kernels need
    os.environ['IA_CU_SPLIT'] = '%d/%d' % (rank, world)
    dist.init_process_group('gloo')
    ctx = _native.Context(0)

    def all_gather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out
    ctx.xchg_init(rank, world, all_gather)
    ok = True
    z = load_e2e('g256')
    dist.barrier()
    t0 = time.time()
    out, Bp, st = run(ctx, z, True)
    t1 = time.time()
    for level, (s, im) in out.items():
        same = (np.array_equal(s, z['s'][level]) and np.array_equal(im, z['im'][level]) and
                np.array_equal(Bp[level], z['Bp_final'][level]))
        ok &= same
    print('[rank %d] g256 pruned, %d-way peer-write shards: %s vs the reference run (%.2f s, bound_violations %d)'
          % (rank, world, 'bit-identical' if ok else 'DIFFERENT', t1 - t0, st.bound_violations), flush=True)
    job = synth.make_job(1024)
    zj = {'L': job.L, 'k': job.k, 'A_pyr': job.A_pyr, 'Ap_pyr': job.Ap_pyr_list, 'B_pyr': job.B_pyr,
          'Bp_init': job.Bp_init, 'weights': job.weights}
    dist.barrier()
    t0 = time.time()
    out, Bp, st = run(ctx, zj, False)
    t1 = time.time()
    plain = _native.Context(0)   # unsharded reference on this rank
    ref, Bp_ref, _ = run(plain, zj, False)
    same = all(np.array_equal(out[l][0], ref[l][0]) and np.array_equal(out[l][1], ref[l][1]) and
               np.array_equal(Bp[l], Bp_ref[l]) for l in range(1, job.L))
    ok &= same
    print('[rank %d] cfg3 1024^2, %d-way peer-write shards (pruned 1024^2 level): %s vs unsharded (%.2f s sharded, '
          'pruned levels %d, bound_violations %d)' % (rank, world, 'bit-identical' if same else 'DIFFERENT', t1 - t0,
                                                      st.pruned_levels, st.bound_violations), flush=True)
    # bench.py's N > 1 shard mode: `world` jobs sharing A stepped together over the sharded DB
    jobs = synth.make_jobs(world, size=1024)

    def run_batch(c):
        Bps = [[x.copy() for x in j.Bp_init] for j in jobs]
        st = _native.Stats()
        c.set_option('prune_min_rows', 524288)
        res = []
        for level in range(1, jobs[0].L):
            specs = [dict(B=j.B_pyr[level], Bc=j.B_pyr[level - 1], Bpc=Bps[n][level - 1], Bp=Bps[n][level],
                          weights=j.weights, kappa_factor=j.kappa_factor(level)) for n, j in enumerate(jobs)]
            res.append(c.synthesize_levels(jobs[0].A_pyr[level], jobs[0].A_pyr[level - 1],
                                           [p[level] for p in jobs[0].Ap_pyr_list],
                                           [p[level - 1] for p in jobs[0].Ap_pyr_list], specs, st))
        return res, Bps, st
    dist.barrier()
    t0 = time.time()
    rb, Bpb, st = run_batch(ctx)
    t1 = time.time()
    ru, Bpu, _ = run_batch(plain)
    same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for la, lb in zip(rb, ru) for a, b in zip(la, lb))
    same &= all(np.array_equal(Bpb[n][l], Bpu[n][l]) for n in range(world) for l in range(1, jobs[0].L))
    ok &= same
    print('[rank %d] %d cfg3 jobs batched over %d-way peer-write shards: %s vs unsharded batched (%.2f s sharded, '
          'bound_violations %d)' % (rank, world, world, 'bit-identical' if same else 'DIFFERENT', t1 - t0,
                                    st.bound_violations), flush=True)
    # owner computes (exchange = 2, bench.py's N > 1 shard mode): rank r brings job r alone,
    # every rank scans its shard for both jobs' queries; job r == its unsharded run
    octx = _native.Context(0)
    octx.set_option('exchange', 2)
    octx.xchg_init(rank, world, all_gather)
    mine = jobs[rank]

    def run_one(c):
        Bp1 = [x.copy() for x in mine.Bp_init]
        st = _native.Stats()
        res = []
        for level in range(1, mine.L):
            res.append(c.synthesize_level(mine.A_pyr[level], mine.A_pyr[level - 1], [p[level] for p in mine.Ap_pyr_list],
                                          [p[level - 1] for p in mine.Ap_pyr_list], mine.B_pyr[level],
                                          mine.B_pyr[level - 1], Bp1[level - 1], Bp1[level], mine.weights,
                                          mine.kappa_factor(level), st))
        return res, Bp1, st
    dist.barrier()
    t0 = time.time()
    ro, Bpo, st = run_one(octx)
    t1 = time.time()
    rp, Bpp, _ = run_one(plain)
    same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(ro, rp))
    same &= all(np.array_equal(Bpo[l], Bpp[l]) for l in range(1, mine.L))
    ok &= same
    print('[rank %d] owner-computes: job %d over %d-way shards: %s vs its unsharded run (%.2f s, pruned levels %d, '
          'bound_violations %d)' % (rank, rank, world, 'bit-identical' if same else 'DIFFERENT', t1 - t0,
                                    st.pruned_levels, st.bound_violations), flush=True)
    octx.close()
    plain.close()
    ctx.close()
    flag = torch.tensor([0 if ok else 1])
    dist.all_reduce(flag)
    dist.destroy_process_group()
    if rank == 0:
        print('XCHG-REHEARSAL %s' % ('OK' if int(flag) == 0 else 'FAILED'), flush=True)
    sys.exit(0 if int(flag) == 0 else 1)


if __name__ == '__main__':
    main()
