#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: B' pixels synthesised per second, exact NN, synthetic
1024x1024 A/A'/B (cfg3, full 10-level pyramid), on the MI355X HIP path.

One "step" = one complete synthesis of B' (every level 1..L-1: DB build, skewed-wavefront
exact-NN + coherence + kappa synthesis) for the synthetic job, with every input already
resident in HBM (pyramids uploaded once, before timing; B' is re-initialised on the device at
the start of each step).  `value` = B' pixels of all ranks / wall time of K timed steps.

  python bench.py [--gpus N --steps K --warmup W]           # N=1 default
  torchrun --nproc-per-node N bench.py --gpus N ...         # one process per GPU

Multi-GPU (N > 1): --mode shard (the default for cfg2/cfg3/cfg4: BASELINE config 3 as named)
splits each pruned level's A database across the N ranks and steps N jobs sharing that A
(synth.make_jobs: job 0 is the cfg job, the others other B images) through it together: every
rank scans its 1/N of the DB for the queries of all N jobs each wavefront step.
  --exchange owner (default): rank r owns job r (its gather, query sort and merge); its sorted
      queries go to every rank and every rank's scan records come back to it, both as one-shot
      xGMI peer writes (include/ia.h exchange = 2); no per-query work is replicated;
  --exchange peer / rccl: every rank holds every job's replica and runs every job's gather and
      per-shard merge; the per-shard winners are exchanged by peer writes fused into the merge
      (peer) or ncclAllGather + a finish kernel (rccl).
Per-GPU scan work stays one job's ("weak"); --shard-jobs 1 with peer / rccl gives the one-job
latency form ("strong").  The replicas aggregate (one independent job per GPU, no collective)
rides along as value_replicas; --mode replicas makes that the value.
cfg5 splits its 64-job sweep job j -> rank j mod N (no collective).

Besides the contract fields the JSON line carries:
  roofline     the dominant kernel (the certified pruned scan k3h_prune3: HBM roofline, algorithmic
               bytes / device time sampled live with HIP events every --time-stride-th wavefront
               step; traffic = PMC bytes per launch of the same config from profiles/), plus
               roofline.gathers: K1 / K1b DB builds and the K2 query gather against HBM peak.
  cpu_baseline the oracle's restatement of the reference loop (per-pixel pad + exact fp64 NN,
               1 thread per pixel) timed on S = 256 consecutive mid-level pixels of the three
               finest levels in spawned workers before the GPU is touched, extrapolated to the
               whole job (rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "B' pixels synthesized/sec, exact NN, 1024² A/A'/B, 1/2/4/8 GPUs; % MFMA peak"
FP32_MFMA_PEAK = 157.3e12   # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
F16_MFMA_PEAK = 2.5e15      # MI355X_MICROARCH.md: BF16/F16 ~2.5 PF dense (same cycles for f16)
HBM_PEAK = 8.0e12           # MI355X_MICROARCH.md: HBM3E ~8 TB/s


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class DeviceJob(object):
    """The job's pyramids as torch device tensors + per-level output buffers."""

    def __init__(self, job, torch, dev, a_from=None):
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(dev)
        self.job = job
        # jobs of one batch share the A side: the same device arrays (ia_synthesize_levels checks it)
        self.A = a_from.A if a_from is not None else [t(x) for x in job.A_pyr]
        self.Ap = a_from.Ap if a_from is not None else [t(np.stack([p[l] for p in job.Ap_pyr_list])) for l in range(job.L)]
        self.B = [t(x) for x in job.B_pyr[:job.L]]
        self.Bp0 = [t(x) for x in job.Bp_init[:job.L]]
        self.Bp = [x.clone() for x in self.Bp0]
        self.W = t(job.weights)
        self.S = [torch.empty((int(np.prod(x.shape[:2])), 2), dtype=torch.int32, device=dev) for x in self.B]
        self.IM = [torch.empty(int(np.prod(x.shape[:2])), dtype=torch.int32, device=dev) for x in self.B]
        self.ch = 1 if job.A_pyr[0].ndim == 2 else job.A_pyr[0].shape[2]

    def _level(self, ctx, l, stats):
        ptrs = dict(A=self.A[l].data_ptr(), Ac=self.A[l - 1].data_ptr(), Ap=self.Ap[l].data_ptr(),
                    Apc=self.Ap[l - 1].data_ptr(), B=self.B[l].data_ptr(), Bc=self.B[l - 1].data_ptr(),
                    Bpc=self.Bp[l - 1].data_ptr(), Bp=self.Bp[l].data_ptr(), weights=self.W.data_ptr(),
                    s_out=self.S[l].data_ptr(), im_out=self.IM[l].data_ptr())
        ctx.synthesize_level_device(self.ch, len(self.job.Ap_pyr_list), self.A[l].shape[:2], self.B[l].shape[:2],
                                    ptrs, self.job.kappa_factor(l), stats)

    def outputs(self):
        """the job's results: B', s and im of every synthesised level (device tensors)"""
        return [x for l in range(1, self.job.L) for x in (self.Bp[l], self.S[l], self.IM[l])]

    def run(self, ctx, torch, stats, pipe=None):
        """pipe = more contexts (one or a list): levels rotate over ctx + them, each level's steps
        waiting only for the steps of the previous level they read (include/ia.h
        ia_pipeline_depend; one host thread per context)"""
        for l in range(self.job.L):
            self.Bp[l].copy_(self.Bp0[l])
        torch.cuda.synchronize()   # libia runs on its own stream
        if pipe is None:
            for l in range(1, self.job.L):
                self._level(ctx, l, stats)
            return
        from ia_amd.pipeline import run_levels_pipelined
        run_levels_pipelined(lambda c, l, st: self._level(c, l, st), [ctx] + (pipe if isinstance(pipe, list) else [pipe]),
                             self.job.L, stats)


class DeviceBatch(object):
    """J jobs sharing the A side (synth.make_jobs) stepped together: one ia_synthesize_levels
    call per level, i.e. one DB and one distance scan per wavefront step for all J jobs.  The
    N > 1 shard mode runs J = N such jobs with the DB sharded N ways: every rank scans 1/N of the
    DB for the queries of all N jobs (the scan work of one job per GPU) and holds every job's
    B-side replica."""

    def __init__(self, jobs, torch, dev):
        self.dj = [DeviceJob(jobs[0], torch, dev)]
        self.dj += [DeviceJob(j, torch, dev, a_from=self.dj[0]) for j in jobs[1:]]
        self.ch = self.dj[0].ch

    def outputs(self):
        return [x for d in self.dj for x in d.outputs()]

    def run(self, ctx, torch, stats):
        for d in self.dj:
            for l in range(d.job.L):
                d.Bp[l].copy_(d.Bp0[l])
        torch.cuda.synchronize()
        d0 = self.dj[0]
        for l in range(1, d0.job.L):
            ptrs = [dict(A=d0.A[l].data_ptr(), Ac=d0.A[l - 1].data_ptr(), Ap=d0.Ap[l].data_ptr(),
                         Apc=d0.Ap[l - 1].data_ptr(), B=d.B[l].data_ptr(), Bc=d.B[l - 1].data_ptr(),
                         Bpc=d.Bp[l - 1].data_ptr(), Bp=d.Bp[l].data_ptr(), weights=d.W.data_ptr(),
                         s_out=d.S[l].data_ptr(), im_out=d.IM[l].data_ptr()) for d in self.dj]
            ctx.synthesize_levels_device(self.ch, len(d0.job.Ap_pyr_list), d0.A[l].shape[:2], d0.B[l].shape[:2], ptrs,
                                         [d.job.kappa_factor(l) for d in self.dj], stats)


class HostCopy(object):
    """Pinned host buffers for a set of device result tensors: fetch() is the D2H copy that ends a
    timed step back on the host (B', s, im of every level, as image_analogies_main returns them);
    digest() hashes the fetched bytes (bit-exact parity checks between runs and ranks)."""

    def __init__(self, tensors, torch):
        self.torch = torch
        self.dev = list(tensors)
        self.host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in self.dev]

    def fetch(self):
        for d, h in zip(self.dev, self.host):
            h.copy_(d, non_blocking=True)

    @property
    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self.dev)

    def digest(self):
        return self.digest_groups([len(self.host)])[0]

    def digest_groups(self, sizes):
        """one sha1 per group of consecutive buffers (cfg5: one per job)"""
        import hashlib
        self.torch.cuda.synchronize()
        out, i = [], 0
        for n in sizes:
            hs = hashlib.sha1()
            for h in self.host[i:i + n]:
                hs.update(h.numpy().tobytes())
            out.append(hs.hexdigest())
            i += n
        return out


EXCHANGE = {'rccl': 0, 'peer': 1, 'owner': 2}   # include/ia.h option "exchange"

LSH_NOTE = ('n/a: the reference snapshot has no LSH path (algorithms.py:69 hard-codes the kdtree index) and '
            'pyflann / libflann are absent offline; the kd-tree path itself is approximate and unrunnable here, '
            'so the baseline is the reference loop with its exact brute-force NN')


def host_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cpu_task(a):
    """CPU-baseline worker (a spawned process): seconds per pixel of n consecutive raster pixels
    of `level` from raster pixel `start` (oracle restatement of the reference loop)."""
    A_pyr, Ap_pyr_list, B_pyr, Bp_init, level, L, k, weights, n, start = a
    from oracle import ia_oracle as O
    return O.time_sample(A_pyr, Ap_pyr_list, B_pyr, Bp_init, level, L, k, weights, n, start=start)


def cpu_per_pixel(job, seconds, S=256, procs=4):
    """Reference loop (oracle restatement: per-pixel np.pad + exact fp64 numpy NN, one thread)
    timed on S consecutive mid-level raster pixels of each of the three finest levels
    (BASELINE.md §4).  The per-pixel work - a full-DB scan, a full-level pad and the 12 causal
    coherence candidates - does not depend on the pixel values, so the sample runs on the job's
    initial state and extrapolates to N_B pixels; coarser levels are priced by scaling the
    smallest sampled level's per-pixel cost with the DB size.  The S pixels are split into
    `procs` consecutive runs timed in spawned single-threaded worker processes, started before
    this process touches the GPU (4 concurrent workers: little memory contention; 8 workers on
    8 busy cores measured +17 % per pixel).  S shrinks if a level's estimate exceeds its share of
    `seconds`.  Returns ({level: s/px}, [sample descriptions])."""
    import multiprocessing as mp
    L = job.L
    lv = [l for l in range(L - 1, 0, -1)][:3]
    budget = seconds / len(lv)
    per_px, sample = {}, []
    base = (job.A_pyr, job.Ap_pyr_list, job.B_pyr, job.Bp_init)
    with mp.get_context('spawn').Pool(procs) as pool:
        for l in lv:
            h, w = job.B_pyr[l].shape[:2]
            n_b = h * w
            mid = n_b // 2 + w // 2                      # an interior pixel half way down the level
            t2 = pool.apply(_cpu_task, (base + (l, L, job.k, job.weights, 2, mid),))
            n = int(max(procs, min(S, n_b - mid, budget * procs / max(t2, 1e-9))))
            cuts = [mid + n * i // procs for i in range(procs + 1)]
            res = pool.map(_cpu_task, [base + (l, L, job.k, job.weights, cuts[i + 1] - cuts[i], cuts[i])
                                       for i in range(procs)])
            per_px[l] = sum(r * (cuts[i + 1] - cuts[i]) for i, r in enumerate(res)) / n
            sample.append('%d consecutive px from raster pixel %d of level %d (%dx%d B, %dx%d A; %.4f s/px)'
                          % (n, mid, l, h, w, job.A_pyr[l].shape[0], job.A_pyr[l].shape[1], per_px[l]))
    lmin = min(lv)
    na_min = np.prod(job.A_pyr[lmin].shape[:2])
    for l in range(1, L):
        if l not in per_px:
            per_px[l] = per_px[lmin] * np.prod(job.A_pyr[l].shape[:2]) / na_min
    return per_px, sample


def _baseline(value, sample, procs, total):
    return {'value': value, 'unit': "B' px/s", 'cores': 1, 'host_cores': host_cores(), 'sample_procs': procs,
            'kind': 'port', 'extrapolated': True, 'lsh': LSH_NOTE,
            'sample': ('oracle/ia_oracle.py reference-loop restatement (per-pixel pad, exact fp64 NN, one core per '
                       'pixel as the reference runs), timed on ' + sample + '; coarser levels scaled by DB size; '
                       'extrapolated whole-job time %.0f s on one core' % total)}


def cpu_baseline(job, seconds, procs=4):
    per_px, sample = cpu_per_pixel(job, seconds, procs=procs)
    total = sum(np.prod(job.B_pyr[l].shape[:2]) * per_px[l] for l in range(1, job.L))
    return _baseline(job.pixels / total, ', '.join(sample), procs, total)


def cpu_baseline_sweep(sw, seconds, procs=4):
    """cfg5: per-pixel costs of each resolution from the deepest job, summed over every job's
    levels (the reference runs the jobs one after the other, multi_script.py:19-32)."""
    from ia_amd import synth
    deep = int(np.argmax(sw.L))
    off = sw.offset(deep)
    job = synth.Job(sw.A_pyr[off:], [p[off:] for p in sw.Ap_pyr_list], sw.B_pyr[off:], sw.Bp_init[deep],
                    sw.jobs[deep].k, sw.weights)
    per_px, sample = cpu_per_pixel(job, seconds, procs=procs)
    total = 0.
    for j in range(len(sw.jobs)):
        for l in range(1, sw.L[j]):
            f = sw.offset(j) + l
            total += np.prod(sw.B_pyr[f].shape[:2]) * per_px[f - off]
    return _baseline(sw.pixels() / total, ', '.join(sample) + ' of the deepest job; every job of the sweep priced '
                     'per level', procs, total)


ALL_CTX = []   # every libia context this process made (timed steps switch option "stamps" on all)


def make_context(args, local):
    """One libia context with every option of the command line (each context of a multi-stream
    cfg5 run gets the same settings)."""
    from ia_amd import _native
    cx = _native.Context(local)
    ALL_CTX.append(cx)
    cx.set_option('matcher', _native.IA_MATCH_F16X3 if args.matcher == 'f16x3' else _native.IA_MATCH_F32)
    cx.set_option('prune', args.prune)
    # always explicit (the library default is 24, so a skipped set_option for 22 ran v24)
    cx.set_option('k3p_variant', args.k3p_variant)     # 20, 21, 22, 24, 25
    cx.set_option('prune_min_rows', args.prune_min_rows)
    if args.scan_wgs:   # (every context; pipelined runs then size the coarser levels' with --coarse-scan-wgs)
        cx.set_option('scan_wgs', args.scan_wgs)
    if args.k3p_blocks != 1:
        cx.set_option('k3p_blocks', args.k3p_blocks)
    if args.prune_group != 1:
        cx.set_option('prune_group', args.prune_group)
    if args.fuse_gather != 1:
        cx.set_option('fuse_gather', args.fuse_gather)
    if args.fuse_unpruned:
        cx.set_option('fuse_unpruned', 1)
    if args.fuse_sort:
        cx.set_option('fuse_sort', args.fuse_sort)
    if not args.prefetch_next:
        cx.set_option('prefetch_next', 0)
    cx.set_option('rec_wt', args.rec_wt)
    cx.set_option('early_gather', args.early_gather)
    if not args.nn_bound:
        cx.set_option('nn_bound', 0)
    if args.shard_unpruned:
        cx.set_option('shard_unpruned', 1)
    if args.shard_emulate > 1:
        cx.set_option('shard_emulate', args.shard_emulate)
        cx.set_option('exchange', EXCHANGE[args.exchange])   # the emulated shards' exchange kernels
    return cx


def pipe_contexts(args, local, ctx):
    """the extra contexts of level pipelining (--pipe-ctx - 1 of them); with --pipe-priority the
    finest level's context (ctx) gets the high stream priority, the others the low one"""
    extra = [make_context(args, local) for _ in range(args.pipe_ctx - 1)]
    if args.pipe_priority and not os.environ.get('IA_CU_SPLIT'):   # CU-masked rehearsal streams keep theirs
        hi, lo = (1, 2) if args.pipe_priority == 1 else (2, 1)      # 2: reversed (experiment)
        ctx.set_option('stream_priority', hi)
        for cx in extra:
            cx.set_option('stream_priority', lo)
    if args.coarse_scan_wgs:
        for cx in extra:
            cx.set_option('scan_wgs', args.coarse_scan_wgs)
    if not args.coarse_fuse_gather:   # the coarser levels' merge and gather as separate launches
        for cx in extra:
            cx.set_option('fuse_gather', 0)
    return extra


def gather_rooflines(st):
    """K1 / K1b (per level) and K2 (sampled steps) against the HBM roofline: algorithmic bytes
    (include/ia.h ia_stats) / device time from libia's HIP events."""
    out = {}

    def one(name, ms, nbytes, launches, bound, what):
        if ms <= 0 or launches <= 0:
            return
        gbs = nbytes / (ms * 1e-3) / 1e9
        out[name] = {'achieved': gbs, 'peak': HBM_PEAK / 1e9, 'unit': 'GB/s', 'frac': gbs * 1e9 / HBM_PEAK,
                     'us_per_launch': ms * 1e3 / launches, 'algorithmic_bytes_per_launch': nbytes / launches,
                     'launches': launches, 'bound': bound, 'bytes': what}
    lv = 'the level with the largest DB (%d rows)' % st['build_rows']
    one('k_db64_build', st['k1b_ms'], st['k1b_bytes'], st['build_levels'], 'hbm',
        'A-side images read once + N_A rows x DS x 8 B written; ' + lv)
    one('k_db_build_h', st['k1_ms'], st['k1_bytes'], st['build_levels'], 'hbm',
        'fp64 rows read (N_A x DS x 8 B) + split-f16 tiles written (7 KiB per 32 rows); ' + lv)
    one('k_gather_query', st['gather_ms_timed'], st['gather_bytes_timed'], st['gather_launches_timed'],
        'latency (one wave per query: dependent window, coherence-row and DB loads)',
        'per query: 55 features + 12 coherence candidate rows (pruned levels) read, fp64 row + f16 fragments + '
        '|q|^2 + pruning record written')
    if st['merge_launches_timed'] > 0:
        out['k_merge_level'] = {'us_per_launch': st['merge_ms_timed'] * 1e3 / st['merge_launches_timed'],
                                'launches': st['merge_launches_timed'],
                                'bound': 'latency (one wave per query: record, rerank-row and coherence-row loads '
                                         'in dependent rounds)'}
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='cfg3', help='synthetic workload (ia_amd.synth.CONFIGS): cfg3 (default), '
                    'cfg2, cfg4 (2048^2 B vs 1024^2 A, kappa 25) or cfg5 (64-job sweep)')
    ap.add_argument('--sequential', action='store_true',
                    help='cfg5: run the sweep one job at a time (the reference\'s order) instead of batching the '
                         'jobs that share a GPU')
    ap.add_argument('--max-batch', type=int, default=16, help='cfg5: jobs per batched level call')
    ap.add_argument('--streams', type=int, default=3,
                    help='cfg5: libia contexts (HIP streams + host threads) the rank\'s jobs are dealt over '
                         '(1 / 2 / 3: 7.7-8.0 / 9.1-9.4 / 9.7 M px/s on one MI355X, profiles/r02/streams)')
    ap.add_argument('--mode', default='auto', choices=['auto', 'replicas', 'shard'],
                    help='N > 1: shard (default for cfg2/cfg3/cfg4: BASELINE config 3 as named, one job whose DB '
                         'is sharded over the ranks, one winner exchange per wavefront step; the replicas aggregate '
                         'rides along as value_replicas) or replicas (one independent job per GPU)')
    ap.add_argument('--exchange', default='owner', choices=['owner', 'peer', 'rccl'],
                    help='shard mode: owner = rank r owns job r, sorted queries out and scan records back as one-shot '
                         'xGMI peer writes (HIP IPC buffers, include/ia.h ia_xchg_*); peer = every rank holds every '
                         'job, per-shard winners exchanged by peer writes fused into the merge; rccl = ncclAllGather '
                         '+ a finish kernel')
    ap.add_argument('--shard-jobs', type=int, default=0,
                    help='jobs stepped together over the sharded DB (0 = N in --mode shard at N > 1, else 1): J '
                         'cfg jobs sharing A (synth.make_jobs), every rank scanning its 1/N of the DB for all of them '
                         '(with --shard-emulate W on one GPU: the W-rank step for the cost model)')
    ap.add_argument('--no-replicas-extra', action='store_true',
                    help='N > 1 shard mode: skip the extra replicas measurement (value_replicas; the single-GPU '
                         'run of the rank\'s job that shard_parity compares against still runs once)')
    ap.add_argument('--strong', type=int, default=1, choices=[0, 1],
                    help='N > 1 shard mode: also time ONE cfg job whose DB is sharded over the N ranks '
                         '(value_strong, the single-analogy reading of BASELINE config 3) and check it bit for '
                         'bit against the single-GPU run (strong_parity)')
    ap.add_argument('--strong-exchange', default='peer', choices=['peer', 'rccl'],
                    help='exchange of the value_strong run: per-shard winners by peer writes fused into the merge '
                         '(peer) or ncclAllGather + a finish kernel (rccl)')
    ap.add_argument('--cpu-procs', type=int, default=4,
                    help='worker processes the CPU-baseline sample is split over (each single-threaded)')
    ap.add_argument('--matcher', default='f16x3', choices=['f16x3', 'f32'],
                    help='distance-scan MFMA: split-f16 (3 f16 MFMAs per 16 k) or fp32; both certified exact')
    ap.add_argument('--prune', type=int, default=1, choices=[0, 1],
                    help='certified pruned distance scan on large 1-channel levels (DESIGN.md §4b); identical results')
    ap.add_argument('--coarse-fuse-gather', type=int, default=1, choices=[0, 1],
                    help='0: the pipelined coarser levels run their merge and next gather as separate launches '
                         '(shorter-resident waves beside the finest level\'s scans); 1 (default): fused like the finest')
    ap.add_argument('--k3p-variant', type=int, default=24, choices=[20, 21, 22, 24, 25],
                    help='pruned-scan kernel version (ia_k3h.hip k3h_prune3, DESIGN.md §4b/§4h/§4i): 20 / 21 = whole '
                         'DB tiles in two register buffers, hi x hi block filter with the corrections fused on '
                         'query-tile pairs (in-kernel query sort / presorted); 22 = the hi-only tile stream, the lo '
                         'halves of filter-passing tiles one tile later; 24 / 25 = two passes: the hi stream by '
                         'LDS-DMA two tiles deep, then the passing tiles\' full chains (default).  Steps wider than 512 '
                         'queries run 21 (the measured fastest presorted form)')
    ap.add_argument('--pipeline', type=int, default=1, choices=[0, 1],
                    help='1 (default; one-job configs and replicas): consecutive levels overlap (two libia '
                         'contexts, each level\'s steps waiting only for the steps of the previous level they read; '
                         'DESIGN.md §6b); 0: levels one after the other (always in the owner-computes shard mode)')
    ap.add_argument('--fuse-gather', type=int, default=1, choices=[0, 1],
                    help='1 (default): on pruned one-job levels the merge of step t and the gather of step t + 1 run '
                         'as one launch (ia_kernels.hip k_merge_gather); 0: separate launches')
    ap.add_argument('--fuse-sort', type=int, default=0, choices=[0, 1, 2],
                    help='1: the fused gathers of step t + 1 also sort its queries for the presorted scan (include/ia.h '
                         'option fuse_sort); 0 (default): the scan sorts them in every workgroup (or K2s on wide steps); '
                         '2: 1 on levels whose widest step has >= 512 queries (DESIGN.md §6d)')
    ap.add_argument('--nn-bound', type=int, default=1, choices=[0, 1],
                    help='1 (default): the pruned levels\' gathers also bound U\' by the causal neighbours\' exact NN rows '
                         '(include/ia.h option nn_bound)')
    ap.add_argument('--rec-wt', type=int, default=1, choices=[0, 1],
                    help='1 (default): the pruned scan stores its records write-through (sc1), so the scan -> merge kernel '
                         'boundary finds no dirty record lines in L2 (include/ia.h option rec_wt, DESIGN.md §6e)')
    ap.add_argument('--early-gather', type=int, default=1, choices=[0, 1],
                    help='1 (default): a fused merge wave runs its next query\'s gather up to the row above\'s feature before '
                         'waiting for that handoff (include/ia.h option early_gather, DESIGN.md §6f)')
    ap.add_argument('--prefetch-next', type=int, default=1, choices=[0, 1],
                    help='1 (default): fused merge + gather waves load the next query\'s step-independent inputs during '
                         'the merge (include/ia.h option prefetch_next)')
    ap.add_argument('--owner-pipeline', type=int, default=0, choices=[0, 1],
                    help='1: pipelined levels in the owner-computes shard mode too (N > 1)')
    ap.add_argument('--fuse-unpruned', type=int, default=0, choices=[0, 1],
                    help='1: the fused merge + gather on unpruned levels too (measured slower, DESIGN.md §6c)')
    ap.add_argument('--pipe-ctx', type=int, default=4, choices=[2, 3, 4, 5],
                    help='contexts the pipelined levels rotate over (default 4: the finest level\'s stream is free '
                         'once level L - 5 ends; 2: level l + 2 follows level l on one stream; 5: measured slower, '
                         'DESIGN.md §6b)')
    ap.add_argument('--pipe-priority', type=int, default=1, choices=[0, 1, 2],
                    help='1: the finest level\'s stream at high priority, the coarser levels\' at low; 2: reversed')
    ap.add_argument('--coarse-scan-wgs', type=int, default=128,
                    help='pipelined levels: workgroups of the coarser levels\' pruned scans (0: one per CU, 256; '
                         'default 128: half the CUs, so the finest level\'s launches are not queued behind a '
                         'whole-GPU scan, DESIGN.md §6g)')
    ap.add_argument('--scan-wgs', type=int, default=0,
                    help='workgroups of every context\'s split-f16 scans (0: one per CU, 256; pipelined runs: '
                         'the finest level\'s, the coarser levels\' follow --coarse-scan-wgs)')
    ap.add_argument('--k3p-blocks', type=int, default=1, choices=[0, 1],
                    help='pruned scan of a step wider than 11 query tiles: 1 = one launch of (query block x DB '
                         'chunk) workgroups, 0 = one launch per query block')
    ap.add_argument('--prune-group', type=int, default=1, choices=[1, 2, 4, 8],
                    help='pruned levels: Morton tiles interleaved in groups of G (ia_prune.hip k_make_table)')
    ap.add_argument('--prune-min-rows', type=int, default=None,
                    help='smallest DB (rows) the pruned scan is used on (default: 262,144 = the 512^2 A level too for '
                         'the pipelined cfg3 and cfg4 jobs, where its lighter scan interferes less with the finest level: '
                         'cfg3 +0.9-1.9 %% on three boxes (profiles/r04/prune512), cfg4 +2.3 %% with option nn_bound '
                         '(profiles/r04/nn_bound); cfg5\'s 512^2 finest levels: 9.27 -> 14.59 M px/s (profiles/r04/nn_bound4); '
                         '524,288 = the 1024^2 level otherwise, libia\'s own default: the sequential cfg3 job loses 1.9 %% '
                         'with 262,144)')
    ap.add_argument('--shard-unpruned', action='store_true',
                    help='shard (or emulate shards of) levels that scan unpruned too (default: only pruned levels, '
                         'DESIGN.md §7)')
    ap.add_argument('--shard-emulate', type=int, default=1,
                    help='run every large level as a W-way DB shard on this one GPU (the multi-rank kernels '
                         'without the all-gather: per-shard scans and winners, then the finish); for the cost model')
    ap.add_argument('--time-stride', type=int, default=16,
                    help='sample K3 timing every S-th wavefront step (HIP events on libia\'s stream; every 4th '
                         'step cost 2 %% of the job, profiles/r02/stride)')
    ap.add_argument('--cpu-seconds', type=float, default=30.0,
                    help='wall-time budget of the CPU-baseline sample (about 10 s per sampled level)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--traffic-json', default=None,
                    help='per-launch HBM bytes of the dominant K3 kernel from a rocprofv3 --pmc pass of THIS '
                         'config (default: profiles/k3p_traffic_<config>.json; absent -> traffic null)')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.mode == 'auto':
        args.mode = 'shard' if (world > 1 and args.config != 'cfg5') else 'replicas'
    if args.config == 'cfg5' and args.mode == 'shard':
        ap.error('cfg5 is a sweep of independent jobs (replicas only): --mode shard does not apply')
    if args.config == 'cfg5' and args.shard_emulate > 1 and not args.sequential:
        ap.error('--shard-emulate takes one job per level call: add --sequential for cfg5')
    if args.prune_min_rows is None:
        args.prune_min_rows = 262144 if ((args.config in ('cfg3', 'cfg4') and args.pipeline) or args.config == 'cfg5') \
            else 524288
    if args.traffic_json is None:
        args.traffic_json = os.path.join(ROOT, 'profiles', 'k3p_traffic_%s.json' % args.config)
    import torch
    import ia_amd  # noqa: F401
    from ia_amd import _native, synth

    dist = None
    # rehearsal of the N > 1 path on a one-GPU box (IA_BENCH_SHARE_GPU=1: ranks share the visible
    # GPUs, IA_BENCH_BACKEND=gloo: RCCL refuses two ranks on one device); never set by the driver
    if os.environ.get('IA_BENCH_SHARE_GPU') == '1':
        local = local % max(torch.cuda.device_count(), 1)
        # exchanges wait on peers' kernels: ranks sharing a GPU get disjoint CU slices (libia
        # streams), else a waiting kernel can hold the CUs the peer needs
        os.environ['IA_CU_SPLIT'] = '%d/%d' % (rank, world)
    backend = os.environ.get('IA_BENCH_BACKEND', 'nccl')
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    dev = torch.device('cuda', local)

    kw, desc = synth.CONFIGS[args.config]
    t0 = time.time()
    sw = None
    if args.config == 'cfg5':
        from ia_amd import sweep
        n = kw['size']
        A = synth.smooth(n, n, 2, 1)
        sw = sweep.Sweep(A, [synth.filt(A)], synth.smooth(n, n, 2, 2), sweep.cfg5_jobs())
        mine = [j for j in range(len(sw.jobs)) if j % world == rank]
        deep = int(np.argmax(sw.L))
        job = synth.Job(sw.A_pyr, sw.Ap_pyr_list, sw.B_pyr, sw.Bp_init[deep], sw.jobs[deep].k, sw.weights)
        job_pixels = sw.pixels()
        job_flops = sum(2.0 * 55 * np.prod(sw.A_pyr[sw.offset(j) + l].shape[:2]) *
                        np.prod(sw.B_pyr[sw.offset(j) + l].shape[:2]) for j in range(len(sw.jobs))
                        for l in range(1, sw.L[j]))
        log('[bench] rank %d: sweep of %d jobs (%d on this rank) built in %.1fs: %d B\' px/step'
            % (rank, len(sw.jobs), len(mine), time.time() - t0, job_pixels))
    else:
        if args.shard_jobs <= 0:
            args.shard_jobs = world if (args.mode == 'shard' and world > 1) else 1
        jobs_b = synth.make_jobs(args.shard_jobs, **kw)
        job = jobs_b[0]
        job_pixels, job_flops = job.pixels, job.flops()
        log('[bench] rank %d: %d x job %s built in %.1fs: L=%d, %d B\' px/step, %.3e NN flops/step per job'
            % (rank, args.shard_jobs, args.config, time.time() - t0, job.L, job.pixels, job.flops()))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # host reference loop, sampled in spawned workers BEFORE this process initialises the GPU
        t1 = time.time()
        cpu = (cpu_baseline_sweep(sw, args.cpu_seconds, args.cpu_procs) if sw is not None
               else cpu_baseline(job, args.cpu_seconds, args.cpu_procs))
        log('[bench] CPU baseline sampled in %.1fs: %.3g px/s' % (time.time() - t1, cpu['value']))
    ctx = make_context(args, local)
    owner = args.mode == 'shard' and world > 1 and args.exchange == 'owner'
    pipe_owner = owner and args.pipeline and args.owner_pipeline
    if owner and args.shard_jobs != world:
        ap.error('--exchange owner: one job per rank (--shard-jobs N)')
    shard_error = None

    def agree(failed):
        """True when any rank failed (every rank gets the same answer)"""
        f = torch.tensor([1.0 if failed else 0.0], device=dev if backend == 'nccl' else 'cpu')
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        return float(f.item()) > 0

    if args.mode == 'shard' and world > 1:
        try:
            if owner:
                ctx.set_option('exchange', 2)
            if args.exchange == 'rccl':
                uid = [_native.comm_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(uid, src=0)
                ctx.comm_init(rank, world, uid[0])
            else:
                def all_gather(b):
                    out = [None] * world
                    dist.all_gather_object(out, b)
                    return out
                ctx.xchg_init(rank, world, all_gather)
            if os.environ.get('IA_BENCH_FAIL_SHARD') == str(rank):   # rehearsal of the fallback only
                raise RuntimeError('IA_BENCH_FAIL_SHARD')
        except Exception as e:   # e.g. no peer access between the GPUs: measured as replicas, said so
            shard_error = 'rank %d: %r' % (rank, e)
            log('[bench] shard setup failed: %s' % shard_error)
        if agree(shard_error is not None):
            shard_error = shard_error or 'a peer rank failed the shard setup'

    def fall_back():
        """the shard exchange failed on some rank: every rank measures replicas instead (the line
        says so in config.shard_error)"""
        nonlocal ctx, owner, pipe_owner
        log('[bench] rank %d: shard mode unavailable (%s): measuring replicas' % (rank, shard_error))
        ctx.close()
        ctx = make_context(args, local)
        args.mode, args.shard_jobs, owner, pipe_owner = 'replicas', 1, False, False
        d = DeviceJob(jobs_b[0], torch, dev)
        p2 = pipe_contexts(args, local, ctx) if args.pipeline else None
        return d, (lambda st, cs=None: d.run(ctx, torch, st, pipe=p2 if cs is None else None))
    ctxs = [ctx]
    if sw is not None:
        from ia_amd import sweep
        dsw = sweep.DeviceSweep(sw, mine, torch, dev)
        ctxs += [make_context(args, local) for _ in range(1, args.streams)]
        run = lambda st, cs=ctxs: dsw.run(cs, st, batched=not args.sequential, max_batch=args.max_batch)
        dj = dsw
    elif owner:   # this rank's own job; the other ranks bring theirs
        dj = DeviceJob(jobs_b[rank], torch, dev)
        if pipe_owner:
            # pipelined levels: the fused merge's waiter wave holds one SIMD until every owner's next
            # queries arrived, so the scans no longer spin on all CUs.  Measured
            # with two ranks on one GPU only (CU halves): 0.51 vs 4.63 M px/s, hence off by default
            ctx.set_option('xo_wait', 1)
            pctx = pipe_contexts(args, local, ctx)
            run = lambda st, cs=None: dj.run(ctx, torch, st, pipe=pctx if cs is None else None)
        else:
            run = lambda st, cs=ctxs: dj.run(cs[0], torch, st)
    elif args.shard_jobs > 1:
        dj = DeviceBatch(jobs_b, torch, dev)
        run = lambda st, cs=ctxs: dj.run(cs[0], torch, st)
    elif args.pipeline:
        dj = DeviceJob(job, torch, dev)
        pctx = pipe_contexts(args, local, ctx)
        # the roofline's single-stream pass (run(st, [ctx])) runs the levels one after the other
        run = lambda st, cs=None: dj.run(ctx, torch, st, pipe=pctx if cs is None else None)
    else:
        dj = DeviceJob(job, torch, dev)
        run = lambda st, cs=ctxs: dj.run(cs[0], torch, st)

    def timed(steps, fn, sample_events, hc=None):
        """steps x fn between barriers + device syncs; max over ranks.  hc (HostCopy): each step
        ends with the D2H copy of its results, inside the timed region"""
        if sample_events and args.time_stride > 0:
            ctx.set_option('time_dist', args.time_stride)
        # kernel-written stamps: the device time of every K3p / merge launch of these steps
        for cx in ALL_CTX:
            if cx.handle:
                cx.set_option('stamps', 1)
        stats = _native.Stats()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t_start = time.perf_counter()
        for _ in range(steps):
            fn(stats)
            if hc is not None:
                hc.fetch()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t_start
        ctx.set_option('time_dist', 0)
        for cx in ALL_CTX:
            if cx.handle:
                cx.set_option('stamps', 0)
        if dist:
            tt = torch.tensor([el], dtype=torch.float64, device=dev if backend == 'nccl' else 'cpu')
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el, stats

    if shard_error is not None:
        dj, run = fall_back()
        ctxs = [ctx]
    if owner and shard_error is None:
        # exchange = 2 lays every rank's slots out from its own job's geometry (include/ia.h): the
        # ranks' jobs must have identical level shapes, checked here instead of timing out
        geo = [tuple(x.shape) for x in dj.job.B_pyr[:dj.job.L]] + [tuple(x.shape) for x in dj.job.A_pyr[:dj.job.L]]
        allgeo = [None] * world
        dist.all_gather_object(allgeo, geo)
        if any(gx != allgeo[0] for gx in allgeo):
            shard_error = 'the ranks\' jobs differ in level shapes (exchange = 2 needs identical shapes)'
            dj, run = fall_back()
            ctxs = [ctx]

    def host_copy():
        """pinned host buffers for the timed job(s)' results (the D2H that ends every timed step)"""
        if sw is not None:
            return HostCopy([x for j in mine for l in range(1, sw.L[j])
                             for x in (dj.Bp[j][l], dj.S[j][l], dj.IM[j][l])], torch)
        return HostCopy(dj.outputs(), torch)
    hc = host_copy()
    for i in range(args.warmup):
        if world > 1 and args.mode == 'shard' and i == 0:
            try:
                run(_native.Stats())
            except Exception as e:   # e.g. IA_ECOMM: a peer's data never arrived
                shard_error = 'rank %d: %r' % (rank, e)
                log('[bench] sharded warmup failed: %s' % shard_error)
            if agree(shard_error is not None):
                shard_error = shard_error or 'a peer rank failed the sharded warmup'
                dj, run = fall_back()
                ctxs = [ctx]
                hc = host_copy()
                run(_native.Stats())
            continue
        run(_native.Stats())
    # with several streams (cfg5), HIP events around one stream's K3 launches also time the other
    # streams' kernels: the timed steps then run without events and the roofline comes from one
    # extra single-stream pass below
    # pipelined levels (or several cfg5 streams): HIP events around one stream's K3 launches would
    # also time the other stream's kernels, so the roofline comes from one extra sequential pass
    concurrent = len(ctxs) > 1 or (args.pipeline and sw is None and (not owner or pipe_owner) and args.shard_jobs <= 1)
    elapsed, stats = timed(args.steps, run, not concurrent, hc)
    # N = 1 self-check: the last timed step's fetched B', s, im (every level)
    # must equal, bit for bit, a one-stream sequential run of the same job - the roofline pass
    # below when the timed steps ran concurrently (pipelined levels, several cfg5 streams), else
    # one extra run
    # (cfg5 at any N: the rank's own jobs, also one sha1 per job - job_digests in the line, gathered
    # over the ranks, so a 2-rank sweep can be compared job by job with a one-GPU run)
    self_check = world == 1 or sw is not None
    h_timed = hc.digest() if self_check else None
    job_digests = None
    if sw is not None:
        dg = dict(zip(mine, hc.digest_groups([3 * (sw.L[j] - 1) for j in mine])))
        if dist:
            allg = [None] * world
            dist.all_gather_object(allg, dg)   # host objects only: no collective on the data path
            for x in allg:
                dg.update(x)
        job_digests = {str(j): dg[j] for j in sorted(dg)}
    dj1 = h_shard = None
    if world > 1 and args.mode == 'shard':
        # this rank's own job (owner mode: job `rank`; every rank holds every job otherwise: job
        # rank mod J) as the sharded run left it
        dj1 = dj.dj[rank % len(dj.dj)] if isinstance(dj, DeviceBatch) else dj
        hx = HostCopy(dj1.outputs(), torch)
        hx.fetch()
        h_shard = hx.digest()
    if concurrent:
        _, stats_rl = timed(1, lambda st: run(st, [ctx]), True)
    else:
        stats_rl = stats
        if self_check:
            run(_native.Stats(), [ctx])
    parity = None
    if self_check:
        hc.fetch()
        parity = hc.digest() == h_timed
        if dist:
            pp = [None] * world
            dist.all_gather_object(pp, parity)
            parity = all(pp)
        log('[bench] timed run %s the one-stream sequential run (sha1 of B\', s, im of every level)'
            % ('equals' if parity else 'DIFFERS FROM'))
    value_replicas = value_strong = shard_parity = strong_parity = None
    strong_info = None
    if world > 1 and args.mode == 'shard':
        # (1) the single-GPU run of this rank's own job (owner mode: job `rank`; every rank holds
        # every job otherwise: job rank mod J), which the sharded result must equal bit for bit;
        # timed, it is the other multi-GPU reading: one independent job per GPU, no collective
        # (value_replicas; never `value`: BASELINE config 3 is the sharded job)
        hc1 = HostCopy(dj1.outputs(), torch)
        rctx = make_context(args, local)
        if args.no_replicas_extra:
            dj1.run(rctx, torch, _native.Stats())
            hc1.fetch()
        else:
            el_r, _ = timed(args.steps, lambda st: dj1.run(rctx, torch, st), False, hc1)
            value_replicas = job_pixels * args.steps * world / el_r
        rctx.close()
        h_single = hc1.digest()
        ok = h_shard == h_single
        shard_parity = not agree(not ok)
        log('[bench] rank %d: sharded run of job %d %s its single-GPU run'
            % (rank, rank if owner else rank % args.shard_jobs, 'equals' if ok else 'DIFFERS FROM'))
        # (2) value_strong: ONE cfg job, its DB sharded over the N ranks (every rank holds the job,
        # scans its 1/N of each pruned level, per-step winner exchange), equal bit for bit to the
        # single-GPU run of that job (rank 0's job 0 above)
        if args.strong:
            strong_error, h_strong = None, None
            sctx = None
            try:
                sctx = make_context(args, local)
                if args.strong_exchange == 'rccl':
                    uid = [_native.comm_unique_id() if rank == 0 else None]
                    dist.broadcast_object_list(uid, src=0)
                    sctx.comm_init(rank, world, uid[0])
                else:
                    def all_gather_s(b):
                        o = [None] * world
                        dist.all_gather_object(o, b)
                        return o
                    sctx.xchg_init(rank, world, all_gather_s)
                ds = DeviceJob(jobs_b[0], torch, dev, a_from=dj1)
                hcs = HostCopy(ds.outputs(), torch)
                ds.run(sctx, torch, _native.Stats())   # warmup
                el_s, st_s = timed(args.steps, lambda st: ds.run(sctx, torch, st), False, hcs)
                value_strong = job_pixels * args.steps / el_s
                h_strong = hcs.digest()
            except Exception as e:
                strong_error = 'rank %d: %r' % (rank, e)
                log('[bench] strong (one-job) run failed: %s' % strong_error)
            if agree(strong_error is not None):
                value_strong = None
                strong_info = {'error': strong_error or 'a peer rank failed the one-job sharded run'}
            else:
                allh = [None] * world
                dist.all_gather_object(allh, (h_strong, h_single))
                ref = allh[0][1]          # rank 0's single-GPU run of job 0
                strong_parity = all(x[0] == ref for x in allh)
                strong_info = {'jobs': 1, 'exchange': args.strong_exchange, 'ms_per_step': el_s * 1e3 / args.steps,
                               'scaling': 'strong', 'parallelism': 'dbshard%d_jobs1' % world,
                               'note': 'one %s job (job 0), every pruned level\'s DB sharded %d ways, per-step '
                                       'certified winner exchange; value_strong = that job\'s B\' px / wall time'
                                       % (args.config, world)}
            if sctx is not None:
                sctx.close()

    # jobs whose pixels the timed steps produced: replicas one per rank; shard mode J jobs (every
    # rank holds all J: counted once); cfg5: the ranks split one sweep
    jobs = 1 if sw is not None else args.shard_jobs if args.shard_jobs > 1 else world if args.mode == 'replicas' else 1
    pixels = job_pixels * args.steps * jobs
    value = pixels / elapsed
    st = stats_rl.as_dict()
    st_all = stats.as_dict()
    log('[bench] rank %d stats: %s' % (rank, json.dumps(st)))

    k3_ms_per_launch = st['dist_ms'] / max(st['dist_launches_timed'], 1)
    flops_per_launch = st['dist_flops_timed'] / max(st['dist_launches_timed'], 1)
    achieved = flops_per_launch / (k3_ms_per_launch * 1e-3) if k3_ms_per_launch > 0 else 0.
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get('hbm_bytes_per_launch')
        except Exception:
            traffic = None
    f16 = st['f16_levels'] > 0
    peak = F16_MFMA_PEAK if f16 else FP32_MFMA_PEAK
    ch = dj.ch
    D = 55 * ch
    # MFMA flops the kernel issues per algorithmic flop: 3 f16 passes over 16*KS padded k
    # (split-f16) or 2*KH padded k (fp32); query-tile padding to 32 not included
    issued = 3.0 * 16 * {1: 4, 2: 7}.get(ch, 0) / D if f16 else (56 if ch == 1 else 112 if ch == 2 else 168) / D
    if st['prune_launches_timed'] > 0:
        # the dominant kernel is the pruned scan (k3h_prune3), and it streams the DB tiles it
        # needs: its roofline is HBM.  achieved = algorithmic bytes (DB tiles loaded x 7 KiB +
        # tile boxes + queries + records) / device time of its timed launches
        p_s = st['prune_ms_timed'] * 1e-3
        p_bytes = st['prune_bytes_timed'] / st['prune_launches_timed']
        p_gbs = st['prune_bytes_timed'] / p_s / 1e9
        p_tf = st['prune_flops_timed'] / p_s / 1e12
        roofline = {'bound': 'hbm', 'achieved': p_gbs, 'peak': HBM_PEAK / 1e9, 'unit': 'GB/s',
                    'frac': p_gbs * 1e9 / HBM_PEAK, 'traffic': traffic,
                    'algorithmic_bytes_per_launch': p_bytes,
                    'kernel': ('k3h_prune3 (certified pruned scan: PCA-box need tests, hi x hi block filter, split-f16 '
                               '3 x v_mfma_f32_32x32x16_f16, fused packed-index top-2)'),
                    'k3_us_per_launch': st['prune_ms_timed'] * 1e3 / st['prune_launches_timed'],
                    'k3_launches_sampled': st['prune_launches_timed'],
                    'mfma_achieved_tflops': p_tf, 'mfma_peak_tflops': peak / 1e12,
                    'mfma_frac': p_tf * 1e12 / peak, 'mfma_issue_frac': p_tf * 1e12 * issued / peak,
                    'all_k3_mfma_tflops': achieved / 1e12,
                    'k3_share_of_step': st['dist_ms'] * (st['dist_flops'] / max(st['dist_flops_timed'], 1)) /
                    max(elapsed * 1e3, 1e-9)}
    else:
        roofline = {'bound': 'mfma', 'achieved': achieved / 1e12, 'peak': peak / 1e12, 'unit': 'TFLOP/s',
                    'frac': achieved / peak, 'traffic': traffic,
                    'mfma_issue_frac': achieved * issued / peak,
                    'kernel': ('k3h_scan (3 x v_mfma_f32_32x32x16_f16 on hi/lo-split operands, fused packed-index top-2)'
                               if f16 else 'k3_dist (v_mfma_f32_32x32x2_f32 distance scan + fused top-2)'),
                    'k3_us_per_launch': k3_ms_per_launch * 1e3, 'k3_launches_sampled': st['dist_launches_timed'],
                    'k3_share_of_step': st['dist_ms'] * (st['dist_flops'] / max(st['dist_flops_timed'], 1)) /
                    max(elapsed * 1e3, 1e-9)}

    # SURVEY §8(d)'s own roofline basis: the brute-force NN flops of the job (sum 2*D*N_A*N_B,
    # nothing pruned) per second, against the fp32 MFMA dense peak.  The timed kernel does not
    # do that work (certified pruning skips most (DB tile, query tile) pairs), so this is an
    # "equivalent" rate and may exceed the peak; pairs_frac is the share actually contracted.
    fp32_equiv = job_flops * args.steps * jobs / elapsed
    roofline['note'] = ('headline = the HBM frac of the dominant kernel (the certified pruned scan streams the DB '
                        'tiles it needs); SURVEY §8(d)\'s fp32-MFMA basis (brute-force 2*D*N_A*N_B flops vs the fp32 '
                        'matrix peak) does not apply under certified pruning, which skips most of that work on '
                        'purpose: fp32_mfma_equiv_* is a work-equivalent rate, not a utilisation'
                        if st['prune_launches_timed'] > 0 else
                        'distance scan on MFMA; flops are the algorithmic 2*D*N_A*M per launch')
    if concurrent:
        roofline['k3_share_of_step'] = None   # single-stream pass vs concurrent timed steps: not comparable
        roofline['timing'] = ('K3/K2/K4 device times from one extra single-stream pass (the timed steps ran %s, '
                              'whose HIP events would overlap)' % ('%d concurrent streams' % len(ctxs) if len(ctxs) > 1
                                                                  else 'pipelined levels on %d streams' % args.pipe_ctx))
    if args.fuse_gather and st['prune_launches_timed'] > 0:
        roofline['fused_gather'] = ('the unsampled steps of a pruned level run K4 of step t and K2p of step t + 1 as one '
                                    'launch (k_merge_gather, DESIGN.md §6c); the sampled steps keep separate K2 / K4 '
                                    'launches, which the gather / merge timings in roofline.gathers measure')
    if st_all['k3p_stamp_launches'] > 0:
        # the timed steps' own launches (kernel-written s_memrealtime stamps, no events): every
        # pruned-scan launch of every timed step, in the configuration that is timed (pipelined
        # levels, concurrent streams)
        k3t = st_all['k3p_stamp_ms'] * 1e-3
        # algorithmic bytes count each DB tile of a launch at most once: a
        # launch of several query blocks (cfg4's wide steps) streams its tiles once per block, and
        # those repeats are priced as waste, not as work (streamed_bytes_per_launch_timed)
        ub = st_all.get('k3p_bytes_unique_all') or st_all['k3p_bytes_all']
        roofline['frac_timed'] = ub / k3t / HBM_PEAK
        roofline['achieved_timed'] = ub / k3t / 1e9
        roofline['k3_us_per_launch_timed'] = st_all['k3p_stamp_ms'] * 1e3 / st_all['k3p_stamp_launches']
        roofline['k3_launches_timed'] = st_all['k3p_stamp_launches']
        roofline['algorithmic_bytes_per_launch_timed'] = ub / st_all['k3p_stamp_launches']
        roofline['streamed_bytes_per_launch_timed'] = st_all['k3p_bytes_all'] / st_all['k3p_stamp_launches']
        if ub < st_all['k3p_bytes_all']:  # the sampled reading on the same basis
            for k in ('achieved', 'frac', 'algorithmic_bytes_per_launch'):
                if k in roofline:   # (absent without sampled timing, --time-stride 0)
                    roofline[k] *= ub / st_all['k3p_bytes_all']
        if roofline.get('traffic'):
            roofline['traffic_over_algorithmic'] = roofline['traffic'] / roofline['algorithmic_bytes_per_launch_timed']
        # the launch = its workgroups' start spread (dispatch, CUs held by concurrent kernels)
        # + their mean duration + the imbalance tail
        roofline['k3_wg_us_timed'] = st_all['k3p_stamp_wg_ms'] * 1e3 / st_all['k3p_stamp_launches']
        roofline['k3_start_spread_us_timed'] = st_all['k3p_stamp_start_ms'] * 1e3 / st_all['k3p_stamp_launches']
        if st_all['merge_stamp_launches'] > 0:
            roofline['merge_us_per_launch_timed'] = st_all['merge_stamp_ms'] * 1e3 / st_all['merge_stamp_launches']
            roofline['merge_launches_timed'] = st_all['merge_stamp_launches']
        # the fused merge + gather (k_merge_gather) of the same level: a latency-bound chain of
        # dependent memory rounds per query (one wave each), priced against HBM for scale only.
        # Bytes per query: the scan's records (20 B per chunk), the query row and
        # its pruning record, the coherence neighbours' s / im, the fp64 rows of the 15 coherence
        # candidates and the reranked MFMA candidates (+ their A' values), then the next query's
        # 55 features, its 30 U' candidates' s / im / NN rows and <= 28 fp64 U' rows, and the
        # writes (B', s, im, NN row, stats word, q64, fragments, pruning record, handoff slot)
        if st_all['merge_stamp_launches'] > 0 and sw is None:
            lvl_px = float(np.prod(job.B_pyr[job.L - 1].shape[:2]))
            q_per_launch = lvl_px * args.steps * jobs / st_all['merge_stamp_launches']
            rr = st_all['reranked'] / max(st_all['pixels'], 1)
            nwg = 256
            bq = nwg * 20 + 496 + 15 * 12 + (15 + rr) * 456 + 440 + 30 * 12 + 28 * 448 + 780
            mus = roofline['merge_us_per_launch_timed']
            roofline['merge'] = {
                'kernel': 'k_merge_gather (fused K4 merge of step t + K2p gather of step t + 1, one wave per query)',
                'bound': 'latency', 'queries_per_launch': q_per_launch, 'reranked_per_query': rr,
                'algorithmic_bytes_per_launch': bq * q_per_launch,
                'achieved_gbs': bq * q_per_launch / (mus * 1e-6) / 1e9,
                'frac_of_hbm': bq * q_per_launch / (mus * 1e-6) / HBM_PEAK,
                'dependent_memory_rounds': 3,
                'rounds': ('(1) the scan records + query row + neighbours\' s / im, (2) the candidates\' fp64 rows '
                           '(the next query\'s features, neighbours and U\' rows load beside it and during the '
                           'merge\'s compute: option early_gather), (3) the row above\'s handoff slot; then the '
                           'late feature and the pruning record from registers'),
                'us_per_launch_timed': mus}
        if st_all['stamp_gaps'] > 0:
            roofline['chain_gap_us_timed'] = st_all['stamp_gap_ms'] * 1e3 / st_all['stamp_gaps']
            if st_all.get('stamp_gaps_sm', 0) > 0 and st_all['stamp_gaps'] > st_all['stamp_gaps_sm']:
                # the two boundaries of a step: scan end -> merge start, merge end -> next scan start
                roofline['chain_gap_scan_merge_us_timed'] = st_all['stamp_gap_sm_ms'] * 1e3 / st_all['stamp_gaps_sm']
                roofline['chain_gap_merge_scan_us_timed'] = ((st_all['stamp_gap_ms'] - st_all['stamp_gap_sm_ms']) * 1e3
                                                             / (st_all['stamp_gaps'] - st_all['stamp_gaps_sm']))
            roofline['chain_window_ms_timed'] = st_all['stamp_window_ms'] / args.steps
        roofline['timing_timed'] = ('frac_timed / *_timed: every pruned-scan (and fused merge) launch of the %d timed '
                                    'steps, device time = max(workgroup end) - min(workgroup start) from s_memrealtime '
                                    'stamps the kernels write (include/ia.h option "stamps")' % args.steps)
    roofline['gathers'] = gather_rooflines(st)
    roofline['fp32_mfma_equiv_tflops'] = fp32_equiv / 1e12
    roofline['fp32_mfma_equiv_frac'] = fp32_equiv / FP32_MFMA_PEAK
    roofline['pairs_frac'] = st['dist_pairs'] / max(st['dist_pairs_full'], 1.)
    if st['dist_pairs_corrected'] > 0:
        # the hi x hi block filter: every box-needed pair runs the hi x hi product; only this share
        # also runs the two correction products and the top-2 epilogue (mfma_* above count 3)
        roofline['pairs_corrected_frac'] = st['dist_pairs_corrected'] / max(st['dist_pairs'], 1.)
        roofline['tiles_passing_frac'] = st['dist_tiles_rows'] / max(st['dist_tiles'], 1.)
    out = {'metric': METRIC, 'value': value, 'unit': "B' px/s", 'n_gpus': world, 'steps': args.steps,
           'warmup': args.warmup, 'ms_per_step': elapsed * 1e3 / args.steps, 'higher_is_better': True,
           'scaling': 'strong' if (sw is not None or (args.mode == 'shard' and jobs < max(world, args.shard_emulate)))
           else 'weak', 'vs_baseline': None,
           'dtype': 'f16x3' if f16 else 'f32',
           'data': 'synthetic', 'config': {'workload': '%s: %s' % (args.config, desc),
                                           'a_shape': list(job.A_pyr[-1].shape), 'b_shape': list(job.B_pyr[-1].shape),
                                           'pyramid_levels': job.L,
                                           'px_per_step': job_pixels, 'nn_flops_per_step': job_flops,
                                           'mode': 'sweep' if sw is not None else args.mode,
                                           'shard_emulate': args.shard_emulate,
                                           'exchange': args.exchange if (args.mode == 'shard' and world > 1) else None,
                                           'parallelism': (('jobs%d' % world) if sw is not None else
                                                           ('replicas%d' % world) if args.mode == 'replicas' and
                                                           args.shard_jobs <= 1 else
                                                           'dbshard%d_jobs%d' % (max(world, args.shard_emulate),
                                                                                 args.shard_jobs)),
                                           'jobs_per_step': jobs,
                                           'k3p_variant': args.k3p_variant,
                                           'level_pipeline': (('%d contexts%s' % (args.pipe_ctx, ', finest level high priority'
                                                                                  if args.pipe_priority else ''))
                                                              if args.pipeline and sw is None and (not owner or pipe_owner)
                                                              and args.shard_jobs <= 1 else None),
                                           'nn': 'exact: %s MFMA candidates + certified fp64 rerank'
                                                 % ('split-f16 (hi/lo x3)' if f16 else 'fp32'),
                                           'precision': ('f16x3 = every operand split into f16 hi + lo, 3 MFMA '
                                                         'products per 16 k (fp32 accumulate); the MFMA value only '
                                                         'nominates candidates, every decision is an fp64 rerank in '
                                                         "numpy's order under a certified error bound, i.e. the "
                                                         "reference's fp64 brute-force decisions"
                                                         if f16 else 'fp32 MFMA candidates + certified fp64 rerank'),
                                           'timed_region': ('per step: every level 1..L-1 (DB build, wavefront '
                                                            'synthesis) from device-resident pyramids, ending with '
                                                            "the D2H copy of every level's B'/s/im (%.1f MB) into "
                                                            'pinned host memory, back on the host' % (hc.nbytes / 1e6))},
           'roofline': roofline,
           'stats': {k: st_all[k] for k in ('pixels', 'steps', 'coherence_wins', 'reranked', 'fallbacks', 'db_ms',
                                        'synth_ms', 'bound_violations', 'kappa_ambiguous', 'f16_levels', 'pruned_levels',
                                        'dist_pairs', 'dist_pairs_full', 'dist_tiles', 'dist_tiles_full',
                                        'dist_pairs_corrected')}}
    if sw is not None:
        out['config']['sweep'] = {'jobs': len(sw.jobs), 'batched': not args.sequential, 'max_batch': args.max_batch,
                                  'streams': args.streams,
                                  'kappas': sorted({j.k for j in sw.jobs}), 'depths': sorted(set(sw.L))}
    if shard_error is not None:
        out['config']['shard_error'] = shard_error
    if world > 1 and args.mode == 'shard':
        out['shard_parity'] = shard_parity
        out['config']['exchange_used'] = args.exchange
        out['config']['shard_parity'] = ("each rank's own job of the timed sharded run (B', s, im of every level, "
                                         'sha1 of the D2H bytes) == the same job run alone on that GPU')
    if args.strong and world > 1 and args.mode == 'shard':
        out['value_strong'] = value_strong
        out['strong_parity'] = strong_parity
        out['config']['strong'] = strong_info
        # BASELINE config 3 is ONE 1024^2 analogy with its A database sharded
        # over the GPUs, so the headline at N > 1 is that one-job run (strong scaling); the N-job
        # weak reading (each rank owns a job, every rank scans its 1/N of the DB for all of them)
        # moves to value_weak beside value_replicas
        out['value_weak'] = value
        out['ms_per_step_weak'] = out['ms_per_step']
        out['config']['weak'] = {'jobs': jobs, 'exchange': args.exchange, 'parallelism': out['config']['parallelism'],
                                 'scaling': 'weak', 'note': 'value_weak = %d %s jobs sharing A, one owned per rank, '
                                                            'every pruned level\'s DB sharded %d ways' % (jobs, args.config, world)}
        if value_strong is not None:
            out['value'] = value_strong
            out['ms_per_step'] = strong_info['ms_per_step']
            out['scaling'] = 'strong'
            out['config']['parallelism'] = strong_info['parallelism']
            out['config']['jobs_per_step'] = 1
        else:   # the one-job run failed on some rank: the weak reading stays the value, said so
            out['config']['headline'] = 'value = the weak reading (the one-job sharded run failed: config.strong)'
    if value_replicas is not None:
        out['value_replicas'] = value_replicas
        out['config']['replicas'] = ('value_replicas = %d independent cfg jobs, one per GPU, no collective '
                                     '(B\' px/s aggregate)' % world)
    if job_digests is not None:
        out['job_digests'] = job_digests
    if parity is not None:
        out['parity'] = parity
        out['config']['parity'] = ("sha1 of the last timed step's fetched B', s, im (every level) == a one-stream "
                                   'sequential run of the same job on this GPU')
    if cpu is not None:
        out['cpu_baseline'] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    for cx in ctxs:
        cx.close()
    if dist:
        dist.destroy_process_group()
    if shard_parity is False or strong_parity is False or parity is False:
        log('[bench] PARITY FAILURE: a run differs from its reference run (parity %s, shard_parity %s, strong_parity %s)'
            % (parity, shard_parity, strong_parity))
        sys.exit(3)


if __name__ == '__main__':
    main()
