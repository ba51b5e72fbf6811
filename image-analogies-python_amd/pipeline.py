"""Level pipelining over two or three libia contexts (include/ia.h ia_pipeline_depend).

Level l + 1 of a job reads level l's B' only around (r / 2, c / 2), so its wavefront step t needs
level l's steps <= t / 2 + 4 and can start long before level l ends.  Levels rotate over two or three
contexts (streams, scratch buffers), one host thread each; before each level call the context
declares which call of the other context (its generation) it depends on, and libia makes each
step wait (a stream event wait) for exactly the steps it reads.  Results equal the sequential
order bit for bit; device-resident levels only (a host-buffer level returns its B' at the end of
its call, too late for the next level's first steps).
"""
import os
import threading


def run_levels_pipelined(level_fn, ctxs, L, stats):
    """Levels 1 .. L-1 of one job over n >= 2 contexts, one host thread each: level_fn(ctx, l,
    stats) runs level l (device buffers); level l + 1 depends step by step on level l
    (ia_pipeline_depend with the generation the level-l call gets), level l + n follows level l
    on the same context.  The finest level runs on ctxs[0]; with n = 3 it starts as soon as the
    next-coarser level's first steps are done instead of after level L - 3 ends."""
    from . import _native
    for c in ctxs:
        c.set_option('pipeline_record', 1)
    base = [c.pipeline_generation() for c in ctxs]
    n = len(ctxs)
    side = lambda l: (L - 1 - l) % n   # the finest level on ctxs[0] (the context bench.py samples)
    gen = {}
    for l in range(1, L):   # the generation number each level call will get on its context
        gen[l] = base[side(l)] + sum(1 for k in range(1, l + 1) if side(k) == side(l))
    sts = [_native.Stats() for _ in ctxs]
    errs = []

    def worker(w):
        try:
            for l in range(1, L):
                if side(l) != w:
                    continue
                if l > 1:
                    ctxs[w].pipeline_depend(ctxs[side(l - 1)], gen[l - 1])
                if l == L - 1 and not os.environ.get('IA_PIPE_RECORD_ALL'):
                    ctxs[w].set_option('pipeline_last', 1)   # nothing depends on the finest level: no per-step events
                level_fn(ctxs[w], l, sts[w])
        except Exception as e:   # the other thread's waits end by timeout (IA_ECOMM)
            errs.append(e)
    th = [threading.Thread(target=worker, args=(w,)) for w in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    for st in sts:
        stats.add(st)
