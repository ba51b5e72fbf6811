"""ctypes boundary to libia.so (include/ia.h).

This is the only way the package reaches the GPU: there is no CPU fallback.  If libia.so is
missing, or no gfx950 device is visible, every entry point raises IAError loudly.
"""
import ctypes
import math
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('IA_LIBIA') or os.path.join(_HERE, 'libia.so')  # override: diagnostic builds

IA_MEM_HOST, IA_MEM_DEVICE = 0, 1
IA_MATCH_F32, IA_MATCH_F16X3 = 0, 1   # option "matcher" (include/ia.h)
_ERRNAMES = {-1: 'IA_EINVAL', -2: 'IA_EHIP', -3: 'IA_ENOMEM', -4: 'IA_ENODEV', -5: 'IA_ECOMM'}


class IAError(RuntimeError):
    pass


class LevelArgs(ctypes.Structure):
    _fields_ = [('ch', ctypes.c_int), ('n_ap', ctypes.c_int), ('a_h', ctypes.c_int), ('a_w', ctypes.c_int),
                ('b_h', ctypes.c_int), ('b_w', ctypes.c_int),
                ('A', ctypes.c_void_p), ('Ac', ctypes.c_void_p), ('Ap', ctypes.c_void_p), ('Apc', ctypes.c_void_p),
                ('B', ctypes.c_void_p), ('Bc', ctypes.c_void_p), ('Bpc', ctypes.c_void_p), ('Bp', ctypes.c_void_p),
                ('weights', ctypes.c_void_p), ('kappa_factor', ctypes.c_double),
                ('s_out', ctypes.c_void_p), ('im_out', ctypes.c_void_p), ('mem', ctypes.c_int),
                ('dbg_src', ctypes.c_void_p), ('dbg_dist', ctypes.c_void_p)]


class Stats(ctypes.Structure):
    _fields_ = [('pixels', ctypes.c_int64), ('steps', ctypes.c_int64), ('coherence_wins', ctypes.c_int64),
                ('reranked', ctypes.c_int64), ('fallbacks', ctypes.c_int64), ('db_ms', ctypes.c_double),
                ('synth_ms', ctypes.c_double), ('dist_launches', ctypes.c_int64), ('dist_flops', ctypes.c_double),
                ('dist_ms', ctypes.c_double), ('dist_launches_timed', ctypes.c_int64),
                ('dist_flops_timed', ctypes.c_double), ('bound_violations', ctypes.c_int64),
                ('f16_levels', ctypes.c_int64), ('pruned_levels', ctypes.c_int64),
                ('dist_pairs', ctypes.c_double), ('dist_pairs_full', ctypes.c_double),
                ('dist_tiles', ctypes.c_double), ('dist_tiles_full', ctypes.c_double),
                ('prune_ms_timed', ctypes.c_double), ('prune_launches_timed', ctypes.c_int64),
                ('prune_flops_timed', ctypes.c_double), ('prune_bytes_timed', ctypes.c_double),
                ('kappa_ambiguous', ctypes.c_int64), ('dist_pairs_corrected', ctypes.c_double),
                ('dist_tiles_rows', ctypes.c_double),
                ('k1b_ms', ctypes.c_double), ('k1b_bytes', ctypes.c_double), ('k1_ms', ctypes.c_double),
                ('k1_bytes', ctypes.c_double), ('build_levels', ctypes.c_int64),
                ('gather_ms_timed', ctypes.c_double), ('gather_launches_timed', ctypes.c_int64),
                ('gather_bytes_timed', ctypes.c_double), ('merge_ms_timed', ctypes.c_double),
                ('merge_launches_timed', ctypes.c_int64), ('build_rows', ctypes.c_int64),
                ('k3p_stamp_ms', ctypes.c_double), ('k3p_stamp_launches', ctypes.c_int64),
                ('k3p_bytes_all', ctypes.c_double), ('merge_stamp_ms', ctypes.c_double),
                ('merge_stamp_launches', ctypes.c_int64), ('stamp_gap_ms', ctypes.c_double),
                ('stamp_gaps', ctypes.c_int64), ('stamp_window_ms', ctypes.c_double), ('prune_rows', ctypes.c_int64),
                ('k3p_stamp_start_ms', ctypes.c_double), ('k3p_stamp_wg_ms', ctypes.c_double),
                ('stamp_gap_sm_ms', ctypes.c_double), ('stamp_gaps_sm', ctypes.c_int64),
                ('k3p_bytes_unique_all', ctypes.c_double)]

    # fields that describe only the levels with the largest DB seen (build_rows / prune_rows)
    _BUILD = ('k1b_ms', 'k1b_bytes', 'k1_ms', 'k1_bytes', 'build_levels')
    _PRUNE = ('prune_ms_timed', 'prune_launches_timed', 'prune_flops_timed', 'prune_bytes_timed', 'k3p_stamp_ms',
              'k3p_stamp_launches', 'k3p_bytes_all', 'merge_stamp_ms', 'merge_stamp_launches', 'stamp_gap_ms',
              'stamp_gaps', 'stamp_window_ms', 'k3p_stamp_start_ms', 'k3p_stamp_wg_ms', 'stamp_gap_sm_ms',
              'stamp_gaps_sm', 'k3p_bytes_unique_all')

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}

    def add(self, other):
        """accumulate another Stats (e.g. of a concurrent context) field by field (the DB-build
        and pruned-scan timings keep the largest level's, as libia does)"""
        for rows, group in (('build_rows', self._BUILD), ('prune_rows', self._PRUNE)):
            if getattr(other, rows) > getattr(self, rows):
                for k in group:
                    setattr(self, k, 0)
                setattr(self, rows, getattr(other, rows))
        for k, _ in self._fields_:
            if k in ('build_rows', 'prune_rows') or (k in self._BUILD and other.build_rows < self.build_rows) or \
                    (k in self._PRUNE and other.prune_rows < self.prune_rows):
                continue
            setattr(self, k, getattr(self, k) + getattr(other, k))


EXPORTS = {
    'ia_init': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    'ia_destroy': (None, [ctypes.c_void_p]),
    'ia_last_error': (ctypes.c_char_p, []),
    'ia_version': (ctypes.c_int, []),
    'ia_set_option': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]),
    'ia_comm_unique_id': (ctypes.c_int, [ctypes.c_char_p]),
    'ia_comm_init': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
    'ia_xchg_alloc': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]),
    'ia_xchg_open': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
    'ia_pipeline_depend': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    'ia_pipeline_generation': (ctypes.c_int, [ctypes.c_void_p]),
    'ia_synthesize_level': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(LevelArgs), ctypes.POINTER(Stats)]),
    'ia_synthesize_levels': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(LevelArgs), ctypes.c_int,
                                            ctypes.POINTER(Stats)]),
    'ia_index_build': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_void_p)]),
    'ia_index_query': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    'ia_index_destroy': (None, [ctypes.c_void_p]),
    'ia_coherence_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    'ia_gaussian_pyramid': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    'ia_color_matrix': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int]),
    'ia_k3_microbench': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double)]),
    'ia_merge_winners': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    'ia_chain_budget': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    'ia_wavefront_shape': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                          ctypes.POINTER(ctypes.c_int64)]),
    'ia_wavefront_step': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_int)]),
    'ia_shard_tiles': (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                      ctypes.POINTER(ctypes.c_int64)]),
    'ia_shard_tiles_pruned': (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    'ia_shard_morton_tile': (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int]),
}

_lib = None
_lock = threading.Lock()


def lib():
    """Load libia.so (raises IAError if it was not built: run __graft_entry__.build())."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise IAError('libia.so not found at %s — build it with `make -C image-analogies-python_amd/csrc` '
                              'or __graft_entry__.build(); there is no CPU fallback' % LIB_PATH)
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in EXPORTS.items():
                if os.environ.get('IA_LIBIA') and not hasattr(L, name):
                    continue   # a diagnostic / earlier-round library (same-box A/B): its own symbol set
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().ia_last_error()
        raise IAError('%s failed (%s): %s' % (what, _ERRNAMES.get(rc, rc), msg.decode() if msg else ''))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def _c64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def check_level_shapes(A, Ac, Ap, Apc, B, Bc, Bpc, Bp, w):
    """The C ABI derives every size from A's channel count and B's shape (include/ia.h
    ia_level_args); check the rest here so a mismatched call raises instead of reading or
    writing past a host buffer.  Ap / Apc are the stacked A' images.  Returns ch."""
    if A.ndim not in (2, 3):
        raise IAError('A must be (h, w) or (h, w, ch)')
    ch = 1 if A.ndim == 2 else A.shape[2]
    if not 1 <= ch <= 3:
        raise IAError('images must have 1, 2 or 3 channels (got %d)' % ch)
    half = lambda x: (-(-x.shape[0] // 2), -(-x.shape[1] // 2)) + x.shape[2:]
    if B.ndim != A.ndim or B.shape[2:] != A.shape[2:]:
        raise IAError('B must have the channel count of A: %s vs %s' % (B.shape, A.shape))
    if Ap.ndim != A.ndim + 1 or Ap.shape[1:] != A.shape or Ap.shape[0] < 1:
        raise IAError("every A' level must have A's shape %s (got %s)" % (A.shape, Ap.shape[1:]))
    if Ac.shape != half(A):
        raise IAError('Ac must be the coarser level of A, %s (got %s)' % (half(A), Ac.shape))
    if Apc.shape != (Ap.shape[0],) + half(A):
        raise IAError("every coarse A' level must be %s (got %s)" % (half(A), Apc.shape[1:]))
    for name, x in (('Bc', Bc), ('Bpc', Bpc)):
        if x.shape != half(B):
            raise IAError('%s must be the coarser level of B, %s (got %s)' % (name, half(B), x.shape))
    if Bp.shape != B.shape:
        raise IAError("Bp must have B's shape %s (got %s)" % (B.shape, Bp.shape))
    if w.shape != (55 * ch,):
        raise IAError('weights must have 55 * ch = %d entries (3x3 / 5x5 windows; got %s)' % (55 * ch, w.shape))
    return ch


class Context(object):
    """One GPU (ia_ctx).  device: HIP ordinal (default: LOCAL_RANK or 0)."""

    def __init__(self, device=None):
        if device is None:
            device = int(os.environ.get('LOCAL_RANK', 0))
        self._h = ctypes.c_void_p()
        check(lib().ia_init(device, ctypes.byref(self._h)), 'ia_init(%d)' % device)
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().ia_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, name, value):
        check(lib().ia_set_option(self._h, name.encode(), int(value)), 'ia_set_option')

    def gaussian_pyramid(self, img, n_reduce, weights7):
        """ia_gaussian_pyramid on a host array: the n_reduce successive pyramid_reduce levels of
        img (finest first), as a list of arrays."""
        img = _c64(img)
        h, w = img.shape[:2]
        ch = 1 if img.ndim == 2 else img.shape[2]
        shapes, hh, ww = [], h, w
        for _ in range(n_reduce):
            hh, ww = (hh + 1) // 2, (ww + 1) // 2
            shapes.append((hh, ww) + img.shape[2:])
        out = np.empty(sum(int(np.prod(x)) for x in shapes) or 1, dtype=np.float64)
        w7 = _c64(weights7)
        check(lib().ia_gaussian_pyramid(self._h, _ptr(img), h, w, ch, n_reduce, _ptr(w7), _ptr(out), IA_MEM_HOST),
              'ia_gaussian_pyramid')
        res, off = [], 0
        for shp in shapes:
            n = int(np.prod(shp))
            res.append(out[off:off + n].reshape(shp))
            off += n
        return res

    def color_matrix(self, img, M):
        """ia_color_matrix: np.einsum('ij,klj->kli', M, img) for an (h, w, 3) host array."""
        img = _c64(img)
        if img.ndim != 3 or img.shape[2] != 3:
            raise IAError('color_matrix: (h, w, 3) image expected')
        out = np.empty_like(img)
        M = _c64(M)
        check(lib().ia_color_matrix(self._h, _ptr(img), img.shape[0] * img.shape[1], _ptr(M), _ptr(out), IA_MEM_HOST),
              'ia_color_matrix')
        return out

    def k3_microbench(self, n_rows, M, reps=20):
        """Mean device microseconds of one split-f16 distance-scan launch (random operands)."""
        us = ctypes.c_double()
        check(lib().ia_k3_microbench(self._h, int(n_rows), int(M), int(reps), ctypes.byref(us)), 'ia_k3_microbench')
        return us.value

    def comm_init(self, rank, world, uid):
        check(lib().ia_comm_init(self._h, rank, world, bytes(uid)), 'ia_comm_init')

    def xchg_init(self, rank, world, all_gather):
        """Peer-write winner exchange of sharded levels (include/ia.h ia_xchg_alloc/open):
        all_gather(bytes) -> list of every rank's bytes in rank order (e.g. a torch.distributed
        all_gather_object wrapper).  Makes this context rank `rank` of a world-rank DB shard."""
        h = ctypes.create_string_buffer(64)
        rc = lib().ia_xchg_alloc(self._h, world, h)
        hs = all_gather(h.raw if rc == 0 else b'')   # every rank takes part, even after a failure
        check(rc, 'ia_xchg_alloc')
        if len(hs) != world or any(len(x) != 64 for x in hs):
            raise IAError('xchg_init: expected %d handles of 64 bytes (a peer failed ia_xchg_alloc)' % world)
        check(lib().ia_xchg_open(self._h, rank, world, b''.join(hs)), 'ia_xchg_open')

    def pipeline_depend(self, prev, gen):
        """The next level call on this context waits, step by step, for the level call number
        `gen` of `prev` (a context with option pipeline_record = 1) - include/ia.h."""
        check(lib().ia_pipeline_depend(self._h, prev.handle if prev is not None else None, int(gen)),
              'ia_pipeline_depend')

    def pipeline_generation(self):
        return lib().ia_pipeline_generation(self._h)

    def synthesize_level(self, A, Ac, Ap_list, Apc_list, B, Bc, Bpc, Bp, weights, kappa_factor, stats=None,
                         debug=None):
        """ia_synthesize_level on host numpy arrays.  Bp (fp64, C-contiguous) is updated in place
        (the reference mutates Bp_pyr[level], image_analogies.py:214).  Returns (s, im):
        s (N, 2) int32 source pixel in A', im (N,) int32 source A' image, raster order.
        debug: a dict to receive the debug=True per-pixel records (include/ia.h dbg_src/dbg_dist):
        'src' (N, 6) int32 [p_app row, col, img, r_star row, col, has_coh], 'dist' (N, 2) fp64
        [d_app, d_coh] (image_analogies.py:224-240), finished on the host as numpy does."""
        job = dict(B=B, Bc=Bc, Bpc=Bpc, Bp=Bp, weights=weights, kappa_factor=kappa_factor, debug=debug)
        return self.synthesize_levels(A, Ac, Ap_list, Apc_list, [job], stats)[0]

    def synthesize_levels(self, A, Ac, Ap_list, Apc_list, jobs, stats=None):
        """ia_synthesize_levels: one level of several jobs that share the A side (A, A' levels l and
        l-1), e.g. a kappa / pyramid-depth sweep (multi_script.py).  jobs: list of dicts with
        B, Bc, Bpc, Bp (updated in place), weights, kappa_factor and optionally debug (a dict, see
        synthesize_level).  One DB, one distance scan per wavefront step for all jobs.  Returns
        [(s, im)] per job, each identical to a separate synthesize_level call."""
        if not 1 <= len(jobs) <= 32:
            raise IAError('synthesize_levels: 1..32 jobs per call (got %d)' % len(jobs))
        A, Ac = _c64(A), _c64(Ac)
        Ap = _c64(np.stack(Ap_list))
        Apc = _c64(np.stack(Apc_list))
        keep, args, outs = [], [], []
        for jb in jobs:
            B, Bc, Bpc, Bp, w = _c64(jb['B']), _c64(jb['Bc']), _c64(jb['Bpc']), jb['Bp'], _c64(jb['weights'])
            if not (isinstance(Bp, np.ndarray) and Bp.dtype == np.float64 and Bp.flags.c_contiguous):
                raise IAError('Bp must be a C-contiguous float64 array (updated in place)')
            ch = check_level_shapes(A, Ac, Ap, Apc, B, Bc, Bpc, Bp, w)
            bh, bw = B.shape[:2]
            s = np.empty((bh * bw, 2), dtype=np.int32)
            im = np.empty(bh * bw, dtype=np.int32)
            dsrc = ddist = None
            if jb.get('debug') is not None:
                dsrc = np.zeros((bh * bw, 6), dtype=np.int32)
                ddist = np.zeros((bh * bw, 2), dtype=np.float64)
            args.append(LevelArgs(ch, Ap.shape[0], A.shape[0], A.shape[1], bh, bw,
                                  _ptr(A), _ptr(Ac), _ptr(Ap), _ptr(Apc), _ptr(B), _ptr(Bc), _ptr(Bpc), _ptr(Bp),
                                  _ptr(w), float(jb['kappa_factor']), _ptr(s), _ptr(im), IA_MEM_HOST,
                                  None if dsrc is None else _ptr(dsrc), None if ddist is None else _ptr(ddist)))
            keep.append((B, Bc, Bpc, w))
            outs.append((s, im, dsrc, ddist, jb.get('debug')))
        arr = (LevelArgs * len(args))(*args)
        st = stats if stats is not None else Stats()
        check(lib().ia_synthesize_levels(self._h, arr, len(args), ctypes.byref(st)), 'ia_synthesize_levels')
        res = []
        for s, im, dsrc, ddist, debug in outs:
            if debug is not None:
                # compute_distance = norm(x) ** 2 on numpy scalars: sqrt, then libm pow(., 2), which
                # can differ from sqrt(v) * sqrt(v) by 1 ulp; finish it here exactly like that
                for qi in np.flatnonzero(dsrc[:, 5]):
                    ddist[qi, 0] = math.sqrt(ddist[qi, 0]) ** 2
                    ddist[qi, 1] = math.sqrt(ddist[qi, 1]) ** 2
                debug['src'], debug['dist'] = dsrc, ddist
            res.append((s, im))
        return res

    def synthesize_level_device(self, ch, n_ap, a_hw, b_hw, ptrs, kappa_factor, stats=None):
        """Same on device pointers (IA_MEM_DEVICE): ptrs = dict of int addresses for
        A, Ac, Ap, Apc, B, Bc, Bpc, Bp, weights, s_out, im_out (e.g. torch tensor data_ptr())."""
        return self.synthesize_levels_device(ch, n_ap, a_hw, b_hw, [ptrs], [kappa_factor], stats)

    def synthesize_levels_device(self, ch, n_ap, a_hw, b_hw, ptr_list, kappa_factors, stats=None):
        """ia_synthesize_levels on device pointers: one ptrs dict per job (the A-side addresses
        must be equal in all of them), one kappa factor per job."""
        args = []
        for ptrs, kf in zip(ptr_list, kappa_factors):
            p = {k: ctypes.c_void_p(int(v)) for k, v in ptrs.items()}
            args.append(LevelArgs(ch, n_ap, a_hw[0], a_hw[1], b_hw[0], b_hw[1], p['A'], p['Ac'], p['Ap'], p['Apc'],
                                  p['B'], p['Bc'], p['Bpc'], p['Bp'], p['weights'], float(kf),
                                  p['s_out'], p['im_out'], IA_MEM_DEVICE))
        arr = (LevelArgs * len(args))(*args)
        st = stats if stats is not None else Stats()
        check(lib().ia_synthesize_levels(self._h, arr, len(args), ctypes.byref(st)), 'ia_synthesize_levels')
        return st


class ExactIndex(object):
    """ia_index_*: exact 1-NN over fp64 rows (FLANN `linear` semantics, numpy summation order)."""

    def __init__(self, ctx, pts):
        pts = _c64(pts)
        if pts.ndim != 2 or pts.shape[0] < 1:
            raise IAError('ExactIndex: pts must be a non-empty (n, d) array')
        self.ctx = ctx
        self.n, self.d = pts.shape
        self._h = ctypes.c_void_p()
        check(lib().ia_index_build(ctx.handle, _ptr(pts), self.n, self.d, ctypes.byref(self._h)), 'ia_index_build')

    def query(self, q):
        q = _c64(np.atleast_2d(q))
        if q.shape[1] != self.d:
            raise IAError('ExactIndex.query: query width %d != index width %d' % (q.shape[1], self.d))
        idx = np.empty(q.shape[0], dtype=np.int64)
        dist = np.empty(q.shape[0], dtype=np.float64)
        check(lib().ia_index_query(self._h, _ptr(q), q.shape[0], _ptr(idx), _ptr(dist)), 'ia_index_query')
        return idx, dist

    def coherence(self, q, px, s, im, A_hw, Bp_w, pad=2):
        """ia_coherence_batch: best_coherence_match (algorithms.py:92-130) of every pixel px[i]
        (row, col) with query feature q[i], against this index's rows (As).  s (n, 2) / im (n)
        must cover every causal neighbour of the batch.  Returns (p (nq, 2), img (nq,),
        r_star (nq, 2)) as int32; p = (-1, -1), img 0, r_star (0, 0) where there is no candidate."""
        q = _c64(np.atleast_2d(q))
        px = np.ascontiguousarray(np.atleast_2d(px), dtype=np.int32)
        s = np.ascontiguousarray(np.asarray(s).reshape(-1, 2), dtype=np.int32)
        im = np.ascontiguousarray(np.asarray(im).reshape(-1), dtype=np.int32)
        if q.shape[1] != self.d or px.shape != (q.shape[0], 2) or len(im) != len(s):
            raise IAError('ExactIndex.coherence: q (nq, %d), px (nq, 2) and len(s) == len(im) expected' % self.d)
        nq = q.shape[0]
        p = np.empty((nq, 2), dtype=np.int32)
        img = np.empty(nq, dtype=np.int32)
        rs = np.empty((nq, 2), dtype=np.int32)
        check(lib().ia_coherence_batch(self._h, _ptr(q), nq, _ptr(px), _ptr(s), _ptr(im), len(s), int(A_hw[0]),
                                       int(A_hw[1]), int(Bp_w), int(pad), _ptr(p), _ptr(img), _ptr(rs)),
              'ia_coherence_batch')
        return p, img, rs

    def close(self):
        if self._h:
            lib().ia_index_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    buf = ctypes.create_string_buffer(128)
    check(lib().ia_comm_unique_id(buf), 'ia_comm_unique_id')
    return buf.raw


def merge_winners(dist, row):
    """Host restatement-free merge (compiled in libia): dist/row (world, nq) -> (nq,) winners."""
    dist = _c64(dist)
    row = np.ascontiguousarray(row, dtype=np.int64)
    world, nq = dist.shape
    do = np.empty(nq, dtype=np.float64)
    ro = np.empty(nq, dtype=np.int64)
    check(lib().ia_merge_winners(_ptr(dist), _ptr(row), world, nq, _ptr(do), _ptr(ro)), 'ia_merge_winners')
    return do, ro


def wavefront_step(h, w, t):
    """(r0, M): step t covers pixels (r, t - 3r) for r in r0 .. r0 + M - 1."""
    r0, m = ctypes.c_int(), ctypes.c_int()
    check(lib().ia_wavefront_step(h, w, t, ctypes.byref(r0), ctypes.byref(m)), 'ia_wavefront_step')
    return r0.value, m.value


def shard_tiles(n_rows, world, rank):
    """Tiles [t0, t1) of `rank`; position j of tile t holds DB row j * ceil(n_rows/32) + t."""
    a, b = ctypes.c_int64(), ctypes.c_int64()
    check(lib().ia_shard_tiles(n_rows, world, rank, ctypes.byref(a), ctypes.byref(b)), 'ia_shard_tiles')
    return a.value, b.value


def shard_tiles_pruned(n_rows, world, rank):
    """Storage tiles [t0, t1) of `rank` on a pruned level (Morton tiles rank, rank + world, ...)."""
    a, b = ctypes.c_int64(), ctypes.c_int64()
    check(lib().ia_shard_tiles_pruned(n_rows, world, rank, ctypes.byref(a), ctypes.byref(b)), 'ia_shard_tiles_pruned')
    return a.value, b.value


def shard_morton_tile(storage_tile, n_tiles, world):
    return lib().ia_shard_morton_tile(storage_tile, n_tiles, world)


TILE_MUL = 2654435761  # IA_TILE_MUL of ia_internal.h


def shard_rows(n_rows, world, rank):
    """Sorted DB rows owned by `rank` (tile-strided layout, see shard_tiles)."""
    t0, t1 = shard_tiles(n_rows, world, rank)
    nt = (n_rows + 31) // 32
    perm = np.arange(t0, t1, dtype=np.int64) * (TILE_MUL % nt) % nt  # ia_tile_perm (ia_internal.h)
    rows = (np.arange(32)[:, None] * nt + perm[None, :]).ravel()
    return np.sort(rows[rows < n_rows])


def chain_budget(n_cu, vgprs, api_blocks_per_cu, wg_threads=64):
    """include/ia.h ia_chain_budget: deadlock-free handoff-chained waves in flight (0: never chain)"""
    return lib().ia_chain_budget(n_cu, vgprs, api_blocks_per_cu, wg_threads)


def wavefront_shape(h, w):
    s, m = ctypes.c_int64(), ctypes.c_int64()
    check(lib().ia_wavefront_shape(h, w, ctypes.byref(s), ctypes.byref(m)), 'ia_wavefront_shape')
    return s.value, m.value
