"""pyflann drop-in over libia's exact GPU index ("minimal" depth).

The reference imports pyflann once (`import pyflann as pf`, algorithms.py:5) and uses it at
three call sites: `pf.FLANN()` (algorithms.py:56), `build_index(pts, algorithm='kdtree')`
(:69, returns a params dict with 'checks') and `nn_index(q, 1, checks=...)` (:74, returns
(indices, squared distances)).  A maintainer who keeps the reference's per-pixel loop replaces
that import with `import flann_mi355x as pf`.  Only the C ABI of include/ia.h is used here
(ctypes, no torch): ia_init, ia_index_build, ia_index_query, ia_index_destroy, ia_last_error.

Semantics change from FLANN's randomised kd-forest to exact 1-NN: squared L2 in fp64 with
numpy's summation order, lowest index on ties (FLANN `linear`, the reference's brute force).
"""
import ctypes
import os

import numpy as np

_LIB = os.environ.get('IA_LIBIA', os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libia.so'))
_vp, _i64 = ctypes.c_void_p, ctypes.c_int64
_L = None
_ctx = None


def _lib():
    global _L, _ctx
    if _L is None:
        L = ctypes.CDLL(_LIB)
        L.ia_init.argtypes = [ctypes.c_int, ctypes.POINTER(_vp)]
        L.ia_index_build.argtypes = [_vp, _vp, _i64, ctypes.c_int, ctypes.POINTER(_vp)]
        L.ia_index_query.argtypes = [_vp, _vp, _i64, _vp, _vp]
        L.ia_index_destroy.argtypes = [_vp]
        L.ia_index_destroy.restype = None
        L.ia_last_error.restype = ctypes.c_char_p
        ctx = _vp()
        if L.ia_init(int(os.environ.get('LOCAL_RANK', 0)), ctypes.byref(ctx)):
            raise RuntimeError(L.ia_last_error().decode())
        _L, _ctx = L, ctx
    return _L


class FLANN(object):
    """pf.FLANN(): one exact index per object (build_index replaces the previous one)."""

    def __init__(self, **kwargs):
        self._h = None
        self._pts = None

    def build_index(self, pts, algorithm='kdtree', **kw):
        L = _lib()
        self.delete_index()
        self._pts = np.ascontiguousarray(pts, dtype=np.float64)
        n, d = self._pts.shape
        h = _vp()
        if L.ia_index_build(_ctx, self._pts.ctypes.data, n, d, ctypes.byref(h)):
            raise RuntimeError(L.ia_last_error().decode())
        self._h = h
        return {'checks': kw.get('checks', 32), 'algorithm': algorithm}

    def nn_index(self, qpts, num_neighbors=1, checks=32, **kw):
        if self._h is None:
            raise RuntimeError('nn_index called before build_index')
        if num_neighbors != 1:
            raise ValueError('flann_mi355x: only num_neighbors=1 is supported')
        q = np.ascontiguousarray(np.atleast_2d(qpts), dtype=np.float64)
        idx = np.empty(len(q), np.int64)
        dist = np.empty(len(q), np.float64)
        if _lib().ia_index_query(self._h, q.ctypes.data, len(q), idx.ctypes.data, dist.ctypes.data):
            raise RuntimeError(_lib().ia_last_error().decode())
        return idx, dist

    def delete_index(self):
        if self._h is not None:
            _lib().ia_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.delete_index()
        except Exception:
            pass
