"""The C ABI without a GPU: libia.so loads, exports every entry point include/ia.h declares,
fails loudly (IA_ENODEV) instead of falling back to the CPU, and its host-side helpers (wavefront
schedule, shard split, winner merge) are right."""
import os
import re

import numpy as np
import pytest

import ia_amd  # noqa: F401
from ia_amd import _native
from conftest import ROOT


def _declared():
    hdr = open(os.path.join(ROOT, 'include', 'ia.h')).read()
    return sorted(set(re.findall(r'\b(ia_[a-z_]+)\s*\(', hdr)))


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    names = _declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(L, n), n
        assert n in _native.EXPORTS, n


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip('a GPU is visible')
    with pytest.raises(_native.IAError, match='IA_ENODEV'):
        _native.Context(0)


def test_last_error_and_einval():
    with pytest.raises(_native.IAError, match='IA_EINVAL'):
        _native.wavefront_step(4, 4, 999)
    with pytest.raises(_native.IAError, match='IA_EINVAL'):
        _native.shard_rows(0, 2, 0)


@pytest.mark.parametrize('h,w', [(1, 1), (1, 7), (7, 1), (2, 2), (3, 5), (4, 6), (8, 8), (15, 23), (59, 90),
                                 (117, 180), (64, 64), (1024, 1024)])
def test_wavefront_covers_level_in_causal_order(h, w):
    """with t = c + 3r every pixel appears exactly once, every causal read
    (rows r-2..r-1 x cols c-2..c+2, and (r, c-2), (r, c-1)) lies in an earlier step, and no
    reflected read of a raster-later pixel lies in the same step."""
    T, M = _native.wavefront_shape(h, w)
    assert T == w + 3 * (h - 1) and M == min(h, (w + 2) // 3)
    step = -np.ones((h, w), dtype=np.int64)
    for t in range(T):
        r0, m = _native.wavefront_step(h, w, t)
        assert 0 <= m <= M and (m >= 1 or w < 3)
        for r in range(r0, r0 + m):
            c = t - 3 * r
            assert 0 <= c < w and step[r, c] == -1
            step[r, c] = t
    assert (step >= 0).all()
    if h * w > 4096:
        return
    refl = lambda i, n: (i % (2 * n)) if (i % (2 * n)) < n else 2 * n - 1 - (i % (2 * n))
    for r in range(h):
        for c in range(w):
            t = step[r, c]
            reads = [(r + dy, c + dx) for dy in (-2, -1) for dx in range(-2, 3)] + [(r, c - 2), (r, c - 1)]
            for (y, x) in reads:
                yy, xx = refl(y, h), refl(x, w)
                if yy * w + xx < r * w + c:
                    assert step[yy, xx] < t          # synthesised before (reference sees final)
                elif (yy, xx) != (r, c):
                    assert step[yy, xx] > t          # still initial in both orders


def test_shard_tiles_partition():
    """Tiles split contiguously over ranks; the rows they hold (tile-strided layout) partition
    0..n_rows-1 exactly; small levels are replicated."""
    for n in (1, 31, 32, 100, 64 * 32 * 8, 70000, 1 << 16):
        nt = (n + 31) // 32
        for world in (1, 2, 4, 8):
            parts = [_native.shard_tiles(n, world, k) for k in range(world)]
            if parts[0] == (0, nt):
                assert all(p == (0, nt) for p in parts)        # replicated level
                continue
            assert parts[0][0] == 0 and parts[-1][1] == nt
            for a, b in zip(parts, parts[1:]):
                assert a[1] == b[0]
            rows = np.concatenate([_native.shard_rows(n, world, k) for k in range(world)])
            assert np.array_equal(np.sort(rows), np.arange(n))


def test_merge_winners_lowest_index_on_ties():
    d = np.array([[1.0, 2.0, 3.0, 0.5], [1.0, 1.5, 3.0, 0.5], [0.9, 2.0, 3.0, 0.5]])
    r = np.array([[10, 20, 30, 7], [5, 21, 31, 3], [11, 22, 29, 9]])
    do, ro = _native.merge_winners(d, r)
    assert list(do) == [0.9, 1.5, 3.0, 0.5]
    assert list(ro) == [11, 21, 29, 3]


def test_ctypes_structs_match_the_c_header(tmp_path):
    """ia_stats / ia_level_args as include/ia.h lays them out (gcc) == the ctypes mirrors in
    _native.py: same size and the same offset for every field, so the Python side can never read
    a shifted counter after a header change."""
    import ctypes
    import shutil
    import subprocess
    from ia_amd import _native
    if shutil.which('gcc') is None:
        pytest.skip('gcc not available')
    structs = {'ia_stats': _native.Stats, 'ia_level_args': _native.LevelArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ia.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines += ['return 0;', '}']
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'layout'
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'include')
    subprocess.check_call(['gcc', '-std=c99', '-I', inc, str(src), '-o', str(exe)])
    got = {}
    for line in subprocess.check_output([str(exe)]).decode().splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, 'sizeof')] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_level_shape_contract_raises_before_the_abi():
    """every size the C ABI derives (weights = 55 * ch, B' = B's shape, coarse levels
    = ceil halves, A' = A's shape, B's channel count = A's) is checked on the host first."""
    import numpy as np
    import ia_amd  # noqa: F401
    from ia_amd import _native
    A, Ac = np.zeros((9, 7)), np.zeros((5, 4))
    B, Bc = np.zeros((6, 8)), np.zeros((3, 4))
    Ap, Apc = np.zeros((1, 9, 7)), np.zeros((1, 5, 4))
    w = np.zeros(55)
    assert _native.check_level_shapes(A, Ac, Ap, Apc, B, Bc, Bc, B.copy(), w) == 1
    bad = [
        (A, Ac, Ap, Apc, B, Bc, Bc, B.copy(), np.zeros(31)),            # n_lg = 3 weight vector
        (A, Ac, Ap, Apc, B, Bc, Bc, np.zeros((6, 7)), w),               # B' shape
        (A, np.zeros((4, 4)), Ap, Apc, B, Bc, Bc, B.copy(), w),         # coarse A
        (A, Ac, np.zeros((1, 9, 6)), Apc, B, Bc, Bc, B.copy(), w),      # A' shape
        (A, Ac, Ap, Apc, B, np.zeros((3, 3)), Bc, B.copy(), w),         # coarse B
        (A, Ac, Ap, Apc, B, Bc, np.zeros((2, 4)), B.copy(), w),         # coarse B'
        (A, Ac, Ap, Apc, np.zeros((6, 8, 3)), np.zeros((3, 4, 3)), np.zeros((3, 4, 3)),
         np.zeros((6, 8, 3)), np.zeros(165)),                           # channels of B != A
    ]
    for args in bad:
        with pytest.raises(_native.IAError):
            _native.check_level_shapes(*args)


def test_window_sizes_other_than_the_reference_are_refused():
    import types
    import ia_amd  # noqa: F401
    from ia_amd.image_analogies import check_windows
    check_windows(types.SimpleNamespace(n_sm=3, n_lg=5, n_half=12))
    for bad in (dict(n_sm=3, n_lg=3, n_half=4), dict(n_sm=5, n_lg=5, n_half=12)):
        with pytest.raises(ValueError):
            check_windows(types.SimpleNamespace(**bad))


def test_chain_budget_from_kernel_attributes():
    """the chained-wave budget (fused merge + gather launches whose waves wait
    for the row above) is derived from the compiled kernel's attributes, not a literal.  Stand-in
    attributes: round 4's k_merge_gather (264 VGPRs: one wave per SIMD, the occupancy API's 4
    one-wave workgroups per CU) gives 2 x 4 x 256 less 1/16 = 1,920 on 256 CUs; fewer resident
    waves shrink it, a kernel that cannot be resident disables chaining."""
    assert _native.chain_budget(256, 264, 4, 64) == 1920
    assert _native.chain_budget(128, 264, 4, 64) == 960              # a CU slice (rehearsal streams)
    assert _native.chain_budget(256, 264, 2, 64) == 960              # the API admits fewer: it wins
    assert _native.chain_budget(256, 200, 8, 64) == 2 * 8 * 256 - (2 * 8 * 256) // 16   # 2 waves per SIMD
    # above 3 waves per SIMD the SGPRs can bind and the API may answer one workgroup too many
    assert _native.chain_budget(256, 96, 20, 64) == 2 * 19 * 256 - (2 * 19 * 256) // 16
    assert _native.chain_budget(256, 600, 4, 64) == 0               # no resident wave: never chain
    assert _native.chain_budget(256, 264, 0, 64) == 0
    assert _native.chain_budget(0, 264, 4, 64) == 0
