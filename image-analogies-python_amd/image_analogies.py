"""Driver with the reference's entry points (image_analogies.py:17-268):
img_setup(A_fname, Ap_fname_list, B_fname, out_path, c) and
image_analogies_main(A_fname, Ap_fname_list, B_fname, out_path, c, debug=False).

Setup (image reading, scaling, YIQ, remap, compression, pyramids, B' initialisation) follows
the reference; the Gaussian pyramids and the YIQ matrices run on the GPU (ia_gaussian_pyramid,
ia_color_matrix: bit-identical to the host restatement) unless config.gpu_preprocess is False.
The per-level loop (image_analogies.py:130-239) is one
ia_synthesize_level call per level on the GPU: create_index's DB for the level, the skewed
wavefront over B', exact NN, coherence, the kappa rule and the B'/s/im writeback.  There is no
CPU path.
"""
import os
import pickle
import time
import warnings

import numpy as np

from . import _native
from .algorithms import default_context
from .config import save_metadata, setup_vars
from .img_preprocess import (compress_values, compute_gaussian_pyramid, convert_to_RGB, convert_to_YIQ,
                             initialize_Bp, remap_luminance)


def _imread(src):
    if isinstance(src, np.ndarray):
        return src
    import matplotlib.image as mpimg
    return mpimg.imread(src)


def _imsave(path, img):
    import matplotlib.image as mpimg
    mpimg.imsave(path, np.clip(img, 0, 1))


def img_setup(A_fname, Ap_fname_list, B_fname, out_path, c):
    """image_analogies.py:17-94.  File names may also be numpy arrays."""
    check_windows(c)
    os.makedirs(out_path, exist_ok=True)
    A_orig, B_orig = _imread(A_fname), _imread(B_fname)
    if A_orig.ndim != B_orig.ndim:
        raise ValueError('A and B must have the same number of channels')
    Ap_orig_list = [_imread(f) for f in Ap_fname_list]
    for Ap_orig in Ap_orig_list:
        if Ap_orig.shape != A_orig.shape:
            raise ValueError("every A' must be aligned with A (same shape)")
    # 0..255 vs 0..1 detection; the reference tests the FIRST ROW of the LAST A' (quirk, :33)
    scale = lambda x: 255. if np.max(x) > 1.0 else 1.0
    sA, sB, sAp = scale(A_orig), scale(B_orig), scale(Ap_orig_list[-1][0])

    gpu = default_context() if getattr(c, 'gpu_preprocess', True) else None
    if c.convert:
        A = convert_to_YIQ(A_orig / sA, gpu)[:, :, 0]
        B_yiq = convert_to_YIQ(B_orig / sB, gpu)
        B = B_yiq[:, :, 0]
        Ap_list = [convert_to_YIQ(x / sAp, gpu)[:, :, 0] for x in Ap_orig_list]
    else:
        A, B = A_orig / sA, B_orig / sB
        Ap_list = [x / sAp for x in Ap_orig_list]
    if c.remap_lum:
        A, Ap_list = remap_luminance(A, Ap_list, B)
    if not c.init_rand:
        B_orig_pyr = compute_gaussian_pyramid(B, c.n_sm, c.n_levels, gpu)
    A, B = compress_values(A, B, c.AB_weight)
    c.num_ch, c.padding_sm, c.padding_lg, c.weights = setup_vars(A)

    A_pyr = compute_gaussian_pyramid(A, c.n_sm, c.n_levels, gpu)
    B_pyr = compute_gaussian_pyramid(B, c.n_sm, c.n_levels, gpu)
    Ap_pyr_list = [compute_gaussian_pyramid(x, c.n_sm, c.n_levels, gpu) for x in Ap_list]
    if c.convert:
        color_pyr_list = [compute_gaussian_pyramid(B_yiq, c.n_sm, c.n_levels, gpu)]
    else:
        color_pyr_list = [compute_gaussian_pyramid(x, c.n_sm, c.n_levels, gpu) for x in Ap_list]

    if len(A_pyr) != len(B_pyr):
        c.max_levels = min(len(A_pyr), len(B_pyr))
        warnings.warn('Warning: input images are very different sizes! The minimum number of levels will be used.')
        if getattr(c, 'level_align', 'coarse') == 'fine' and len(B_pyr) > len(A_pyr):
            # extension: pair B's finest levels with A's (B level k+d <-> A level k)
            d = len(B_pyr) - len(A_pyr)
            B_pyr = B_pyr[d:]
            if c.convert:
                color_pyr_list = [p[d:] for p in color_pyr_list]
            if not c.init_rand:
                B_orig_pyr = B_orig_pyr[d:]
    else:
        c.max_levels = len(B_pyr)
    src = B_pyr if c.init_rand else B_orig_pyr
    Bp_pyr = initialize_Bp(src, init_rand=c.init_rand, seed=getattr(c, 'seed', None))
    return A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, color_pyr_list, c


def check_windows(c):
    """The kernels hard-code the reference's 3x3 coarse / 5x5 fine windows (config.py:15-16;
    feature width 55 * ch): refuse other sizes loudly instead of misreading the weight vector."""
    n_sm, n_lg = getattr(c, 'n_sm', 3), getattr(c, 'n_lg', 5)
    if (n_sm, n_lg) != (3, 5) or int(getattr(c, 'n_half', 12)) != 12:
        raise ValueError('only n_sm = 3, n_lg = 5, n_half = 12 are supported (the reference defaults; '
                         'got n_sm = %r, n_lg = %r, n_half = %r)' % (n_sm, n_lg, getattr(c, 'n_half', None)))


def synthesize_pyramid(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, c, ctx=None, stats=None, on_level=None, debug=None):
    """The level loop of image_analogies_main (image_analogies.py:130-239) on the GPU.
    Bp_pyr levels 1..max_levels-1 are synthesised in place; returns ({level: s}, {level: im}).
    debug: a dict that receives {level: {'src', 'dist'}} per-pixel debug records
    (_native.Context.synthesize_level).
    Warns when a kappa decision sat where libm's pow (the reference's `** 2`) could round the
    other way than the kernel's y * y (ia_stats.kappa_ambiguous; 0 on every fixture)."""
    check_windows(c)
    ctx = ctx or default_context()
    L = c.max_levels
    S, IM = {}, {}
    stats = stats if stats is not None else _native.Stats()
    amb0 = stats.kappa_ambiguous
    for level in range(1, L):
        Bp_pyr[level] = np.ascontiguousarray(Bp_pyr[level], dtype=np.float64)
        kf = 1 + (2 ** (level - L)) * c.k          # image_analogies.py:206
        dbg = None if debug is None else debug.setdefault(level, {})
        S[level], IM[level] = ctx.synthesize_level(
            A_pyr[level], A_pyr[level - 1], [p[level] for p in Ap_pyr_list], [p[level - 1] for p in Ap_pyr_list],
            B_pyr[level], B_pyr[level - 1], Bp_pyr[level - 1], Bp_pyr[level], c.weights, kf, stats, debug=dbg)
        if on_level is not None:
            on_level(level, S, IM)
    if stats.kappa_ambiguous > amb0:
        warnings.warn('%d kappa decisions were within libm pow rounding of the threshold: those pixels may '
                      'differ from the reference (ia_stats.kappa_ambiguous)' % (stats.kappa_ambiguous - amb0))
    return S, IM


def level_colour(level, Bp_pyr, S, IM, color_pyr_list, c):
    """Colour output of a level (image_analogies.py:216-217, 255-258)."""
    if c.convert:
        gpu = default_context() if getattr(c, 'gpu_preprocess', True) else None
        return np.clip(convert_to_RGB(np.dstack([Bp_pyr[level], color_pyr_list[0][level][:, :, 1:]]), gpu), 0, 1)
    h, w = Bp_pyr[level].shape[:2]
    src = np.stack([p[level] for p in color_pyr_list])[IM[level], S[level][:, 0], S[level][:, 1]]
    out = np.empty((h * w, 3))
    out[:] = src.reshape(h * w, -1)
    return out.reshape(h, w, 3)


def debug_structures(S_l, IM_l, dbg, shape):
    """The debug=True bookkeeping of image_analogies.py:141-153,224-240 and :244-246 for one level,
    from the GPU's per-pixel records (include/ia.h dbg_src / dbg_dist).  Returns
    {'sa', 'sc', 'rstars', 'p_src', 'app_dist', 'coh_dist', 'img_src'}: sa = p_app per pixel;
    sc / rstars = p_coh (= s[r_star] + q - r_star) / r_star where a coherence candidate existed,
    (0, 0) otherwise (also at the level's first pixel); p_src colours coherence-chosen pixels
    [1, 1, 0], NN-chosen ones [1, 0, 0] and pixels without a candidate [0, 0, 0]; img_src = im /
    max(im) (0/0 = nan with one A' image, as in the reference)."""
    h, w = shape
    src, dist = dbg['src'], dbg['dist']
    n = h * w
    sa = [(int(x[0]), int(x[1])) for x in src[:, :2]]
    sc, rstars = [], []
    p_src = np.nan * np.ones((h, w, 3))
    app_dist = np.zeros((h, w))
    coh_dist = np.zeros((h, w))
    for qi in range(n):
        r, col = divmod(qi, w)
        if qi > 0 and src[qi, 5]:
            rr, rc = int(src[qi, 3]), int(src[qi, 4])
            nb = rr * w + rc
            p_coh = (int(S_l[nb, 0]) + r - rr, int(S_l[nb, 1]) + col - rc)
            sc.append(p_coh)
            rstars.append((rr, rc))
            app_dist[r, col], coh_dist[r, col] = dist[qi]
            if (int(S_l[qi, 0]), int(S_l[qi, 1])) == p_coh:          # np.allclose(p, p_coh)
                p_src[r, col] = [1, 1, 0]
            else:
                p_src[r, col] = [1, 0, 0]
        else:
            sc.append((0, 0))
            rstars.append((0, 0))
            p_src[r, col] = [0, 0, 0]
    with np.errstate(invalid='ignore', divide='ignore'):
        img_src = (np.asarray(IM_l).astype(np.float64) / np.max(IM_l)).reshape(h, w)
    return {'sa': sa, 'sc': sc, 'rstars': rstars, 'p_src': p_src, 'app_dist': app_dist, 'coh_dist': coh_dist,
            'img_src': img_src}


def _save_debug(out_path, level, d, Bp_l, S_l, IM_l):
    """image_analogies.py:244-253: the five debug maps as .eps and the [sa, sc, rstars, s, im]
    pickle (binary mode; the reference's text-mode open fails on Python 3)."""
    try:
        import matplotlib
        matplotlib.use('Agg')
        import matplotlib.pyplot as plt
        from .img_preprocess import savefig_noborder
        paths = ['%d_psrc.eps', '%d_appdist.eps', '%d_cohdist.eps', '%d_output.eps', '%d_imgsrc.eps']
        for path, var in zip(paths, [d['p_src'], d['app_dist'], d['coh_dist'], Bp_l, d['img_src']]):
            fig = plt.imshow(var, interpolation='nearest', cmap='gray')
            savefig_noborder(out_path + path % level, fig)
            plt.close()
    except ImportError:
        warnings.warn('matplotlib is not importable: debug .eps maps skipped')
    s_list = [np.array([int(x[0]), int(x[1])]) for x in S_l]
    with open(out_path + '%d_srcs.pickle' % level, 'wb') as f:
        pickle.dump([d['sa'], d['sc'], d['rstars'], s_list, [int(x) for x in IM_l]], f)


def image_analogies_main(A_fname, Ap_fname_list, B_fname, out_path, c, debug=False):
    """image_analogies.py:97-268.  Writes metadata.txt, level_<l>_color.jpg and
    <dirname>.jpg per level like the reference; debug=True additionally writes the reference's
    debug maps (<l>_psrc/appdist/cohdist/output/imgsrc.eps) and pickles [sa, sc, rstars, s, im]
    per level (image_analogies.py:141-153,224-253), built from the GPU's per-pixel records.
    Returns {'Bp_pyr', 's', 'im', 'stats'} (+ 'debug': {level: debug_structures} when debug)."""
    begin = time.time()
    A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, color_pyr_list, c = img_setup(A_fname, Ap_fname_list, B_fname, out_path, c)
    names = ['A_fname', 'Ap_fname_list', 'B_fname', 'c.convert', 'c.remap_lum', 'c.init_rand', 'c.AB_weight', 'c.k']
    vals = [A_fname if isinstance(A_fname, str) else '<array>',
            [f if isinstance(f, str) else '<array>' for f in Ap_fname_list],
            B_fname if isinstance(B_fname, str) else '<array>', c.convert, c.remap_lum, c.init_rand, c.AB_weight, c.k]
    save_metadata(out_path, names, vals)
    print('Environment Setup: %f' % (time.time() - begin))

    stats = _native.Stats()
    state = {'t': time.time()}

    def on_level(level, S, IM):
        col = level_colour(level, Bp_pyr, S, IM, color_pyr_list, c)
        _imsave(out_path + 'level_%d_color.jpg' % level, col)
        _imsave(out_path + out_path.rstrip('/').split('/')[-1] + '.jpg', col)
        if debug:
            dbg_out[level] = debug_structures(S[level], IM[level], dbg_raw[level], Bp_pyr[level].shape[:2])
            _save_debug(out_path, level, dbg_out[level], Bp_pyr[level], S[level], IM[level])
        now = time.time()
        print('Level %d time: %f' % (level, now - state['t']))
        state['t'] = now

    dbg_raw, dbg_out = ({}, {}) if debug else (None, None)
    S, IM = synthesize_pyramid(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, c, stats=stats, on_level=on_level, debug=dbg_raw)
    print('Total time: %f' % (time.time() - begin))
    print('GPU synthesis time: %f (DB build %f)' % (stats.synth_ms / 1e3, stats.db_ms / 1e3))
    out = {'Bp_pyr': Bp_pyr, 's': S, 'im': IM, 'stats': stats.as_dict()}
    if debug:
        out['debug'] = dbg_out
    return out
