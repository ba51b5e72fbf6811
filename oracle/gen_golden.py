#!/opt/conda/bin/python3.9
"""Golden-vector generator: runs the REAL reference code (flair2005/image-analogies-python)
in THIS container and writes small .npz fixtures under tests/golden/.

TEST INFRASTRUCTURE ONLY — never imported by the product package.

Recipe:
  1. copy /root/reference/*.py into a private tmpdir and run `lib2to3` on the copy
     (the reference is Python 2: tuple parameters algorithms.py:78,92, print statements
     image_analogies.py:114, xrange algorithms.py:56 / img_preprocess.py:67). Nothing from the
     reference (source or bytecode) is written into /root/repo; the tmpdir is deleted.
  2. runtime shims, none of which change the reference's decisions:
     - `pyflann` is absent offline: a stand-in FLANN whose nn_index is the EXACT first-argmin
       of `((pts - q)**2).sum(axis=1)` in fp64 (FLANN `linear` semantics, lowest-index ties).
       algorithms.py:69 asks for 'kdtree' (randomised, approximate) — that path is parity-unpinned.
     - config.n_half / pad_sm / pad_lg are np.float64 (config.py:18-20) and modern numpy refuses
       float slice bounds: set to the ints 12 / 1 / 2.
     - algorithms.np.floor/ceil return Python ints (algorithms.py:39,81-82 index with them).
     - skimage 0.18.3 pyramid_gaussian needs multichannel=True for (h,w,3) images
       (img_preprocess.py:56; the Py2-era skimage treated ndim==3 as multichannel).
     - plt.imread returns in-memory arrays; plt.imsave captures the colour output.
  3. state is captured by wrapping functions in the `image_analogies` module namespace.
  4. compute_distance's last bits depend on the ddot kernel OpenBLAS (DYNAMIC_ARCH) picks for
     the host CPU.  Containers whose CPUID OpenBLAS does not recognise fall back to the generic
     'Prescott' kernel, a different summation order than the SkylakeX kernel the round-1
     fixtures were made with.  OPENBLAS_CORETYPE=SkylakeX is therefore set before numpy loads,
     and _check_blas_order() refuses to write fixtures unless np.dot matches the order
     oracle/ia_oracle.py blas_ddot_sq (and the kernels' blas_dot_sq) restate.

Run:  /opt/conda/bin/python3.9 oracle/gen_golden.py            (base fixtures, ~1-2 min)
      /opt/conda/bin/python3.9 oracle/gen_golden.py cfg1 g128 ties128 k25 g256
                                        (round-2 larger e2e cases, one by one; g256 ~10-15 min)
"""
import os
import shutil
import subprocess
import sys
import tempfile
import types

os.environ.setdefault('OPENBLAS_CORETYPE', 'SkylakeX')   # before numpy loads OpenBLAS (step 4)
import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, '..', 'tests', 'golden')
REF = '/root/reference'


def _check_blas_order():
    sys.path.insert(0, os.path.join(HERE, '..'))
    from oracle.ia_oracle import blas_ddot_sq
    rs = np.random.RandomState(0)
    for n in list(range(1, 60)) + [110, 165]:
        for _ in range(8):
            x = rs.rand(n) * 1e-2
            if np.dot(x, x) != blas_ddot_sq(x):
                raise SystemExit('gen_golden: np.dot(x, x) (n=%d) does not follow the SkylakeX ddot order; '
                                 'OPENBLAS_CORETYPE=%s' % (n, os.environ.get('OPENBLAS_CORETYPE')))


# ----------------------------------------------------------------------------- shims
class _ExactFlann(object):
    """Stand-in for pyflann.FLANN: exact linear scan, fp64, first-argmin (lowest index).

    Large indexes (the g512 case) split the rows over threads: every row's distance is the
    same numpy expression on the same row ((p - q)**2 summed along the row), and the argmin runs
    on the concatenation, so the result is the single-threaded one bit for bit."""
    THREADS = int(os.environ.get('GEN_GOLDEN_THREADS', '1'))
    _pool = None

    def build_index(self, pts, algorithm='kdtree', **kw):
        self.pts = np.ascontiguousarray(pts, dtype=np.float64)
        n = len(self.pts)
        t = self.THREADS if n >= 65536 else 1
        self.cuts = [n * i // t for i in range(t + 1)]
        self.d = np.empty(n)
        if t > 1 and _ExactFlann._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            _ExactFlann._pool = ThreadPoolExecutor(self.THREADS)
        return {'checks': 32, 'algorithm': algorithm}

    def _part(self, q, a, b):
        self.d[a:b] = ((self.pts[a:b] - q) ** 2).sum(axis=1)

    def nn_index(self, q, num_neighbors=1, checks=32, **kw):
        q = np.asarray(q, dtype=np.float64)
        if len(self.cuts) == 2:
            d = ((self.pts - q) ** 2).sum(axis=1)
        else:
            fs = [self._pool.submit(self._part, q, a, b) for a, b in zip(self.cuts[:-1], self.cuts[1:])]
            for f in fs:
                f.result()
            d = self.d
        i = int(np.argmin(d))
        return np.array([i]), np.array([d[i]])


class _IntNp(object):
    """numpy proxy whose floor/ceil return Python ints for scalars."""

    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def floor(x):
        r = np.floor(x)
        return int(r) if np.ndim(r) == 0 else r

    @staticmethod
    def ceil(x):
        r = np.ceil(x)
        return int(r) if np.ndim(r) == 0 else r


def load_reference(tmp):
    for f in os.listdir(REF):
        if f.endswith('.py'):
            shutil.copy(os.path.join(REF, f), tmp)
    subprocess.check_call([sys.executable, '-m', 'lib2to3', '-w', '-n', tmp],
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    pf = types.ModuleType('pyflann')
    pf.FLANN = _ExactFlann
    sys.modules['pyflann'] = pf
    sys.path.insert(0, tmp)
    import matplotlib
    matplotlib.use('Agg')
    import config
    import img_preprocess
    import algorithms
    import image_analogies
    config.n_half, config.pad_sm, config.pad_lg = 12, 1, 2
    algorithms.np = _IntNp()
    from skimage.transform import pyramid_gaussian as _pg

    def pg(img, **kw):
        return _pg(img, multichannel=(img.ndim == 3), **kw)
    img_preprocess.pyramid_gaussian = pg
    return config, img_preprocess, algorithms, image_analogies


# ----------------------------------------------------------------------------- inputs
def smooth(h, w, sigma, seed, ch=None):
    from scipy.ndimage import gaussian_filter
    rs = np.random.RandomState(seed)
    if ch is None:
        x = gaussian_filter(rs.rand(h, w), sigma)
    else:
        x = np.dstack([gaussian_filter(rs.rand(h, w), sigma) for _ in range(ch)])
    x = x - x.min()
    return x / x.max()


def filt(A):
    from scipy.ndimage import gaussian_filter
    s = (2, 2, 0) if A.ndim == 3 else 2
    return np.clip(A ** 2.2 + 0.5 * (A - gaussian_filter(A, s)), 0, 1)


def blocky(h, w, seed, ch=None):
    """piecewise-constant image -> many exactly duplicated DB rows (tie stress, G7)."""
    rs = np.random.RandomState(seed)
    v = rs.randint(0, 3, size=((h + 3) // 4, (w + 3) // 4)).astype(np.float64) / 2.0
    x = np.kron(v, np.ones((4, 4)))[:h, :w]
    if ch:
        x = np.dstack([x] * ch)
    return x


# ----------------------------------------------------------------------------- end to end
def _sha1(x):
    import hashlib
    return hashlib.sha1(np.ascontiguousarray(x, dtype=np.float64).tobytes()).hexdigest()


def run_case(mods, name, A, Ap_list, B, convert=False, remap=False, init_rand=True,
             AB_weight=1, k=0.5, seed=3, lean=False, slim=False, n_levels=None):
    """lean: larger cases keep the fixture small: int32 index arrays, no colour pyramid when it
    equals the A' pyramid (convert=False), colour output of the finest level only.
    slim (g512): the reference's A / A' / B pyramids, the per-level outputs s (int16) / im
    (uint8), and the sha1 of every B' initialisation and final B' level - the test rebuilds the
    seeded B' initialisation with the product's host code (proved equal by the hashes), and
    compares its own s / im exactly and its B' by hash.  (The pyramids are stored because
    skimage's least-squares resize transform differs from the product's restatement in the last
    ulp, test_host_preprocess.py; the B' arrays are A' values at s, so their hashes suffice.)  n_levels: keep the finest n_levels images of every pyramid
    (the bench's cfg2 shape: 512^2 with 5 levels) by wrapping the reference's
    compute_gaussian_pyramid (img_preprocess.py:50-65: pyramid_gaussian builds each image from
    the previous one, so the finest five are the same arrays as in the full pyramid)."""
    config, img_preprocess, algorithms, ia = mods
    import matplotlib.pyplot as plt
    orig_cgp = ia.compute_gaussian_pyramid
    if n_levels is not None:
        ia.compute_gaussian_pyramid = lambda img, m: orig_cgp(img, m)[-n_levels:]
    imgs = {'A': A, 'B': B}
    for j, Ap in enumerate(Ap_list):
        imgs['Ap%d' % j] = Ap
    colour = {}
    plt.imread = lambda f: imgs[os.path.basename(f)]
    plt.imsave = lambda f, x, *a, **kw: colour.__setitem__(os.path.basename(f), np.array(x))

    config.convert, config.remap_lum, config.init_rand = convert, remap, init_rand
    config.AB_weight, config.k = AB_weight, k

    cap = {'app': [], 'coh': [], 'dist': []}
    orig_setup = ia.img_setup

    def img_setup(*a):
        r = orig_setup(*a)
        A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, color_pyr_list, c = r
        cap['A_pyr'] = [x.copy() for x in A_pyr]
        cap['Ap_pyr'] = [[x.copy() for x in p] for p in Ap_pyr_list]
        cap['B_pyr'] = [x.copy() for x in B_pyr]
        cap['Bp_init'] = [x.copy() for x in Bp_pyr]
        cap['color_pyr'] = [[x.copy() for x in p] for p in color_pyr_list]
        cap['Bp_live'] = Bp_pyr
        return r
    ia.img_setup = img_setup

    orig_bam = ia.best_approximate_match

    def bam(flann, params, q):
        r = orig_bam(flann, params, q)
        cap['app'].append(int(r))
        return r
    ia.best_approximate_match = bam

    orig_bcm = ia.best_coherence_match
    cap['s'] = {}

    def bcm(As, hw, q, s, im, px, w, c):
        r = orig_bcm(As, hw, q, s, im, px, w, c)
        cap['s'][id(s)] = (s, im)
        cap['coh'].append((int(r[0][0]), int(r[0][1]), int(r[1])))
        return r
    ia.best_coherence_match = bcm

    orig_cd = ia.compute_distance

    def cd(a, q, w):
        r = orig_cd(a, q, w)
        cap['dist'].append(float(r))
        return r
    ia.compute_distance = cd

    tmp = tempfile.mkdtemp()
    np.random.seed(seed)
    ia.image_analogies_main('A', ['Ap%d' % j for j in range(len(Ap_list))], 'B', tmp + '/out/', config)
    shutil.rmtree(tmp)
    ia.img_setup, ia.best_approximate_match = orig_setup, orig_bam
    ia.best_coherence_match, ia.compute_distance = orig_bcm, orig_cd
    ia.compute_gaussian_pyramid = orig_cgp

    L = config.max_levels
    if slim:
        out = {'L': L, 'k': k, 'seed': seed, 'weights': config.weights, 'n_ap': len(Ap_list),
               'n_levels': -1 if n_levels is None else n_levels, 'slim': True,
               'n_app': len(cap['app'])}
        sh = {}
        for l in range(L):
            out['A_%d' % l] = cap['A_pyr'][l]
            out['B_%d' % l] = cap['B_pyr'][l]
            for j, p in enumerate(cap['Ap_pyr']):
                out['Ap%d_%d' % (j, l)] = p[l]
            sh['A_%d' % l] = _sha1(cap['A_pyr'][l])
            sh['B_%d' % l] = _sha1(cap['B_pyr'][l])
            sh['Bp0_%d' % l] = _sha1(cap['Bp_init'][l])
            sh['Bp_%d' % l] = _sha1(cap['Bp_live'][l])
            for j, p in enumerate(cap['Ap_pyr']):
                sh['Ap%d_%d' % (j, l)] = _sha1(p[l])
        out['sha1_keys'] = np.array(sorted(sh))
        out['sha1_vals'] = np.array([sh[x] for x in sorted(sh)])
        for l, (s, im) in zip(range(1, L), cap['s'].values()):
            out['s_%d' % l] = np.array([np.asarray(p, dtype=np.int64) for p in s]).reshape(-1, 2).astype(np.int16)
            out['im_%d' % l] = np.array(im, dtype=np.uint8)
        np.savez_compressed(os.path.join(OUT, 'e2e_%s.npz' % name), **out)
        print('case %-10s L=%d levels, %d px synthesised (slim)' % (name, L, len(cap['app'])))
        return
    ity = np.int32 if lean else np.int64
    out = {'A': A, 'B': B, 'Ap': np.stack(Ap_list), 'L': L, 'convert': convert, 'remap': remap,
           'init_rand': init_rand, 'AB_weight': AB_weight, 'k': k, 'seed': seed,
           'weights': config.weights, 'app_ix': np.array(cap['app'], dtype=ity),
           'coh': np.array(cap['coh'], dtype=ity).reshape(-1, 3),
           'dist': np.array(cap['dist'], dtype=np.float64), 'lean': lean}
    for l in range(len(cap['A_pyr'])):
        out['A_%d' % l] = cap['A_pyr'][l]
    for j, p in enumerate(cap['Ap_pyr']):
        for l in range(len(p)):
            out['Ap%d_%d' % (j, l)] = p[l]
    for j, p in enumerate(cap['color_pyr']):
        if lean and not convert:
            break   # identical to the A' pyramid
        for l in range(len(p)):
            out['color%d_%d' % (j, l)] = p[l]
    for l in range(len(cap['B_pyr'])):
        out['B_%d' % l] = cap['B_pyr'][l]
        out['Bp0_%d' % l] = cap['Bp_init'][l]
        out['Bp_%d' % l] = cap['Bp_live'][l]
    # s / im per level in level order (dict preserves insertion order)
    for l, (s, im) in zip(range(1, L), cap['s'].values()):
        out['s_%d' % l] = np.array([np.asarray(p, dtype=np.int64) for p in s]).reshape(-1, 2).astype(ity)
        out['im_%d' % l] = np.array(im, dtype=ity)
    for f, x in colour.items():
        if f.startswith('level_') and (not lean or int(f.split('_')[1]) == L - 1):
            out['out_' + f.split('_')[1]] = x
    np.savez_compressed(os.path.join(OUT, 'e2e_%s.npz' % name), **out)
    print('case %-10s L=%d levels, %d px synthesised' % (name, L, len(cap['app'])))


def big_cases(mods, names):
    """Round-2 fixtures at the sizes the pruned scan and cfg1 need (VERDICT r1 'do this' 1):
    cfg1 = the shore-crop stand-in of BASELINE config 1 (117x180 RGB -> YIQ luminance, k = 0.5,
    seeds 1/2/3); g128 / g256 = the bench generator at 128^2 / 256^2; ties128 =
    piecewise-constant 128^2 (exact duplicate DB rows at a size where every level can prune);
    k25 = 96^2 with kappa 25 (cfg4's high-kappa coherence)."""
    todo = {
        'cfg1': lambda: run_case(mods, 'cfg1', smooth(117, 180, 2, 1, ch=3), [filt(smooth(117, 180, 2, 1, ch=3))],
                                 smooth(117, 180, 2, 2, ch=3), convert=True, k=0.5, seed=3, lean=True),
        'g128': lambda: run_case(mods, 'g128', smooth(128, 128, 2, 1), [filt(smooth(128, 128, 2, 1))],
                                 smooth(128, 128, 2, 2), seed=3, lean=True),
        'ties128': lambda: run_case(mods, 'ties128', blocky(128, 128, 16), [1 - blocky(128, 128, 16)],
                                    blocky(128, 128, 17), seed=5, lean=True),
        'k25': lambda: run_case(mods, 'k25', smooth(96, 96, 2, 18), [filt(smooth(96, 96, 2, 18))],
                                smooth(96, 96, 2, 19), k=25.0, seed=6, lean=True),
        'g256': lambda: run_case(mods, 'g256', smooth(256, 256, 2, 1), [filt(smooth(256, 256, 2, 1))],
                                 smooth(256, 256, 2, 2), seed=3, lean=True),
        # round 6: BASELINE config 2's shape, the size at which the product's
        # default path prunes (512^2 DB rows >= prune_min_rows): 512^2, the finest 5 pyramid
        # levels, slim fixture.  ~1.5-2.5 h of container CPU with GEN_GOLDEN_THREADS=6.
        'g512': lambda: run_case(mods, 'g512', smooth(512, 512, 2, 1), [filt(smooth(512, 512, 2, 1))],
                                 smooth(512, 512, 2, 2), seed=3, slim=True, n_levels=5),
        # check of the slim writer and the level cap against e2e_g64 (not committed)
        'g64slim': lambda: run_case(mods, 'g64slim', smooth(64, 64, 2, 1), [filt(smooth(64, 64, 2, 1))],
                                    smooth(64, 64, 2, 2), seed=3, slim=True, n_levels=4),
    }
    for n in names:
        todo[n]()


def main():
    _check_blas_order()
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp()
    want = sys.argv[1:] or ['base']
    try:
        mods = load_reference(tmp)
        config, img_preprocess, algorithms, ia = mods
        big_cases(mods, [n for n in want if n != 'base'])
        if 'base' not in want:
            return

        # G1 weights (config.py:68-79)
        np.savez(os.path.join(OUT, 'weights.npz'),
                 w1=config.compute_weights(3, 5, 12, 1), w3=config.compute_weights(3, 5, 12, 3))

        # G2 feature layout KATs (algorithms_test.py:10-115 inputs) + a random 3-level case
        g2 = {}
        for ch in (None, 3):
            sm = 0.5 * np.ones((4, 5) + ((ch,) if ch else ()))
            sm[0, 0] = 0
            lg = 0.3 * np.ones((7, 10) + ((ch,) if ch else ()))
            lg[0, 0] = 1
            config.num_ch, config.padding_sm, config.padding_lg, config.weights = config.setup_vars(lg)
            tag = 'c%d' % (ch or 1)
            g2[tag + '_full'] = algorithms.compute_feature_array([sm, lg], config, full_feat=True)[1]
            g2[tag + '_half'] = algorithms.compute_feature_array([sm, lg], config, full_feat=False)[1]
            pd = img_preprocess.pad_img_pair(sm, lg, config)
            g2[tag + '_px00_full'] = algorithms.extract_pixel_feature(pd, (0, 0), config, full_feat=True)
            g2[tag + '_px00_half'] = algorithms.extract_pixel_feature(pd, (0, 0), config, full_feat=False)
        rs = np.random.RandomState(7)
        for ch in (None, 3):
            shp = (lambda h, w: (h, w) + ((ch,) if ch else ()))
            pyr = [rs.rand(*shp(5, 6)), rs.rand(*shp(9, 11)), rs.rand(*shp(17, 22))]
            pyr2 = [rs.rand(*shp(5, 6)), rs.rand(*shp(9, 11)), rs.rand(*shp(17, 22))]
            config.num_ch, config.padding_sm, config.padding_lg, config.weights = config.setup_vars(pyr[-1])
            config.max_levels = 3
            tag = 'rand_c%d' % (ch or 1)
            for l, p in enumerate(pyr):
                g2['%s_A_%d' % (tag, l)] = p
                g2['%s_Ap_%d' % (tag, l)] = pyr2[l]
            fl, prm, As, As_size = algorithms.create_index(pyr, [pyr2], config)
            for l in (1, 2):
                g2['%s_As_%d' % (tag, l)] = As[l]
            # per-pixel query features (image_analogies.py:166-168) on level 2 with B=pyr, B'=pyr2
            Bf = algorithms.compute_feature_array(pyr, config, full_feat=True)
            pd = img_preprocess.pad_img_pair(pyr2[1], pyr2[2], config)
            qs = []
            h, w = pyr[2].shape[:2]
            for r in range(h):
                for c_ in range(w):
                    qs.append(np.hstack([Bf[2][r * w + c_],
                                         algorithms.extract_pixel_feature(pd, (r, c_), config, full_feat=False)]))
            g2['%s_Q_2' % tag] = np.array(qs)
            g2['%s_nn_2' % tag] = np.array([algorithms.best_approximate_match(fl[2], prm[2], q) for q in qs])
        np.savez_compressed(os.path.join(OUT, 'features.npz'), **g2)

        # G3 pyramids (img_preprocess.py:47-63 with skimage 0.18.3) + G4 colour / remap
        g3 = {}
        rs = np.random.RandomState(11)
        shapes = [(117, 180), (33, 47), (64, 64), (64, 64, 3), (25, 40), (9, 13, 3), (45, 77)]
        for i, shp in enumerate(shapes):
            img = rs.rand(*shp)
            pyr = img_preprocess.compute_gaussian_pyramid(img, 3)
            g3['img_%d' % i] = img
            g3['n_%d' % i] = len(pyr)
            for l, p in enumerate(pyr):
                g3['pyr_%d_%d' % (i, l)] = p
        np.savez_compressed(os.path.join(OUT, 'pyramids.npz'), **g3)

        rgb = np.random.RandomState(0xba5eba11).rand(25, 25, 3)
        A, Ap, B = rs.rand(25, 25), rs.rand(25, 25), rs.rand(30, 30)
        Ar, Apr = img_preprocess.remap_luminance(A, [Ap], B)
        np.savez(os.path.join(OUT, 'color.npz'), rgb=rgb, yiq=img_preprocess.convert_to_YIQ(rgb),
                 back=img_preprocess.convert_to_RGB(img_preprocess.convert_to_YIQ(rgb)),
                 A=A, Ap=Ap, B=B, A_remap=Ar, Ap_remap=Apr[0])

        # G5 / G7 end-to-end source maps (image_analogies.py:97-268)
        A32 = smooth(32, 32, 2, 1)
        run_case(mods, 'g32', A32, [filt(A32)], smooth(32, 32, 2, 2))
        A24 = smooth(24, 24, 1.5, 4)
        run_case(mods, 'g24k5', A24, [filt(A24)], smooth(24, 24, 1.5, 5), k=5.0, seed=9)
        Ar = smooth(37, 50, 2, 6)
        run_case(mods, 'rect', Ar, [filt(Ar)], smooth(29, 43, 2, 7), seed=4)
        A64 = smooth(64, 64, 2, 1)
        run_case(mods, 'g64', A64, [filt(A64)], smooth(64, 64, 2, 2))
        Ac = smooth(32, 32, 2, 8, ch=3)
        run_case(mods, 'yiq', Ac, [filt(Ac)], smooth(32, 32, 2, 9, ch=3), convert=True)
        run_case(mods, 'remap', Ac, [filt(Ac)], smooth(32, 32, 2, 9, ch=3) * 0.6, convert=True, remap=True)
        A3 = smooth(20, 24, 1.5, 10, ch=3)
        run_case(mods, 'rgb3', A3, [filt(A3)], smooth(20, 24, 1.5, 11, ch=3))
        A2 = smooth(24, 24, 2, 12)
        run_case(mods, 'multiap', A2, [filt(A2), 1 - A2], smooth(24, 24, 2, 13))
        run_case(mods, 'noinit', A2, [filt(A2)], smooth(24, 24, 2, 13), init_rand=False, AB_weight=0.5)
        Ab = blocky(32, 32, 14)
        run_case(mods, 'ties', Ab, [1 - Ab], blocky(32, 32, 15))
    finally:
        shutil.rmtree(tmp)
        sys.path.remove(tmp)


if __name__ == '__main__':
    main()
