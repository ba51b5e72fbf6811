"""Host-side preprocessing (★H rows of SURVEY §8): colour conversion, luminance remapping,
Gaussian pyramids, B' initialisation, symmetric padding and the DB index codec — the semantics
of the reference's img_preprocess.py, restated in this package's own numpy/scipy code
(skimage is not a dependency: compute_gaussian_pyramid restates skimage 0.18.3's
pyramid_gaussian, see _pyramid_reduce)."""
import numpy as np
from scipy import ndimage as ndi

# RGB -> YIQ and back (img_preprocess.py:6-22, constants from the same source)
_RGB2YIQ = np.array([[0.299, 0.587, 0.114],
                     [0.596, -0.275, -0.321],
                     [0.212, -0.523, 0.311]])
_YIQ2RGB = np.array([[1., 0.956, 0.621],
                     [1., -0.272, -0.647],
                     [1., -1.105, 1.702]])


def convert_to_YIQ(img, ctx=None):
    """img_preprocess.py:6-13 (input must already be on the 0..1 scale).  ctx: a libia Context
    to run the matrix on the GPU (ia_color_matrix, bit-identical to numpy's einsum)."""
    if not 0 <= np.max(img) <= 1:
        raise ValueError('convert_to_YIQ expects an image scaled to [0, 1]')
    if ctx is not None:
        return ctx.color_matrix(img, _RGB2YIQ)
    return np.einsum('ij,klj->kli', _RGB2YIQ, img)


def convert_to_RGB(img, ctx=None):
    """img_preprocess.py:16-22 (ctx: on the GPU, as convert_to_YIQ)."""
    if ctx is not None:
        return ctx.color_matrix(img, _YIQ2RGB)
    return np.einsum('ij,klj->kli', _YIQ2RGB, img)


def remap_luminance(A, Ap_list, B):
    """Affine luminance remap of A and every A' to B's mean / std (img_preprocess.py:25-40);
    single channel only."""
    if not (A.ndim == Ap_list[0].ndim == B.ndim == 2):
        raise ValueError('remap_luminance works on single-channel (luminance) images')
    gain = np.std(B) / np.std(A)
    mA, mB = np.mean(A), np.mean(B)
    return gain * (A - mA) + mB, [gain * (Ap - mA) + mB for Ap in Ap_list]


def compress_values(A, B, ratio):
    """img_preprocess.py:43-44."""
    return ratio * A, ratio * B


def _bilinear_downsize(img, out_h, out_w):
    """skimage 0.18.3 resize(order=1, mode='reflect', anti_aliasing=False, clip=True): each output
    pixel samples the input at f*(o + 0.5) - 0.5 (f = in / out) with bilinear weights, then the
    result is clipped to the input's range.  Sample coordinates never leave the image for f >= 1."""
    h, w = img.shape[:2]
    rr = (h / float(out_h)) * (np.arange(out_h) + 0.5) - 0.5
    cc = (w / float(out_w)) * (np.arange(out_w) + 0.5) - 0.5
    r0, c0 = np.floor(rr).astype(int), np.floor(cc).astype(int)
    r1, c1 = np.ceil(rr).astype(int), np.ceil(cc).astype(int)
    dr, dc = rr - r0, cc - c0
    if img.ndim == 3:
        dr, dc = dr[:, None, None], dc[None, :, None]
    else:
        dr, dc = dr[:, None], dc[None, :]
    tl, tr = img[r0][:, c0], img[r0][:, c1]
    bl, br = img[r1][:, c0], img[r1][:, c1]
    top = (1 - dc) * tl + dc * tr
    bottom = (1 - dc) * bl + dc * br
    return np.clip((1 - dr) * top + dr * bottom, img.min(), img.max())


def _pyramid_reduce(img):
    """One skimage pyramid_reduce step (downscale 2): Gaussian smoothing with sigma = 2*2/6
    (mode 'reflect' = half-sample symmetric, truncate 4 -> 7 taps; the channel axis is not
    smoothed) followed by the bilinear resize to ceil(h/2) x ceil(w/2)."""
    sigma = 2 * 2 / 6.0
    sig = (sigma, sigma, 0) if img.ndim == 3 else sigma
    smooth = ndi.gaussian_filter(img, sig, mode='reflect')
    return _bilinear_downsize(smooth, -(-img.shape[0] // 2), -(-img.shape[1] // 2))


def gaussian_weights():
    """scipy.ndimage.gaussian_filter's 7-tap kernel for sigma = 2/3, truncate 4 (its
    _gaussian_kernel1d restated: exp(-0.5 / sigma^2 x^2) normalised by its sum)."""
    sigma = 2 * 2 / 6.0
    radius = int(4.0 * sigma + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x ** 2)
    return phi / phi.sum()


def compute_gaussian_pyramid(img, min_size, n_levels=None, ctx=None):
    """Coarsest-first Gaussian pyramid (img_preprocess.py:47-63).  The number of reductions is
    the number of halvings until min(h, w) <= min_size; (h, w, 3) images are reduced per channel
    (SURVEY §7 hard part 6).  n_levels (extension) caps the pyramid at that many images.
    ctx: a libia Context to run the reductions on the GPU (ia_gaussian_pyramid: the same
    arithmetic, operation for operation, so the levels are bit-identical)."""
    img = np.asarray(img, dtype=np.float64)
    side = min(img.shape[:2])
    reductions = 0
    while side > min_size:
        side = side // 2
        reductions += 1
    if n_levels is not None:
        reductions = min(reductions, int(n_levels) - 1)
    pyr = [img]
    if ctx is not None:
        # a reduction that leaves the shape unchanged (1-pixel sides) ends the host loop below;
        # ceil-halving changes the shape unless both sides are 1
        n = 0
        h, w = img.shape[:2]
        while n < reductions and (h, w) != (1, 1):
            h, w = (h + 1) // 2, (w + 1) // 2
            n += 1
        pyr += ctx.gaussian_pyramid(img, n, gaussian_weights())
        reductions = 0
    for _ in range(reductions):
        nxt = _pyramid_reduce(pyr[-1])
        if nxt.shape == pyr[-1].shape:
            break
        pyr.append(nxt)
    pyr = pyr[::-1]
    if len(pyr) > 1:
        assert min(pyr[1].shape[:2]) > min_size or n_levels is not None
    return pyr


def initialize_Bp(B_pyr, init_rand=True, seed=None):
    """Initial B' pyramid (img_preprocess.py:66-78): per level in coarse-to-fine order either
    uniform random values drawn from the legacy MT19937 stream (np.random.rand order, so a
    seeded run reproduces the reference draw for draw), or a copy of B's pyramid."""
    rng = np.random if seed is None else np.random.RandomState(seed)
    out = []
    for lvl in B_pyr:
        if init_rand:
            out.append(rng.rand(int(np.prod(lvl.shape))).reshape(lvl.shape))
        else:
            out.append(lvl.copy())
    return out


def pad_img_pair(img_sm, img_lg, c):
    """Symmetric (edge-duplicating) padding of a coarse/fine pair (img_preprocess.py:81-83)."""
    return [np.pad(img_sm, c.padding_sm, mode='symmetric'), np.pad(img_lg, c.padding_lg, mode='symmetric')]


# DB row-id codec (img_preprocess.py:85-106): row = (img * h + r) * w + c
def px2ix(pxs, w):
    return (np.asarray(pxs[0]) * w + np.asarray(pxs[1])).astype(int)


def ix2px(ixs, w):
    ixs = np.asarray(ixs)
    return np.array([ixs // w, ixs % w])


def Ap_ix2px(ixs, h, w):
    ixs = np.asarray(ixs)
    img_nums = ixs // (h * w)
    return ix2px(ixs - img_nums * h * w, w), img_nums


def Ap_px2ix(pxs, img_nums, h, w):
    return (((h * np.asarray(img_nums)) + np.asarray(pxs[0])) * w + np.asarray(pxs[1])).astype(int)


def savefig_noborder(fileName, fig):
    """img_preprocess.py:109-113: save the current matplotlib image without axes or border."""
    import matplotlib.pyplot as plt
    plt.axis('off')
    fig.axes.get_xaxis().set_visible(False)
    fig.axes.get_yaxis().set_visible(False)
    plt.savefig(fileName, bbox_inches='tight', pad_inches=0)
