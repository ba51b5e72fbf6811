"""Parameters — same names and defaults as the reference's config.py (config.py:7-26), used the
same way: as a mutable module namespace (`import ... config as c; c.k = 5`, multi_script.py:5,31).

Differences, all deliberate:
  * n_half / pad_sm / pad_lg are ints (the reference makes them np.float64, config.py:18-20,
    which modern numpy refuses as slice bounds — SURVEY A6).
  * new knobs (defaults reproduce the reference): n_levels, level_align, seed, device.
"""
import numpy as np

# Set Parameters and Variables (config.py:7-16)
convert = False    # Convert to YIQ (also use color from B if true or Ap if false)
remap_lum = False  # remap luminance of A/Ap to B
init_rand = True   # initialize Bp as random

AB_weight = 1      # relative weighting of A and B relative to Ap and Bp
k = 0.5            # 0.5 <= k <= 5 for texture synthesis
n_sm = 3           # coarse scale neighborhood size
n_lg = 5           # fine scale neighborhood size

n_half = (n_lg * n_lg) // 2   # fine scale half neighborhood size (config.py:18, as int)
pad_sm = n_sm // 2            # config.py:19
pad_lg = n_lg // 2            # config.py:20

# runtime slots filled by setup_vars / img_setup (config.py:22-26)
num_ch = None
max_levels = None
padding_sm = None
padding_lg = None
weights = None

# --- additions (not in the reference) ----------------------------------------------------
n_levels = None      # pyramid depth override (BASELINE cfg2: 5 levels); None = reference rule
level_align = 'coarse'  # 'coarse' = reference (image_analogies.py:82-86), 'fine' = B level k+1 <-> A level k
seed = None          # np.random seed for initialize_Bp (reference: unseeded global RNG)
device = None        # HIP device ordinal (None: LOCAL_RANK or 0)
gpu_preprocess = True  # Gaussian pyramids + YIQ matrices on the GPU (bit-identical to the host code)


def setup_vars(img):
    """Derive the per-image slots (config.py:29-42): channel count, np.pad widths for the
    coarse / fine windows, and the compute_distance weight vector."""
    if img.ndim not in (2, 3):
        raise ValueError('image must be (h, w) or (h, w, ch)')
    ch = img.shape[2] if img.ndim == 3 else 1
    if ch == 1:
        pads = (int(pad_sm), int(pad_lg))
    else:
        pads = tuple(((p, p), (p, p), (0, 0)) for p in (int(pad_sm), int(pad_lg)))
    return ch, pads[0], pads[1], compute_weights(n_sm, n_lg, n_half, ch)


def save_metadata(out_path, names, vars):
    """Write `name: value` lines to <out_path>metadata.txt (config.py:45-49)."""
    lines = ['%s: %s\n' % (n, v) for n, v in zip(names, vars)]
    with open(out_path + 'metadata.txt', 'w') as fh:
        fh.writelines(lines)


def matlab_style_gauss2D(shape=(3, 3), sigma=0.5):
    """MATLAB fspecial('gaussian', shape, sigma) (config.py:52-65): unnormalised Gaussian on a
    centred integer grid, entries below eps*max zeroed, then normalised to sum 1."""
    rows, cols = shape
    yy = np.arange(rows, dtype=np.float64)[:, None] - (rows - 1) / 2.
    xx = np.arange(cols, dtype=np.float64)[None, :] - (cols - 1) / 2.
    g = np.exp(-(xx * xx + yy * yy) / (2. * sigma * sigma))
    g[g < np.finfo(np.float64).eps * g.max()] = 0
    total = g.sum()
    return g / total if total != 0 else g


def compute_weights(n_sm, n_lg, n_half, num_ch):
    """Weight vector of compute_distance (config.py:68-79), laid out like a DB row
    (SURVEY Appendix A): [G3(.5)/9 | G5(1)/25 | G3(.5)/9 | G5(1)[:n_half]/n_half], every
    spatial weight repeated num_ch times (channel-minor)."""
    g_sm = np.repeat(matlab_style_gauss2D((n_sm, n_sm), 0.5).ravel(), num_ch)
    g_lg = np.repeat(matlab_style_gauss2D((n_lg, n_lg), 1).ravel(), num_ch)
    coarse = g_sm * (1. / (n_sm * n_sm))
    fine = g_lg * (1. / (n_lg * n_lg))
    causal = g_lg[:int(n_half) * num_ch] * (1. / n_half)
    return np.concatenate([coarse, fine, coarse, causal])
