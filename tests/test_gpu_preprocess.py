"""GPU preprocessing: ia_gaussian_pyramid and ia_color_matrix must reproduce the
host restatement (ia_amd.img_preprocess: numpy + scipy.ndimage) bit for bit, and through it the
reference's skimage 0.18.3 pyramids (golden pyramids.npz, tolerance 1e-12 as the host test) and
YIQ vectors (golden color.npz, bit-exact); img_setup / image_analogies_main give identical
results with config.gpu_preprocess on and off."""
import os
import types

import numpy as np
import pytest

from golden_util import GOLDEN, load_e2e

pytestmark = pytest.mark.gpu


def test_gpu_pyramid_matches_host_and_skimage(ctx):
    import ia_amd  # noqa: F401
    from ia_amd import img_preprocess as ip
    g = np.load(os.path.join(GOLDEN, 'pyramids.npz'))
    i = 0
    while 'img_%d' % i in g:
        img = g['img_%d' % i]
        host = ip.compute_gaussian_pyramid(img, 3)
        gpu = ip.compute_gaussian_pyramid(img, 3, ctx=ctx)
        assert len(gpu) == len(host) == int(g['n_%d' % i])
        for l, (a, b) in enumerate(zip(gpu, host)):
            assert a.shape == b.shape and np.array_equal(a, b), (i, l)
            assert np.abs(a - g['pyr_%d_%d' % (i, l)]).max() < 1e-12
        i += 1
    rs = np.random.RandomState(5)
    for shp in [(1024, 1024), (117, 180, 3), (2, 7), (5, 1), (1, 1)]:
        img = rs.rand(*shp)
        for n in (None, 3):
            host = ip.compute_gaussian_pyramid(img, 3, n)
            gpu = ip.compute_gaussian_pyramid(img, 3, n, ctx=ctx)
            assert len(gpu) == len(host) and all(np.array_equal(a, b) for a, b in zip(gpu, host)), shp


def test_gpu_color_matrix_matches_reference(ctx):
    import ia_amd  # noqa: F401
    from ia_amd import img_preprocess as ip
    g = np.load(os.path.join(GOLDEN, 'color.npz'))
    assert np.array_equal(ip.convert_to_YIQ(g['rgb'], ctx), g['yiq'])
    assert np.array_equal(ip.convert_to_RGB(ip.convert_to_YIQ(g['rgb'], ctx), ctx), g['back'])
    x = np.random.RandomState(1).rand(300, 200, 3)
    assert np.array_equal(ip.convert_to_YIQ(x, ctx), ip.convert_to_YIQ(x))
    assert np.array_equal(ip.convert_to_RGB(x, ctx), ip.convert_to_RGB(x))


@pytest.mark.parametrize('name', ['yiq', 'remap', 'noinit', 'rgb3'])
def test_img_setup_gpu_equals_host(tmp_path, name):
    """img_setup on the golden inputs: every pyramid level and B' init identical with
    gpu_preprocess on and off, and equal to the reference's own pyramids within 1e-12."""
    from ia_amd import config
    from ia_amd.image_analogies import img_setup
    z = load_e2e(name)
    outs = []
    for gpu in (False, True):
        c = types.SimpleNamespace(**{k: getattr(config, k) for k in dir(config) if not k.startswith('_')})
        c.convert, c.remap_lum, c.init_rand = bool(z['convert']), bool(z['remap']), bool(z['init_rand'])
        c.AB_weight, c.k, c.seed, c.gpu_preprocess = float(z['AB_weight']), float(z['k']), int(z['seed']), gpu
        outs.append(img_setup(z['A'], list(z['Ap']), z['B'], str(tmp_path) + '/%d/' % gpu, c))
    for a, b in zip(outs[0][:4], outs[1][:4]):
        flat_a = [x for p in (a if isinstance(a[0], list) else [a]) for x in p]
        flat_b = [x for p in (b if isinstance(b[0], list) else [b]) for x in p]
        assert all(np.array_equal(x, y) for x, y in zip(flat_a, flat_b))
    for l, x in enumerate(outs[1][0]):
        assert np.abs(x - z['A_pyr'][l]).max() < 1e-12
