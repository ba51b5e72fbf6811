"""Host preprocessing cost: img_setup (image_analogies.py:17-94:
scale, YIQ split, remap, compress, three Gaussian pyramids, B' init) at the BASELINE sizes,
timed on this host's CPU (numpy, 1 thread), against the GPU synthesis time of the same job.
  python tools/host_setup_timing.py <out.json> [gpu_ms_per_job]"""
import json
import os
import sys
import time
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ia_amd  # noqa: E402,F401
from ia_amd import synth  # noqa: E402
from ia_amd.image_analogies import img_setup  # noqa: E402


def cfg(convert):
    from ia_amd import config
    c = types.SimpleNamespace(**{k: getattr(config, k) for k in dir(config) if not k.startswith('_')})
    c.convert, c.remap_lum, c.init_rand, c.AB_weight, c.k, c.seed, c.n_levels = convert, False, True, 1, 0.5, 3, None
    c.level_align = 'coarse'
    return c


out = {}
for name, (ah, bh, ch) in {'cfg3 1024^2 grey': (1024, 1024, 1), 'cfg3 1024^2 RGB (YIQ path)': (1024, 1024, 3),
                          'cfg4 B 2048^2 vs A 1024^2 grey': (1024, 2048, 1)}.items():
    A = synth.smooth(ah, ah, 2, 1, ch=None if ch == 1 else ch)
    Ap = synth.filt(A)
    B = synth.smooth(bh, bh, 2, 2, ch=None if ch == 1 else ch)
    c = cfg(ch == 3)
    if bh != ah:
        c.level_align = 'fine'
    t0 = time.perf_counter()
    img_setup(A, [Ap], B, '/tmp/host_setup_out/', c)
    out[name] = time.perf_counter() - t0
res = {'host_setup_s': out, 'cores': 1, 'cpu': 'this container (numpy single-threaded ops)',
       'what': 'img_setup: scaling, YIQ split (RGB case), compress_values, A/A\'/B Gaussian pyramids '
               '(skimage 0.18.3 restated), initialize_Bp'}
if len(sys.argv) > 2:
    g = float(sys.argv[2])
    res['gpu_ms_per_job_cfg3'] = g
    res['setup_share_cfg3'] = out['cfg3 1024^2 grey'] / (out['cfg3 1024^2 grey'] + g / 1e3)
json.dump(res, open(sys.argv[1], 'w'), indent=1)
print(json.dumps(res, indent=1))
