"""Time the split-f16 distance scan (K3h) alone for every k3_variant: cfg3 plateau shape
(1,048,576 DB rows x 342 queries) plus smaller shapes.  Prints one JSON line per measurement.
  python3 tools/k3_micro.py [variants...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ia_amd  # noqa: F401,E402
from ia_amd import _native  # noqa: E402

variants = [int(v) for v in sys.argv[1:]] or [0, 1]
ctx = _native.Context(0)
for n_rows, M in [(1048576, 342), (1048576, 171), (262144, 171), (65536, 86)]:
    for v in variants:
        ctx.set_option('k3_variant', v)
        us = ctx.k3_microbench(n_rows, M, 30)
        tf = 2.0 * 55 * n_rows * M / (us * 1e-6) / 1e12
        print(json.dumps({'variant': v, 'n_rows': n_rows, 'M': M, 'us': round(us, 2), 'alg_TFLOPs': round(tf, 1)}),
              flush=True)
ctx.close()
