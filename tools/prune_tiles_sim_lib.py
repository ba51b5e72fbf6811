"""helpers shared by prune_tiles_sim.py and hh_filter_sim.py"""
import numpy as np


def morton(cols, bits):
    """interleave the bits of k quantised columns (each in [0, 2^bits))"""
    key = np.zeros(len(cols[0]), dtype=np.uint64)
    for b in range(bits - 1, -1, -1):
        for c in cols:
            key = (key << np.uint64(1)) | ((c >> np.uint64(b)) & np.uint64(1))
    return key


def quant(p, lo, hi, bits):
    return np.clip(((p - lo) / (hi - lo) * (2 ** bits - 1)).astype(np.int64), 0, 2 ** bits - 1).astype(np.uint64)
