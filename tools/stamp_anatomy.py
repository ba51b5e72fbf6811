"""Anatomy of the pruned level's launches from raw kernel stamps (IA_STAMP_DUMP=<file>, written by
libia for every stamped level with the largest pruned DB: bench.py with --steps 1 gives two records,
the timed pipelined job and the single-stream roofline pass).

Per K3p launch: workgroup start spread, mean / max workgroup duration, the tail (last end - the
slowest... ), per merge launch: wave start spread, median / p90 / max wave duration, the index of
the last-ending wave and its own duration.  Times in us (100 MHz ticks)."""
import sys

import numpy as np


def records(path):
    raw = np.fromfile(path, dtype=np.uint64)
    i = 0
    while i < len(raw):
        k3n, nwg, mgn, mgs = (int(x) for x in raw[i:i + 4])
        i += 4
        k3 = raw[i:i + k3n * nwg * 2].reshape(k3n, nwg, 2)
        i += k3n * nwg * 2
        mg = raw[i:i + mgn * mgs * 2].reshape(mgn, mgs, 2)
        i += mgn * mgs * 2
        yield k3, mg


def launch_stats(x):
    """x: (launches, slots, 2) raw stamps; returns per-launch dicts (us)"""
    out = []
    for L in x:
        ok = L[:, 0] != 0
        if not ok.any():
            continue
        st = (L[ok, 0] & ~np.uint64(1)).astype(np.int64)
        en = L[ok, 1].astype(np.int64)
        idx = np.nonzero(ok)[0]
        d = (en - st) * 1e-2
        t0 = st.min()
        last = int(np.argmax(en))
        out.append(dict(span=(en.max() - t0) * 1e-2, spread=(st.max() - t0) * 1e-2, mean=d.mean(), med=np.median(d),
                        p90=np.percentile(d, 90), mx=d.max(), last_idx=int(idx[last]), last_dur=d[last],
                        last_start=(st[last] - t0) * 1e-2, n=int(ok.sum()),
                        late=(st - t0 > 2.0).mean()))  # share of waves starting > 2 us after the first
    return out


def summary(name, ls):
    if not ls:
        return
    keys = ['span', 'spread', 'mean', 'med', 'p90', 'mx', 'last_dur', 'last_start', 'late']
    a = {k: np.array([x[k] for x in ls]) for k in keys}
    print('%s: %d launches, %.0f slots each' % (name, len(ls), np.mean([x['n'] for x in ls])))
    for k in keys:
        print('  %-10s mean %7.2f  p50 %7.2f  p90 %7.2f  p99 %7.2f' % (k, a[k].mean(), np.percentile(a[k], 50),
                                                                    np.percentile(a[k], 90), np.percentile(a[k], 99)))
    li = np.array([x['last_idx'] for x in ls])
    n = np.array([x['n'] for x in ls])
    print('  last-ending wave index / slots: mean %.2f; in the last 5%%: %.2f; in the first 5%%: %.2f'
          % ((li / n).mean(), (li >= 0.95 * n).mean(), (li < 0.05 * n).mean()))


if __name__ == '__main__':
    for j, (k3, mg) in enumerate(records(sys.argv[1])):
        print('=== record %d' % j)
        summary('K3p', launch_stats(k3))
        summary('merge+gather', launch_stats(mg))
