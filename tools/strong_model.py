"""strong-scaling bound of ONE cfg3 job (1024^2 A/A'/B) over W GPUs, from one-GPU
emulation with the current kernels and kernel-written launch stamps (include/ia.h option
"stamps").  The 1024^2 level is a chain of 4,093 dependent wavefront steps; a decomposition can
only shorten each step.

(b) row-interleaved query split: B row r on GPU r mod W, the DB replicated.  Per step a GPU
    gathers, scans (the whole DB) and merges the ~342 / W queries of its rows; the fused
    merge + gather's row-to-row handoff (ia_kernels.hip k_merge_gather) then crosses GPUs on
    every row.  Emulated by a B of width 1024 / W against the 1024^2 A (level_align 'fine': B's
    finest level pairs with A's): its plateau steps hold 342 / W queries over the same DB, so its
    per-step K3p and merge + gather device times are one GPU's share of a W-way split.
        step(W) = K3p(342 / W) + merge_gather(342 / W) + x_handoff
(a) DB-shard winner exchange (exchange 1, every rank holds the job): per step K2p + the scan of
    1/W of the DB for all 342 queries + the merge + an exchange; from a rocprofv3 trace of
    bench.py --shard-emulate W --shard-jobs 1 --exchange peer (tools/shard_model.py), not here.

Prints one JSON line per W: per-step device times, the modelled 1024^2-level time
(4,093 steps) and the modelled job time against the measured one-GPU step.
  python3 tools/strong_model.py [x_handoff_us] [W ...]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ia_amd  # noqa: F401,E402
from ia_amd import _native, synth  # noqa: E402


def finest_step_times(ctx, job):
    """synthesise the job level by level (device-resident inputs via host buffers are fine: the
    stamps time kernels only); per-launch means of the pruned level's K3p and fused merges"""
    Bp = [x.copy() for x in job.Bp_init]
    st = _native.Stats()
    ctx.set_option('stamps', 1)
    t0 = time.time()
    for level in range(1, job.L):
        ctx.synthesize_level(job.A_pyr[level], job.A_pyr[level - 1], [p[level] for p in job.Ap_pyr_list],
                             [p[level - 1] for p in job.Ap_pyr_list], job.B_pyr[level], job.B_pyr[level - 1],
                             Bp[level - 1], Bp[level], job.weights, job.kappa_factor(level), st)
    ctx.set_option('stamps', 0)
    d = st.as_dict()
    return {'k3p_us': d['k3p_stamp_ms'] * 1e3 / max(d['k3p_stamp_launches'], 1),
            'merge_us': d['merge_stamp_ms'] * 1e3 / max(d['merge_stamp_launches'], 1),
            'steps': d['k3p_stamp_launches'], 'fallbacks': d['fallbacks'], 'wall_s': time.time() - t0}


def main():
    x = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    Ws = [int(a) for a in sys.argv[2:]] or [1, 2, 4, 8]
    ctx = _native.Context(0)
    base = None
    for W in Ws:
        bw = 1024 // W
        job = synth.make_job(size=1024, b_size=(1024, bw), level_align='fine')
        finest_step_times(ctx, job)   # warm-up (DB build paths, allocations)
        r = finest_step_times(ctx, job)
        step = r['k3p_us'] + r['merge_us'] + (x if W > 1 else 0.0)
        level_ms = 4093 * step / 1e3
        if W == 1:
            base = level_ms
        r.update({'W': W, 'b_shape': [1024, bw], 'queries_per_step': min(1024, (bw + 2) // 3), 'x_handoff_us': x,
                  'step_us': step, 'level_1024_ms_model': level_ms,
                  'speedup_vs_W1': (base / level_ms) if base else None,
                  'efficiency': (base / level_ms / W) if base else None})
        print(json.dumps(r), flush=True)
    ctx.close()


if __name__ == '__main__':
    main()
