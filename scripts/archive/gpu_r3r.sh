#!/bin/bash
# round 3, session R: the bench defaults (pipelined levels) at N = 1, and the N = 2 owner path with
# pipelined levels on one GPU (ranks on CU halves) + the agreed fallback
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 15 > gpurun_out/r/bench.json 2> gpurun_out/r/bench.err || { echo "bench failed"; tail -20 gpurun_out/r/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('cfg3', round(d['value']), round(d['ms_per_step'],1), round(r['frac'],3), r['k3_us_per_launch'], d['config']['level_pipeline'], round(d['cpu_baseline']['value'],2))"
bash scripts/gpu_r3l.sh || exit 1
echo R3R-OK
