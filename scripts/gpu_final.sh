#!/bin/bash
# Round evidence at HEAD: the round script (suite, smoke, PMC of K3p, bench + CPU baseline,
# rocprofv3 stats + breakdown), then the cfg4 and cfg5 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_round.sh || exit 1
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { echo "cfg4 failed"; tail -5 gpurun_out/bench_cfg4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { echo "cfg5 failed"; tail -5 gpurun_out/bench_cfg5.err; exit 1; }
for c in cfg4 cfg5; do python3 -c "import json; d=json.load(open('gpurun_out/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],1))"; done
echo FINAL-OK
