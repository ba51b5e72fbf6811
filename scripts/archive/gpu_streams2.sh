#!/bin/bash
# cfg5: 3 vs 4 vs 6 libia contexts on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/streams2
for i in 1 2; do
  for s in 3 4 6; do
    timeout -k 10 300 python -u bench.py --config cfg5 --streams $s --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/streams2/s${s}_$i.json 2> gpurun_out/streams2/s${s}_$i.err || { echo "bench $s failed"; tail -5 gpurun_out/streams2/s${s}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/streams2/s${s}_$i.json')); print($s, round(d['value']), round(d['ms_per_step'],1))"
  done
done
echo ALL-OK
