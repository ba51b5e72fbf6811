#!/bin/bash
# bench line with K3 timing events every 4th vs every 16th step, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/stride
for i in 1 2; do
  for s in 4 16; do
    timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --time-stride $s > gpurun_out/stride/s${s}_$i.json 2> gpurun_out/stride/s${s}_$i.err || { echo "bench $s failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/stride/s${s}_$i.json')); r=d['roofline']; print($s, round(d['value']), round(d['ms_per_step'],1), round(r['k3_us_per_launch'],2), r['k3_launches_sampled'])"
  done
done
echo ALL-OK
