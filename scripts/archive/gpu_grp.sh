#!/bin/bash
# prune_group: parity, then a same-box A/B of the cfg3 bench line over G = 1, 2, 4, 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/grp
timeout -k 10 300 python -u -m pytest tests/test_gpu_prune.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "groups or rejects" > gpurun_out/grp/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/grp/pytest.log; exit 1; }
tail -1 gpurun_out/grp/pytest.log; grep "^group\|group [0-9]:" gpurun_out/grp/pytest.log
for i in 1 2; do
  for g in 1 2 4 8; do
    timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --prune-group $g > gpurun_out/grp/g${g}_$i.json 2> gpurun_out/grp/g${g}_$i.err || { echo "bench $g failed"; tail -3 gpurun_out/grp/g${g}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/grp/g${g}_$i.json')); r=d['roofline']; print($g, round(d['value']), round(d['ms_per_step'],1), round(r['k3_us_per_launch'],1), d['stats']['fallbacks'], round(r['pairs_frac'],3))"
  done
done
echo ALL-OK
