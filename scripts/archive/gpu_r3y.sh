#!/bin/bash
# round 3, session Y: pruning the 512^2 level too (its steps then run the fused merge + gather) in
# the pipelined job: A/B against the default, two passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/y
for pass in 1 2; do
  for pm in 524288 262144; do
    f=gpurun_out/y/pm${pm}_$pass
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --prune-min-rows $pm > $f.json 2> $f.err || { echo "bench $pm failed"; tail -20 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
  done
done
echo R3Y-OK
