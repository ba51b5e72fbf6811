#!/bin/bash
# round 3, session AG: stream priority of the pipelined levels: finest high (1), none (0), reversed (2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ag
for pass in 1 2; do
  for pp in 1 0 2; do
    f=gpurun_out/ag/p${pp}_$pass
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipe-priority $pp > $f.json 2> $f.err || { echo "bench $pp failed"; tail -20 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
  done
done
echo R3AG-OK
