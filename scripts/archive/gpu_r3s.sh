#!/bin/bash
# round 3, session S: level pipelining variants on one box (contexts 2 / 3, finest-level stream
# priority), two alternating passes of each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s
for pass in 1 2; do
  for v in "2 0" "3 0" "2 1" "3 1"; do
    set -- $v
    f=gpurun_out/s/c$1_p$2_$pass
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipe-ctx $1 --pipe-priority $2 > $f.json 2> $f.err || { echo "bench $v failed"; tail -20 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1), d['config']['level_pipeline'])"
  done
done
echo R3S-OK
