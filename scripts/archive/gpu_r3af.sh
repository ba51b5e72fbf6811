#!/bin/bash
# round 3, session AF: hardware queues per process (GPU_MAX_HW_QUEUES 4 = the box default vs 8)
# x pipelined contexts (4, 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/af
for pass in 1 2; do
  for v in "4 4" "8 4" "8 5"; do
    set -- $v
    f=gpurun_out/af/q$1_c$2_$pass
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipe-ctx $2 > $f.json 2> $f.err || { echo "bench $v failed"; tail -20 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
  done
done
echo R3AF-OK
