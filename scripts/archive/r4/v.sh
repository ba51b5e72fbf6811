#!/bin/bash
# with the round-4 defaults: cfg5 streams / batch size, cfg3 / cfg4 pipeline contexts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4v; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms')"; }
for i in 1 2; do
  for v in "c5:--config cfg5 --steps 2" "c5s4:--config cfg5 --steps 2 --streams 4" "c5s2:--config cfg5 --steps 2 --streams 2" "c5b8:--config cfg5 --steps 2 --max-batch 8" "c3:--steps 10" "c3ctx3:--steps 10 --pipe-ctx 3" "c3ctx5:--steps 10 --pipe-ctx 5" "c4ctx3:--config cfg4 --steps 3 --pipe-ctx 3" "c4:--config cfg4 --steps 3"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
