#!/bin/bash
# cfg5 A/B of bench flags (two passes): ab_cfg5.sh OUT "name|flags" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for pass in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r n flags <<< "$spec"
    timeout -k 10 300 python -u bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline $flags > $O/${n}_$pass.json 2> $O/${n}_$pass.err || { echo "bench $n failed"; tail -20 $O/${n}_$pass.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${n}_$pass.json'))
print('%-8s' % '$n', $pass, round(d['value']/1e6,3), 'M px/s parity', d.get('parity'), round(d['ms_per_step'],1), 'ms')"
  done
done
echo ALL-OK
