#!/bin/bash
# kernarg placement: the chain gaps with HIP_FORCE_DEV_KERNARG=1 vs the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'window', round(r.get('chain_window_ms_timed',0),1))"; }
for i in 1 2; do
  for v in "def:0" "devka:1"; do
    n=${v%%:*}; k=${v#*:}
    if [ $k = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
    timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --pipeline 0 > $O/${n}_seq_$i.json 2> $O/${n}_seq_$i.err || { echo "bench $n seq failed"; tail -20 $O/${n}_seq_$i.err; exit 1; }
    summ $O/${n}_seq_$i.json ${n}_seq
  done
done
echo ALL-OK
