#!/bin/bash
# row-interleaved strong-scaling emulation; tiles with filter-passing blocks; pruning coarser levels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 400 python -u tools/strong_model.py 3 1 2 4 8 > $O/strong_rows.jsonl 2> $O/strong_rows.err || { echo "strong model failed"; tail $O/strong_rows.err; exit 1; }
cat $O/strong_rows.jsonl
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'tiles_pass', round(r.get('tiles_passing_frac',0),3), 'pairs_corr', round(r.get('pairs_corrected_frac',0),3), 'fallbacks', d['stats']['fallbacks'])"; }
for v in "base:" "p512:--prune-min-rows 262144" "p256:--prune-min-rows 65536" "base2:" "p512b:--prune-min-rows 262144" "cfg4:--config cfg4"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline $a > $O/${n}.json 2> $O/${n}.err || { echo "bench $n failed"; tail -20 $O/${n}.err; exit 1; }
  summ $O/${n}.json $n
done
echo ALL-OK
